#!/bin/bash
# expansion remainder-stream variants: parity (default build) + config 3-RBF / 5 timing per variant
set -e
out=gpurun_out/exp; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_overlap.py > $out/pytest.log 2>&1
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  PLSSVM_MI_LIB=$lib timeout -k 10 300 python bench.py --config csr_rbf_1m --no-cpu --steps 50 --warmup 2 > $out/rbf_$v.json 2> $out/rbf_$v.err
  PLSSVM_MI_LIB=$lib timeout -k 10 300 python bench.py --config fp22_rbf_2m --no-cpu --steps 30 --warmup 2 > $out/fp22_$v.json 2> $out/fp22_$v.err
done
