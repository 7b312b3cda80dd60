#!/bin/bash
# dense RBF exp variants: parity of the default build, then timing of default / 256-table / degree 6
set -e
out=gpurun_out/dexp; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py > $out/pytest.log 2>&1
for v in base t256 deg6 base; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config dense_rbf_100k --no-cpu --no-extra --steps 10 --warmup 2 > $out/$v.json 2> $out/$v.err
done
