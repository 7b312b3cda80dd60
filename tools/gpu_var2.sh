#!/bin/bash
# A/B of a variant on configs 3 and 3-RBF (parity of the variant through test_gpu_sparse first)
set -e
v=$1
out=gpurun_out/var2; mkdir -p $out
PLSSVM_MI_LIB=variants/$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_sparse.py -k "not geometries" > $out/pytest_$v.log 2>&1
for rep in 1 2; do
for w in base $v; do
  lib=""; [ "$w" != base ] && lib=variants/$w.so
  PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config csr_linear_1m --no-cpu --steps 300 --warmup 3 > $out/lin_${w}_$rep.json 2> $out/lin_${w}_$rep.err
  PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config csr_rbf_1m --no-cpu --steps 50 --warmup 2 > $out/rbf_${w}_$rep.json 2> $out/rbf_${w}_$rep.err
done
done
