#!/bin/bash
# dense RBF epilogue ablations (timing only): base, variants/abl{1,2,3}.so, and the linear kernel on the same data
set -e
out=gpurun_out/dabl; mkdir -p $out
for v in base abl1 abl2 abl3; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config dense_rbf_100k --no-cpu --no-extra --steps 10 --warmup 2 > $out/$v.json 2> $out/$v.err
done
timeout -k 10 200 python bench.py --config dense_rbf_100k --kernel linear --no-cpu --no-extra --steps 10 --warmup 2 > $out/linear.json 2> $out/linear.err
timeout -k 10 200 python bench.py --config dense_rbf_100k --kernel polynomial --no-cpu --no-extra --steps 10 --warmup 2 > $out/poly.json 2> $out/poly.err
