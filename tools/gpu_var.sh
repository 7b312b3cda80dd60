#!/bin/bash
# A/B of compile-time variants on one config: tools/gpu_var.sh <config> <steps> name...
set -e
cfg=$1; steps=$2; shift 2
out=gpurun_out/var; mkdir -p $out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  for rep in 1 2; do
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu --steps $steps --warmup 3 > $out/${cfg}_${v}_$rep.json 2> $out/${cfg}_${v}_$rep.err
  done
done
