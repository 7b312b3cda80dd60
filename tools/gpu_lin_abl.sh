#!/bin/bash
# sparse-linear pass timings (kernel trace) for the default build and a variant: tools/gpu_lin_abl.sh name...
set -e
export TMPDIR=/tmp
root=$(pwd)
out=$root/gpurun_out/labl; mkdir -p $out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=$root/variants/$v.so
  cd /tmp
  PLSSVM_MI_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr_$v -o run -- python3 $root/bench.py --config csr_linear_1m --no-cpu --steps 50 --warmup 3 > $out/$v.json 2> $out/$v.err
  cd $root
done
