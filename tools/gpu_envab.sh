#!/bin/bash
# A/B of environment settings on one config: tools/gpu_envab.sh <config> <steps> "<ENV=..>" ...
set -e
cfg=$1; steps=$2; shift 2
out=gpurun_out/envab; mkdir -p $out
i=0
for rep in 1 2; do
  i=0
  for e in "" "$@"; do
    i=$((i+1))
    env $e timeout -k 10 300 python bench.py --config $cfg --no-cpu --steps $steps --warmup 2 > $out/${cfg}_${i}_$rep.json 2> $out/${cfg}_${i}_$rep.err
  done
done
