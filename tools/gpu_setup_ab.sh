#!/bin/bash
# Setup-phase timings (PLSSVM_MI_TIMING=1) of the sparse rbf configs under setup variants (env assignments).
# usage (GPU box, repo root): bash tools/gpu_setup_ab.sh "<configs>" "<VAR=val ...>" ["<VAR=val ...>" ...]
set -u
configs=$1; shift
mkdir -p gpurun_out/setup_ab
for c in $configs; do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    env $v PLSSVM_MI_TIMING=1 timeout -k 10 200 python bench.py --config "$c" --steps 5 --warmup 1 --no-cpu --kp-reps 2 --solve \
      > gpurun_out/setup_ab/${c}_$i.json 2> gpurun_out/setup_ab/${c}_$i.err || exit $?
    echo "== $c [$v]"; grep -E "plssvm_mi\]|learn at" gpurun_out/setup_ab/${c}_$i.err | grep -v "^\s*$"
  done
done
