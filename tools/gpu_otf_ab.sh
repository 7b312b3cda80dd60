#!/bin/bash
# A/B of library variants on the on-the-fly 1 % density K·p (tools/density_1pct.py), same box.
# usage (GPU box, repo root): bash tools/gpu_otf_ab.sh <variant>...   ("base" = the in-tree build)
set -u
mkdir -p gpurun_out/ab
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  PLSSVM_MI_LIB=$lib timeout -k 10 300 python tools/density_1pct.py --algo onthefly --reps 3 > gpurun_out/ab/otf_$v.json 2> gpurun_out/ab/otf_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/ab/otf_$v.json')); print('otf $v', d['kp_s'], d['max_rel_err'], d['ok'])"
done
