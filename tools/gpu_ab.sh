#!/bin/bash
# A/B of library variants (variants/<name>.so; "base" = the in-tree build) on bench configurations, same box.
# usage (GPU box, repo root): bash tools/gpu_ab.sh "<configs>" <variant>...  -> gpurun_out/ab/<config>_<variant>.json
set -u
configs=$1; shift
mkdir -p gpurun_out/ab
for c in $configs; do
  for v in base "$@"; do
    lib=""; [ "$v" != base ] && lib=variants/$v.so
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config "$c" --steps 40 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/ab/${c}_$v.json 2> gpurun_out/ab/${c}_$v.err || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/ab/${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['roofline']['launch_ms'],4),round(b['kp_ms'],4))"
  done
done
