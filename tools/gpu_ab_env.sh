#!/bin/bash
# A/B of environment settings (same library) on one bench configuration, same box.
# usage (GPU box, repo root): bash tools/gpu_ab_env.sh <config> <name>=<VAR=val[,VAR=val]> ...  ("base" = no change)
#   -> gpurun_out/ab/<config>_env_<name>.json
set -u
c=$1; shift
mkdir -p gpurun_out/ab
for spec in "base=" "$@"; do
  name=${spec%%=*}; vars=${spec#*=}
  ( IFS=','; for kv in $vars; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 200 python bench.py --config "$c" --steps 40 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/ab/${c}_env_$name.json 2> gpurun_out/ab/${c}_env_$name.err ) || exit $?
  python3 -c "import json;b=json.loads(open('gpurun_out/ab/${c}_env_$name.json').read().strip().splitlines()[-1]);print('$c $name',round(b['value'],1),round(b['roofline']['launch_ms'],4),round(b['kp_ms'],4))"
done
