#!/bin/bash
# Remainder-stream geometry of one config-5 rank share of 8 (sharded, one-reduction CG): row-block class x window
# groups. usage (GPU box, repo root): bash tools/gpu_share_geom.sh  -> gpurun_out/share_geom/<rbb>_<g>.json
set -u
out=gpurun_out/share_geom
mkdir -p "$out"
for cfg in default 32768:8 32768:4 16384:4 16384:8 8192:2 8192:4 4096:1 4096:2; do
  if [ "$cfg" = default ]; then env=""; else env="PLSSVM_MI_EXP_RBB=${cfg%:*} PLSSVM_MI_EXP_G=${cfg#*:}"; fi
  env PLSSVM_MI_SHARD=1 $env timeout -k 10 200 python bench.py --config fp22_rbf_2m --sim-rank 3/8 --cg-variant one_reduction \
    --steps 30 --warmup 2 --no-cpu --no-extra --no-solve --kp-reps 5 > "$out/${cfg/:/_}.json" 2> "$out/${cfg/:/_}.err" || exit $?
  python3 -c "import json;b=json.loads(open('$out/${cfg/:/_}.json').read().strip().splitlines()[-1]);r=b['roofline'];print('$cfg', round(b['ms_per_step'],4), round(r['launch_ms'],4), round(b['kp_ms'],4))"
done
