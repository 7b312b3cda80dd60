#!/bin/bash
# Remainder-stream geometry A/B on config 5 (PLSSVM_MI_EXP_RBB / PLSSVM_MI_EXP_G), same box, bench CG it/s
set -e
o=gpurun_out/geom; mkdir -p $o
for rep in 1 2; do
  for g in "def" "16384:1" "16384:2" "32768:2"; do
    if [ $g = def ]; then e=""; else e="PLSSVM_MI_EXP_RBB=${g%%:*} PLSSVM_MI_EXP_G=${g##*:}"; fi
    env $e timeout -k 10 300 python -u bench.py --config fp22_rbf_2m --steps 40 --warmup 5 --no-cpu --no-solve 2>/dev/null | tail -1 > $o/${g/:/_}_r$rep.json
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/geom/*.json")):
    d = json.load(open(f)); r = d["roofline"]
    print(f, round(d["value"], 1), round(r["launch_ms"], 4), round(r["kp_ms"], 4), r["pair_slots"])
PY
