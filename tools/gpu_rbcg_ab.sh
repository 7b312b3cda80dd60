#!/bin/bash
# A/B of the row-block pass carrying the CG vector updates (PLSSVM_MI_RB_CG) on config 3, same box
set -e
o=gpurun_out/rbcg; mkdir -p $o
for rep in 1 2 3; do
  for v in 0 1; do
    PLSSVM_MI_RB_CG=$v timeout -k 10 200 python -u bench.py --config csr_linear_1m --steps 200 --warmup 20 --no-cpu --no-solve 2>/dev/null | tail -1 > $o/rb${v}_r$rep.json
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/rbcg/*.json")):
    d = json.load(open(f)); print(f, round(d["value"], 1), round(d["ms_per_step"], 5))
PY
