#!/bin/bash
# A/B of the direction update carrying the expansion's w pass (PLSSVM_MI_DIR_W) + config-3 setup timing.
# usage (GPU box): tools/gpu_dirw_ab.sh ; writes gpurun_out/dw/
set -e
o=gpurun_out/dw; mkdir -p $o
PLSSVM_MI_TIMING=1 timeout -k 10 300 python -u bench.py --config csr_linear_1m --solve --no-cpu > $o/c3.log 2>&1
for rep in 1 2; do
  for v in 0 1; do
    for c in csr_rbf_1m fp22_rbf_2m; do
      PLSSVM_MI_DIR_W=$v timeout -k 10 300 python -u bench.py --config $c --steps 40 --warmup 5 --no-cpu 2>/dev/null | tail -1 > $o/${c}_dw${v}_r${rep}.json
    done
    PLSSVM_MI_SHARD=1 PLSSVM_MI_DIR_W=$v timeout -k 10 300 python -u bench.py --config fp22_rbf_2m --sim-rank 0/8 --steps 40 --warmup 5 --no-cpu 2>/dev/null | tail -1 > $o/share0_dw${v}_r${rep}.json
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/dw/*.json")):
    d = json.load(open(f)); print(f, round(d["value"], 1), round(d["ms_per_step"], 4))
PY
