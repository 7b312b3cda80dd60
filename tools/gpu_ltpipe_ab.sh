#!/bin/bash
# A/B of the lower-triangle join + H pipeline (PLSSVM_MI_EXP_LT_PIPE chunks): setup phases and learn_s
# usage (GPU box): tools/gpu_ltpipe_ab.sh ; writes gpurun_out/lp/
set -e
o=gpurun_out/lp; mkdir -p $o
for rep in 1 2; do
  for v in 1 8 16; do
    for c in csr_rbf_1m fp22_rbf_2m; do
      PLSSVM_MI_TIMING=1 PLSSVM_MI_EXP_LT_PIPE=$v timeout -k 10 300 python -u bench.py --config $c --solve --steps 5 --warmup 1 --no-cpu > $o/${c}_p${v}_r${rep}.json 2> $o/${c}_p${v}_r${rep}.err
    done
  done
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/lp/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["learn"]["learn_s"], d["config"]["setup_s"])
PY
