#!/bin/bash
# learn_s and setup phases of the sparse BASELINE sets (bench --solve, PLSSVM_MI_TIMING=1), two runs each
# usage (GPU box): tools/gpu_setup_times.sh <tag> [env assignments...]; writes gpurun_out/st_<tag>/
set -e
tag=$1; shift
o=gpurun_out/st_$tag; mkdir -p $o
for rep in 1 2; do
  for c in csr_rbf_1m fp22_rbf_2m csr_linear_1m; do
    env "$@" PLSSVM_MI_TIMING=1 timeout -k 10 300 python -u bench.py --config $c --solve --steps 5 --warmup 1 --no-cpu > $o/${c}_r${rep}.json 2> $o/${c}_r${rep}.err
  done
done
python3 - $o <<'PY'
import json, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1]); print(f, d["learn"]["learn_s"], d["config"]["setup_s"], round(d["value"], 1))
PY
