#!/bin/bash
# Config 5's rank shares at 8 GPUs with both CG recurrences and the one-GPU iteration on the same box
# (predicted scaling inputs). usage (GPU box): bash tools/gpu_shares_cg.sh <tag>  -> gpurun_out/<tag>/
set -u
out=gpurun_out/$1
mkdir -p "$out"
for v in one_reduction reference; do
  PLSSVM_MI_SHARD=1 bash tools/sim_shares.sh fp22_rbf_2m 8 --cg-variant $v --kp-reps 3 || exit $?
  mv gpurun_out/shares_fp22_rbf_2m_8.jsonl "$out/shares_$v.jsonl"
done
timeout -k 10 300 python bench.py --config fp22_rbf_2m --steps 40 --warmup 2 --no-cpu > "$out/one_gpu.json" 2> "$out/one_gpu.err" || exit $?
python3 -c "import json;b=json.loads(open('$out/one_gpu.json').read().strip().splitlines()[-1]);print('one GPU', b['ms_per_step'])"
