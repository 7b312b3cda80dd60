#!/bin/bash
# Predicted strong scaling without the collective: bench.py --sim-rank r/W for every rank r of a
# W-GPU job on one GPU (each run computes exactly rank r's share of the implicit matrix).
# usage (GPU box): tools/sim_shares.sh <config> <W> [extra bench args]; writes gpurun_out/shares_<config>_<W>.jsonl
set -e
config=$1; W=$2; shift 2
out=gpurun_out/shares_${config}_${W}.jsonl
: > "$out"
for r in $(seq 0 $((W - 1))); do
  timeout -k 10 300 python bench.py --config "$config" --sim-rank "$r/$W" --steps 5 --warmup 1 --no-cpu "$@" 2>/dev/null >> "$out"
done
python3 - "$out" <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
ms = [r["ms_per_step"] for r in rows]
print(json.dumps({"config": rows[0]["config"]["workload"], "W": len(rows), "ms_per_step_by_rank": ms,
                  "max_ms": max(ms), "mean_ms": sum(ms) / len(ms)}))
PY
