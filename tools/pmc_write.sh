#!/bin/bash
# WRITE_SIZE pass (HBM write bytes per dispatch) of one bench configuration (GPU box, repo root):
# tools/pmc_write.sh <tag> <config> [bench args] -> gpurun_out/pmcw_<tag>/ (per-kernel mean bytes in summary.json)
set -e
tag=$1; config=$2; shift 2
root=$(pwd)
out=$root/gpurun_out/pmcw_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out" -o run -- \
  python3 "$root/bench.py" --config "$config" --steps 2 --warmup 0 --kp-reps 1 --no-cpu --no-extra --no-solve "$@" \
  > "$out/bench.json" 2> "$out/bench.log"
python3 - "$out" <<'PY'
import csv, sys, collections, glob, json
out = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])))
d = collections.defaultdict(list)
for r in rows:
    d[r["Kernel_Name"][:90]].append(float(r["Counter_Value"]))
res = {k: {"dispatches": len(v), "write_kib_mean": sum(v) / len(v)} for k, v in d.items()}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
PY
find "$out" -name "run_counter_collection.csv" -size +8M -exec gzip {} \;
echo "pmcw $tag done"
