#!/bin/bash
# PMC pass over the dense pairwise tile kernel (config 2): MFMA busy / co-exec / wait cycles.
# usage (GPU box): tools/pmc_dense.sh <tag> [extra bench args]
set -e
tag=$1; shift
root=$(pwd)
out=$root/gpurun_out/pmc_dense_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU \
  --output-format csv -d "$out" -o run -- python3 "$root/bench.py" --steps 1 --warmup 0 --kp-reps 1 --no-cpu "$@" > "$out/bench.json" 2> "$out/bench.log"
python3 - "$out" <<'PY'
import csv, sys, collections, glob
out = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])))
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "kp_tile_kernel" in r["Kernel_Name"]:
        d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in list(d.items())[-1:]:
    print({a: int(b) for a, b in v.items()})
    print("mfma_busy/busy_cu", v["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1, v["SQ_BUSY_CU_CYCLES"]))
PY
