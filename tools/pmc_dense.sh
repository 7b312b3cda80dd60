#!/bin/bash
# PMC pass over the dense pairwise tile kernel: MFMA busy / co-exec / wait cycles (one rocprofv3 --pmc
# pass, 8 SQ counters). usage (GPU box): tools/pmc_dense.sh <tag> [extra bench args, e.g. --config X]
# Writes gpurun_out/pmc_dense_<tag>/summary.json: counters of the last kp_tile_kernel dispatch and
# mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x SQ_BUSY_CU_CYCLES).
set -e
tag=$1; shift
root=$(pwd)
out=$root/gpurun_out/pmc_dense_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_COEXEC_CYCLES SQ_INSTS_VALU \
  --output-format csv -d "$out" -o run -- python3 "$root/bench.py" --steps 1 --warmup 0 --kp-reps 1 --no-cpu --no-extra --no-solve "$@" > "$out/bench.json" 2> "$out/bench.log"
python3 - "$out" "$*" <<'PY'
import csv, sys, collections, glob, json
out, args = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])))
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in rows:
    if "kp_tile_kernel" in r["Kernel_Name"]:
        d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
last = list(d.values())[-1]
b = open(out + "/bench.json").read()
b = json.loads(b[b.index('{"metric'):].splitlines()[0])
res = {"config": b["config"]["workload"], "N": b["config"]["N"], "d": b["config"]["d"],
       "kernel": b["config"]["kernel"], "dtype": b["dtype"], "n_gpus": b["n_gpus"], "bench_args": args,
       "counters": {a: int(b) for a, b in last.items()},
       "mfma_util": last["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, 4 * last["SQ_BUSY_CU_CYCLES"]),
       "coexec_cycles": int(last["SQ_VALU_MFMA_COEXEC_CYCLES"])}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(res))
PY
find "$out" -name '*counter_collection.csv' -size +8M -exec gzip {} \;
