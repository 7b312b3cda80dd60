#!/bin/bash
# PMC pass over one kernel of a bench configuration: instruction mix and stall picture (one rocprofv3 --pmc pass,
# 8 SQ counters). usage (GPU box): tools/pmc_kernel.sh <tag> <config> <kernel name substring> [bench args]
#   -> gpurun_out/pmc_<tag>/summary.json (counters of the last dispatch of the kernel)
set -e
tag=$1; config=$2; kname=$3; shift 3
root=$(pwd)
out=$root/gpurun_out/pmc_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT \
  --output-format csv -d "$out" -o run -- python3 "$root/bench.py" --config "$config" --steps 2 --warmup 0 --kp-reps 1 --no-cpu --no-extra --no-solve "$@" > "$out/bench.json" 2> "$out/bench.log"
python3 - "$out" "$kname" <<'PY'
import csv, sys, collections, glob, json
out, kname = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(out + "/**/run_counter_collection.csv", recursive=True)[0])))
d = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in rows:
    if kname in r["Kernel_Name"]:
        d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:160]
last_id = list(d)[-1]
last = d[last_id]
res = {"kernel": names[last_id], "dispatches": len(d), "counters": {a: int(b) for a, b in last.items()},
       "valu_active_per_wave_cycle": last["SQ_ACTIVE_INST_VALU"] / max(1.0, last["SQ_WAVE_CYCLES"]),
       "wait_inst_any_per_wave_cycle": last["SQ_WAIT_INST_ANY"] / max(1.0, last["SQ_WAVE_CYCLES"]),
       "valu_per_vmem_rd": last["SQ_INSTS_VALU"] / max(1.0, last["SQ_INSTS_VMEM_RD"])}
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps(res))
PY
find "$out" -name '*counter_collection.csv' -size +8M -exec gzip {} \;
