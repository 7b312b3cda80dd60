#!/bin/bash
# Instruction mix of the remainder stream (exp_hcell_kernel) in the pair-flag (RF = 2) and chunk-flag (RF = 1) layouts
# on config 5: one rocprofv3 --pmc pass each (8 SQ counters), per slot of the stream.
# usage (GPU box, repo root): bash tools/pmc_hcell_rf.sh <tag>  -> gpurun_out/pmc_rf_<tag>/{pairs,flags}.json
set -u
root=$(pwd)
out=$root/gpurun_out/pmc_rf_$1
mkdir -p "$out"
export TMPDIR=/tmp
for rows in pairs flags; do
  cd /tmp
  PLSSVM_MI_EXP_ROWS=$rows timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS \
    --output-format csv -d "$out/$rows" -o run -- python3 "$root/bench.py" --config fp22_rbf_2m --steps 2 --warmup 0 --kp-reps 1 --no-cpu --no-extra --no-solve > "$out/$rows.bench.json" 2> "$out/$rows.log" || exit $?
  cd "$root"
  python3 - "$out" "$rows" <<'PY'
import csv, sys, collections, glob, json
out, rows = sys.argv[1], sys.argv[2]
f = glob.glob(f"{out}/{rows}/**/run_counter_collection.csv", recursive=True)[0]
d = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "exp_hcell_kernel" in r["Kernel_Name"]:
        d[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
last = list(d.values())[-1]
b = json.loads(open(f"{out}/{rows}.bench.json").read().strip().splitlines()[-1])
slots = b["roofline"]["pair_slots"]
res = {"layout": rows, "stream_layout": b["roofline"].get("stream_layout"), "slots": slots,
       "launch_ms": b["roofline"]["launch_ms"], "counters": {k: int(v) for k, v in last.items()},
       "per_slot": {k: v / slots for k, v in last.items() if k.startswith("SQ_INSTS")},
       "wait_any_per_wave_cycle": last["SQ_WAIT_INST_ANY"] / max(1.0, last["SQ_WAVE_CYCLES"]),
       "valu_active_per_wave_cycle": last["SQ_ACTIVE_INST_VALU"] / max(1.0, last["SQ_WAVE_CYCLES"])}
json.dump(res, open(f"{out}/{rows}.json", "w"), indent=1)
print(json.dumps(res))
PY
  find "$out/$rows" -name '*counter_collection.csv' -size +4M -exec gzip {} \;
done
