#!/bin/bash
# Round 6: repeated same-box A/B of the remainder walk (3-RBF) and rocprof kernel stats of the FP22 SELL step depth.
set -u
root=$(pwd)
for i in 1 2 3; do
  bash tools/gpu_ab.sh csr_rbf_1m prewalk || exit $?
done
for v in su4 su6 su8; do
  lib=""; [ "$v" != su4 ] && lib=$root/variants/f22$v.so
  PLSSVM_MI_LIB=$lib bash tools/prof_stats.sh $v --config fp22_rbf_2m --steps 20 --warmup 2 --no-extra --no-solve || exit $?
  python3 - "$v" <<'PY'
import csv, glob, sys
t = sys.argv[1]
f = glob.glob(f"gpurun_out/stats_{t}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sell_spmv" in r["Name"] or "exp_hcell" in r["Name"]:
        print(t, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
