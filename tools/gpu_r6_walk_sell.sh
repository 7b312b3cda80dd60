#!/bin/bash
# Round-6 check of the remainder walk and the FP22 SELL step depth (one gpurun call).
set -u
bash tools/gpu_ab.sh "fp22_rbf_2m csr_rbf_1m" prewalk || exit $?
bash tools/gpu_suite.sh r6walk2 tests/test_gpu_remainder.py tests/test_gpu_sparse.py tests/test_gpu_cg_trace_long.py -k "expansion or remainder or geometries or bf16 or row_ or dot2 or long" || exit $?
bash tools/prof_stats.sh su4 --config fp22_rbf_2m --steps 20 --warmup 2 --no-extra --no-solve || exit $?
PLSSVM_MI_LIB=variants/f22su8.so bash tools/prof_stats.sh su8 --config fp22_rbf_2m --steps 20 --warmup 2 --no-extra --no-solve || exit $?
for t in su4 su8; do
  python3 - "$t" <<'PY'
import csv, glob, sys
t = sys.argv[1]
f = glob.glob(f"gpurun_out/stats_{t}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "sell_spmv" in r["Name"] or "exp_hcell" in r["Name"]:
        print(t, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
done
