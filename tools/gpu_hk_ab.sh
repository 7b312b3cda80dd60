#!/bin/bash
# Same-box kernel durations (rocprofv3 --kernel-trace --stats) of the setup kernels, base vs cur, per config.
# usage (GPU box): tools/gpu_hk_ab.sh <variant>... ; writes gpurun_out/hk/
set -e
R=$PWD; o=$R/gpurun_out/hk; mkdir -p $o
export TMPDIR=/tmp
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != cur ] && lib=$R/variants/$v/libplssvm_mi355x.so
    for c in csr_rbf_1m fp22_rbf_2m; do
      (cd /tmp && PLSSVM_MI_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/${c}_${v}_r$rep -o run -- python3 $R/bench.py --config $c --solve --steps 2 --warmup 0 --no-cpu --no-extra > /dev/null 2>&1)
      find $o/${c}_${v}_r$rep -type f ! -name '*kernel_stats.csv' -delete
    done
  done
done
python3 - $o <<'PY'
import csv, glob, sys
for f in sorted(glob.glob(sys.argv[1] + "/*/**/run_kernel_stats.csv", recursive=True)):
    rows = {r["Name"]: float(r["AverageNs"]) / 1e6 for r in csv.DictReader(open(f))}
    pick = {k.split("(")[0].split("::")[-1][:32]: round(v, 1) for k, v in rows.items() if "rowjoin" in k}
    print(f.split("/")[-4] if "/r" in f else f, pick)
PY
