#!/bin/bash
# A/B of compile-time variants on one config: tools/gpu_var.sh <config> <steps> name...
# (BENCH_ARGS: extra bench.py arguments, e.g. "--sim-rank 0/8"; TAG: output name suffix)
set -e
cfg=$1; steps=$2; shift 2
out=gpurun_out/var; mkdir -p $out
for v in base "$@"; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  for rep in 1 2; do
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --no-cpu --steps $steps --warmup 3 ${BENCH_ARGS:-} \
      > $out/${cfg}${TAG:-}_${v}_$rep.json 2> $out/${cfg}${TAG:-}_${v}_$rep.err
  done
done
python3 - "$out" "$cfg${TAG:-}" <<'PY'
import glob, json, sys
for f in sorted(glob.glob(f"{sys.argv[1]}/{sys.argv[2]}_*.json")):
    l = [x for x in open(f) if x.startswith("{")]
    if l:
        r = json.loads(l[-1])
        print(f.split("/")[-1], round(r["ms_per_step"], 4), round(r["value"], 1))
PY
