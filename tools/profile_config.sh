#!/bin/bash
# Profile one bench.py configuration on the GPU box (run under gpurun, from the repo root):
#   1. rocprofv3 --kernel-trace --stats  (per-kernel average durations; the bench line of the same run)
#   2. rocprofv3 --pmc FETCH_SIZE        (separate pass: HBM read bytes per dispatch, for roofline.traffic)
# usage: tools/profile_config.sh <tag> <config> [extra bench.py args]
# outputs under gpurun_out/prof_<tag>/ ; tools/pmc_traffic.py turns them into profiles/ summaries.
set -eu
tag=$1; config=$2; shift 2
root=$(pwd)
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --config "$config" --steps 5 --warmup 1 --no-cpu --no-extra --no-solve "$@" > "$out/bench_trace.json" 2> "$out/trace.log"
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc" -o run -- \
  python3 "$root/bench.py" --config "$config" --steps 2 --warmup 0 --kp-reps 2 --no-cpu --no-extra --no-solve "$@" > "$out/bench_pmc.json" 2> "$out/pmc.log"
# keep only the summaries gpurun copies back (traces of long runs exceed its 64 MiB limit)
find "$out" -type f ! -name '*kernel_stats.csv' ! -name '*counter_collection.csv' ! -name '*.json' ! -name '*.log' -delete
find "$out" -name '*counter_collection.csv' -size +8M -exec gzip {} \;
du -sh "$out"
echo "profile $tag ($config) done"
