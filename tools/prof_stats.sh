#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench.py configuration (under gpurun, from the repo root)
# usage: tools/prof_stats.sh <tag> <bench args...>   -> gpurun_out/stats_<tag>/...kernel_stats.csv + bench.json
set -eu
tag=$1; shift
root=$(pwd)
out=$root/gpurun_out/stats_$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
  python3 "$root/bench.py" --no-cpu "$@" > "$out/bench.json" 2> "$out/bench.err"
find "$out" -type f ! -name '*kernel_stats.csv' ! -name '*.json' ! -name '*.err' -delete
echo "stats $tag done"
