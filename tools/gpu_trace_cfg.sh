#!/bin/bash
# kernel trace of one bench config (short run): tools/gpu_trace_cfg.sh <config> <steps> [tag]
set -e
export TMPDIR=/tmp
root=$(pwd)
cfg=$1; steps=$2; tag=${3:-$1}
out=$root/gpurun_out/trc_$tag; mkdir -p $out
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python3 $root/bench.py --config $cfg --no-cpu --steps $steps --warmup 2 > $out/bench.json 2> $out/bench.err
