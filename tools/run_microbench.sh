#!/bin/bash
# Build and run tools/spmv_microbench.hip on the GPU box for several unroll depths.
set -e
mkdir -p gpurun_out
for u in "$@"; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPLSSVM_MI_SELL_UNROLL=$u tools/spmv_microbench.hip -o /tmp/mb_$u 2>/dev/null
  echo "== unroll $u"
  timeout -k 10 200 /tmp/mb_$u
done
