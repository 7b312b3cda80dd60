#!/bin/bash
# sparse-linear CG parity + throughput + kernel trace
set -e
export TMPDIR=/tmp
root=$(pwd)
out=$root/gpurun_out/lin; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_golden.py -k "not geometries" > $out/pytest.log 2>&1
for nb in 256 128; do
PLSSVM_MI_SELL_BLOCKS=$nb timeout -k 10 200 python bench.py --config csr_linear_1m --no-cpu --steps 300 --warmup 3 > $out/lin$nb.json 2> $out/lin$nb.err
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr -o run -- python3 $root/bench.py --config csr_linear_1m --no-cpu --steps 100 --warmup 3 > $out/tr.json 2> $out/tr.err
