#!/bin/bash
# CG graph blocks: parity + CSR linear / RBF throughput with and without graphs + kernel trace
set -e
export TMPDIR=/tmp
root=$(pwd)
out=$root/gpurun_out/graph
mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sparse.py > $out/pytest.log 2>&1
for g in 1 0; do
  PLSSVM_MI_GRAPH=$g timeout -k 10 200 python bench.py --config csr_linear_1m --no-cpu --steps 200 --warmup 3 > $out/lin_g$g.json 2> $out/lin_g$g.err
  PLSSVM_MI_GRAPH=$g timeout -k 10 200 python bench.py --config csr_rbf_1m --no-cpu --steps 100 --warmup 3 > $out/rbf_g$g.json 2> $out/rbf_g$g.err
done
cd /tmp
PLSSVM_MI_GRAPH=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr0 -o run -- python3 $root/bench.py --config csr_linear_1m --no-cpu --steps 100 --warmup 3 > $out/tr0.json 2> $out/tr0.err
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $out/tr1 -o run -- python3 $root/bench.py --config csr_linear_1m --no-cpu --steps 100 --warmup 3 > $out/tr1.json 2> $out/tr1.err
