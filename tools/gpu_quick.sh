#!/bin/bash
# GPU parity of the CG / sparse paths + the three sparse bench rows
set -e
out=gpurun_out/quick; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_sparse.py tests/test_gpu_overlap.py > $out/pytest.log 2>&1
timeout -k 10 200 python bench.py --config csr_linear_1m --no-cpu --steps 300 --warmup 3 > $out/lin.json 2> $out/lin.err
timeout -k 10 200 python bench.py --config csr_rbf_1m --no-cpu --steps 50 --warmup 3 > $out/rbf.json 2> $out/rbf.err
timeout -k 10 300 python bench.py --config fp22_rbf_2m --no-cpu --steps 30 --warmup 2 > $out/fp22.json 2> $out/fp22.err
