#!/bin/bash
# multi-rank (host-staged world-2 groups on one GPU) + sparse + overlap parity
set -e
out=gpurun_out/mr; mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multirank.py tests/test_gpu_overlap.py > $out/pytest.log 2>&1
