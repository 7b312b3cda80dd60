#!/bin/bash
# sparse GPU parity (CSR paths incl. the densified fallback)
set -e
out=gpurun_out/sparse; mkdir -p $out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_sparse.py > $out/pytest.log 2>&1
