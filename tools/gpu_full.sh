#!/bin/bash
# full GPU test suite (one process) + smoke
set -e
out=gpurun_out/full; mkdir -p $out
timeout -k 10 1000 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > $out/pytest.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1
