#!/bin/bash
# One gpurun call: the whole GPU test suite in one process (-> gpurun_out/<tag>/pytest.log).
# usage (GPU box, repo root): bash tools/gpu_suite.sh <tag> [pytest args...]
set -u
out=gpurun_out/${1:-suite}; shift || true
mkdir -p "$out"
timeout -k 10 1080 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > "$out/pytest.log" 2>&1
rc=$?
grep -E "FAILED|ERROR" "$out/pytest.log" | head -40
tail -3 "$out/pytest.log"
exit $rc
