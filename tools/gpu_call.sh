#!/bin/bash
# One gpurun call: the GPU test suite (one process), smoke(), the default bench line.
# usage (GPU box, repo root): bash tools/gpu_call.sh [tag]   -> gpurun_out/<tag>/{pytest.log,smoke.log,bench.json}
set -u
out=gpurun_out/${1:-suite}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$out/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
timeout -k 10 240 python bench.py > "$out/bench.json" 2> "$out/bench.err"; echo "bench rc=$?"
python3 - "$out/bench.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for n, r in [("headline", b)] + list(b.get("extra", {}).items()):
    print(n, round(r["value"], 1), round(r["roofline"]["launch_ms"], 4), round(r["kp_ms"], 4), round(r["roofline"]["frac"], 3))
PY
