#!/bin/bash
# One gpurun call: selected GPU tests (one process) then the default bench line.
# usage (GPU box, repo root): bash tools/gpu_quick.sh <tag> <pytest selection...>
set -u
tag=$1; shift
out=gpurun_out/$tag
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu "$@" > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$out/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py > "$out/bench.json" 2> "$out/bench.err"; brc=$?; echo "bench rc=$brc"
[ $brc -eq 0 ] || exit $brc
python3 - "$out/bench.json" <<'PY'
import json, sys
b = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for n, r in [("headline", b)] + list(b.get("extra", {}).items()):
    print(n, round(r["value"], 2), round(r["roofline"]["launch_ms"], 4), round(r["kp_ms"], 4), round(r["roofline"]["frac"], 3),
          r.get("learn", {}).get("learn_s"))
PY
exit $rc
