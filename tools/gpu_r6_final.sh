#!/bin/bash
# Round 6 final measurements (one gpurun call): remainder parity with printed errors, the 3-RBF profile, the pair /
# chunk flag PMC passes, and the default bench line.
set -u
mkdir -p gpurun_out/r6final
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_gpu_remainder.py \
  tests/test_gpu_sparse.py -k "remainder or row_pairs or row_flags or geometries" > gpurun_out/r6final/pytest.log 2>&1 || exit $?
grep -E "^remainder |passed|failed" gpurun_out/r6final/pytest.log
bash tools/profile_config.sh r06_csr_rbf_1m csr_rbf_1m || exit $?
bash tools/pmc_hcell_rf.sh r6final || exit $?
timeout -k 10 400 python bench.py > gpurun_out/r6final/bench.json 2> gpurun_out/r6final/bench.err || exit $?
python3 - <<'PY'
import json
b = json.loads(open("gpurun_out/r6final/bench.json").read().strip().splitlines()[-1])
for n, r in [("headline", b)] + list(b.get("extra", {}).items()):
    print(n, round(r["value"], 2), round(r["roofline"]["launch_ms"], 4), round(r["kp_ms"], 4), round(r["roofline"]["frac"], 3),
          r.get("learn", {}).get("learn_s"))
PY
