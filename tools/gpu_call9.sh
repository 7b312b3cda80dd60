set -u
mkdir -p gpurun_out/c9
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/c9/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c9/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c9/smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > gpurun_out/c9/bench.json 2> gpurun_out/c9/bench.err; echo "bench rc=$?"
python3 -c "
import json
b=json.loads(open('gpurun_out/c9/bench.json').read().strip().splitlines()[-1])
for n,r in [('headline',b)]+list(b['extra'].items()):
    print(n, round(r['value'],1), round(r['roofline']['launch_ms'],4), round(r['kp_ms'],4), round(r['roofline']['frac'],3))"
bash tools/profile_config.sh r03_csr_linear_1m csr_linear_1m || exit $?
for v in int2 s16; do
  sv=""; [ $v = int2 ] && sv=int2
  PLSSVM_MI_OTF_SEG=$sv timeout -k 10 300 python tools/density_1pct.py --algo onthefly --reps 3 > gpurun_out/c9/dens_$v.json 2> gpurun_out/c9/dens_$v.err || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/c9/dens_$v.json')); print('$v', d['kp_s'], d['max_rel_err'], d['ok'])"
done
