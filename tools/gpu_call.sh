set -u
mkdir -p gpurun_out/c1
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/c1/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c1/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c1/smoke.log 2>&1 || exit $?
timeout -k 10 240 python bench.py > gpurun_out/c1/bench.json 2> gpurun_out/c1/bench.err; echo "bench rc=$?"; cat gpurun_out/c1/bench.json | cut -c1-600
for v in otf_v1 otf_v2; do
  PLSSVM_MI_LIB=variants/$v.so timeout -k 10 300 python tools/density_1pct.py --algo onthefly --reps 3 > gpurun_out/c1/dens_$v.json 2> gpurun_out/c1/dens_$v.err || exit $?
  cat gpurun_out/c1/dens_$v.json | cut -c1-400
done
