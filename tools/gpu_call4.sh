set -u
mkdir -p gpurun_out/c4
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py tests/test_gpu_overlap.py tests/test_gpu_fullsize.py > gpurun_out/c4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c4/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in csr_rbf_1m fp22_rbf_2m; do
  for v in index flags; do
    PLSSVM_MI_EXP_ROWS=$v timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/c4/rows_${c}_$v.json 2> gpurun_out/c4/rows_${c}_$v.err || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/c4/rows_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['roofline']['launch_ms'],4),b['kp_ms'],b['roofline']['stream_layout'],b['roofline']['alg_bytes'])"
  done
done
