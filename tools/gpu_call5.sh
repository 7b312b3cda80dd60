set -u
mkdir -p gpurun_out/c5
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_sparse.py -k "expansion or sparse_kp" > gpurun_out/c5/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/c5/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for c in csr_rbf_1m fp22_rbf_2m; do
  for v in jh1 jh0 jh1b; do
    lib=""; [ $v = jh0 ] && lib=variants/jh0.so
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/c5/jh_${c}_$v.json 2> gpurun_out/c5/jh_${c}_$v.err || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/c5/jh_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['roofline']['launch_ms'],4),b['kp_ms'])"
  done
done
