set -u
mkdir -p gpurun_out/c8
for c in csr_rbf_1m fp22_rbf_2m csr_linear_1m; do
  for v in u4 u6 u8; do
    lib=""; [ $v != u4 ] && lib=variants/$v.so
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps 40 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/c8/u_${c}_$v.json 2> gpurun_out/c8/u_${c}_$v.err || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/c8/u_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['roofline']['launch_ms'],4),b['kp_ms'])"
  done
done
