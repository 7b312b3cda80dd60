set -u
mkdir -p gpurun_out/c2
bash tools/gpu_profiles.sh r03 || exit $?
# remainder-stream step depth A/B (EXP_NH = 2 in-tree, 3, 4), same box
for c in csr_rbf_1m fp22_rbf_2m; do
  for v in nh2 nh3 nh4; do
    lib=""; [ $v != nh2 ] && lib=variants/$v.so
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 2 --no-cpu --kp-reps 20 > gpurun_out/c2/nh_${c}_$v.json 2> gpurun_out/c2/nh_${c}_$v.err || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/c2/nh_${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['roofline']['launch_ms'],4),b['kp_ms'])"
  done
done
