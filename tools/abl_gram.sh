set -e
for cfg in "fp22_rbf_2m --sim-rank 0/8" "csr_rbf_1m"; do
 for a in 0 1 2 3; do
  echo "== $cfg ablate=$a"
  PLSSVM_MI_GRAM_ABLATE=$a timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu 2>gpurun_out/abl_err.log | python -c "import json,sys;d=json.loads(sys.stdin.read().strip().splitlines()[-1]);r=d['roofline'];print(r['launch_ms'],r.get('stream_GBps'),r['pairs'],r['pair_slots'])"
 done
done
