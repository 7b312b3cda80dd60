set -u
mkdir -p gpurun_out/cg1ab
for c in csr_linear_1m csr_rbf_1m fp22_rbf_2m; do
  for v in reference one_reduction reference one_reduction; do
    timeout -k 10 200 python bench.py --config $c --cg-variant $v --steps 60 --warmup 3 --no-cpu --no-solve --kp-reps 3 > gpurun_out/cg1ab/${c}_$v.json 2>/dev/null || exit $?
    python3 -c "import json;b=json.loads(open('gpurun_out/cg1ab/${c}_$v.json').read().strip().splitlines()[-1]);print('$c $v', round(b['value'],1), round(b['ms_per_step'],4))"
  done
done
