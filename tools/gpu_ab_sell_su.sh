#!/bin/bash
# same-box A/B of the SELL passes' entries per lane per step for real-typed values (variants/suN.so)
set -e
mkdir -p gpurun_out/su
for rep in 1 2; do
  for c in csr_linear_1m csr_rbf_1m; do
    for v in base su12 su16; do
      lib=""; [ "$v" != base ] && lib=variants/$v.so
      PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config $c --no-cpu --steps 100 --warmup 3 --kp-reps 20 > gpurun_out/su/${c}_${v}_$rep.json 2> gpurun_out/su/${c}_${v}_$rep.err
      python3 -c "import json;b=json.loads(open('gpurun_out/su/${c}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$c $v',round(b['value'],1),round(b['kp_ms'],4))"
    done
  done
done
