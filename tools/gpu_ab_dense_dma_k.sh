#!/bin/bash
# same-box A/B of the fp64 tile kernel's DMA order for the linear and polynomial kernel functions (config 2's shape)
set -e
mkdir -p gpurun_out/abk
for rep in 1 2; do
  for k in linear polynomial; do
    for v in base dma_early; do
      lib=""; [ "$v" != base ] && lib=variants/$v.so
      PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --kernel $k --no-extra --no-cpu --no-solve --steps 10 --warmup 2 --kp-reps 5 > gpurun_out/abk/${k}_${v}_$rep.json 2> gpurun_out/abk/${k}_${v}_$rep.err
      python3 -c "import json;b=json.loads(open('gpurun_out/abk/${k}_${v}_$rep.json').read().strip().splitlines()[-1]);print('$k $v',round(b['value'],3),round(b['roofline']['launch_ms'],3))"
    done
  done
done
