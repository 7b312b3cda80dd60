#!/bin/bash
# same-box A/B of the tile kernel's DMA order (variants/dma_early.so = old order) + dense parity
set -e
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/parity.log 2>&1
for rep in 1 2; do
  for v in base dma_early; do
    lib=""; [ "$v" != base ] && lib=variants/$v.so
    PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --no-extra --no-cpu --no-solve --steps 10 --warmup 2 --kp-reps 5 > gpurun_out/ab/d2_${v}_$rep.json 2> gpurun_out/ab/d2_${v}_$rep.err
    python3 -c "import json;b=json.loads(open('gpurun_out/ab/d2_${v}_$rep.json').read().strip().splitlines()[-1]);print('dense_rbf $v',round(b['value'],3),round(b['roofline']['launch_ms'],3),round(b['roofline']['frac'],4))"
  done
done
for v in base dma_early; do
  lib=""; [ "$v" != base ] && lib=variants/$v.so
  PLSSVM_MI_LIB=$lib timeout -k 10 200 python bench.py --config dense_linear_500k --no-cpu --steps 1 --warmup 0 --kp-reps 1 > gpurun_out/ab/dl_${v}.json 2> gpurun_out/ab/dl_${v}.err
  python3 -c "import json;b=json.loads(open('gpurun_out/ab/dl_${v}.json').read().strip().splitlines()[-1]);print('dense_linear $v',round(b['value'],4),round(b['roofline']['launch_ms'],1),round(b['roofline']['frac'],4))"
done
