#!/bin/bash
# The bench's N > 1 flow on a one-GPU box: two ranks on the same device, joined by the host-staged exchange
# (RCCL refuses two ranks on one device), through torch.distributed.run exactly as the driver launches N > 1.
set -u
mkdir -p gpurun_out/world2
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 5 --warmup 1 --host-exchange > gpurun_out/world2/bench.json 2> gpurun_out/world2/bench.err
rc=$?; echo "world-2 bench rc=$rc"; tail -c 700 gpurun_out/world2/bench.json; exit $rc
