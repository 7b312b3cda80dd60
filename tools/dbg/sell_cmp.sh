#!/bin/bash
set -u
mkdir -p gpurun_out/sc
timeout -k 10 300 python tools/dbg/sell_cmp.py gpurun_out/sc/a.npz > gpurun_out/sc/a.log 2>&1 || exit $?
PLSSVM_MI_LIB=variants/$1.so timeout -k 10 300 python tools/dbg/sell_cmp.py gpurun_out/sc/b.npz > gpurun_out/sc/b.log 2>&1 || exit $?
python3 -c "
import numpy as np
a=np.load('gpurun_out/sc/a.npz'); b=np.load('gpurun_out/sc/b.npz')
for k in a.files: print(k, 'bitwise' if np.array_equal(a[k], b[k]) else 'DIFF max %g' % np.abs(a[k]-b[k]).max())
"
shift
bash tools/gpu_ab.sh "csr_linear_1m csr_rbf_1m fp22_rbf_2m" "$@"
