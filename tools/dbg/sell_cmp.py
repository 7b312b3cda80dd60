"""debug: K·p outputs of the in-tree library vs a variant (PLSSVM_MI_LIB), bitwise (GPU). usage: sell_cmp.py out.npz"""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

out = {}
cases = [("linear", np.float32, False, (300000, 50000, 50)), ("linear", np.float64, False, (200000, 20000, 30)),
         ("rbf", np.float32, False, (300000, 50000, 50)), ("rbf", np.float32, True, (300000, 100000, 50)),
         ("rbf", np.float64, False, (100000, 5000, 20)), ("polynomial", np.float32, False, (50000, 2000, 16)),
         ("linear", np.float32, True, (100000, 3000, 9))]
for kern, dt, f22, (n, d, k) in cases:
    csr, _ = datagen.sparse_csr(n, d, k, seed=n + d, dtype=np.float32 if dt == np.float32 else np.float64)
    p = pm.Parameter(kern, gamma=1.0 / d, coef0=1.0, real_type=dt)
    if f22:
        from plssvm_sparse_fp22_amd import fp22
        p.csr = (csr[0], csr[1], fp22.pack(csr[2]), n, d)
        p.val_fmt = pm._abi.VAL_FP22
    else:
        p.csr = (csr[0], csr[1], csr[2].astype(dt), n, d)
    with pm.CSVM(p) as svm:
        svm.setup_data_on_device()
        svm.generate_q()
        x = np.random.default_rng(3).uniform(-1, 2, n - 1).astype(dt)
        ret = np.zeros(n - 1, dt)
        svm.run_device_kernel(None, ret, x, 1.0)
        out[f"{kern}_{np.dtype(dt).name}_{f22}"] = ret
        print(kern, dt, f22, svm.info()["sparse_algo"], flush=True)
np.savez(sys.argv[1], **out)
