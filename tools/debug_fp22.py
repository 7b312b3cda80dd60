"""Debug helper (GPU box): where do FP22 sparse Gram K·p results go NaN (linear pairwise)?"""
import sys, numpy as np
sys.path.insert(0, ".")
import plssvm_sparse_fp22_amd as pm
if len(sys.argv) > 1:  # compare another build of the library
    pm._abi.LIB_PATH = sys.argv[1]
from plssvm_sparse_fp22_amd import datagen
from plssvm_sparse_fp22_amd.fp22 import pack, unpack
n, d, k = 20000, 4000, 50
csr, y = datagen.sparse_csr(n, d, k, seed=5, dtype=np.float32)
dec = unpack(pack(csr[2]), csr[2].size)
res = {}
for fmt in ("real", "fp22"):
    p = pm.Parameter("linear", real_type=np.float32)
    if fmt == "fp22":
        p.csr = (csr[0], csr[1], pack(csr[2]), n, d); p.val_fmt = pm._abi.VAL_FP22
    else:
        p.csr = (csr[0], csr[1], dec, n, d)
    with pm.CSVM(p, kp_mode="pairwise") as svm:
        svm.setup_data_on_device()
        res["q_" + fmt] = svm.generate_q()
        for trial in range(2):
            r = svm.run_device_kernel(None, np.zeros(n - 1, np.float32), np.ones(n - 1, np.float32), 1.0)
            bad = np.flatnonzero(~np.isfinite(r))
            print(fmt, trial, "nonfinite", bad.size, "blocks", np.unique(bad // 2048)[:20], "first", bad[:10], flush=True)
        res[fmt] = r
qd = np.abs(res["q_fp22"] - res["q_real"])
print("q max abs diff", qd.max(), "rows with diff", np.flatnonzero(qd > 1e-3)[:10], (qd > 1e-3).sum())
ok = np.isfinite(res["fp22"])
print("max rel diff on finite rows", np.max(np.abs(res["fp22"][ok] - res["real"][ok]) / np.abs(res["real"][ok])))
