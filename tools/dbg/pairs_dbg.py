"""debug: pair flags vs chunk flags on one configuration (GPU)."""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

def svm_for(csr, rows):
    os.environ["PLSSVM_MI_EXP_ROWS"] = rows
    p = pm.Parameter("rbf", gamma=1.0 / csr[4], real_type=np.float32)
    p.csr = csr
    return pm.CSVM(p, sparse_algo="expansion")

for rbb, g in [("4096", "1"), ("8192", "3"), ("auto", "0")]:
    if rbb != "auto":
        os.environ["PLSSVM_MI_EXP_RBB"] = rbb; os.environ["PLSSVM_MI_EXP_G"] = g
    else:
        os.environ.pop("PLSSVM_MI_EXP_RBB", None); os.environ.pop("PLSSVM_MI_EXP_G", None)
    csr, _ = datagen.sparse_csr(140000, 3000, 20, seed=23, dtype=np.float32)
    x = np.random.default_rng(9).uniform(-1, 2, csr[3] - 1).astype(np.float32)
    out = {}
    for rows in ("index", "flags", "pairs"):
        with svm_for(csr, rows) as svm:
            svm.setup_data_on_device()
            info = svm.info()
            out[rows] = svm.kp_part(x, "overlap").astype(np.float64)
            print(rbb, rows, "layout", info["exp_layout"], "slots", info["pair_slots"], "RB?", info["exp_waves"], flush=True)
    d = np.abs(out["pairs"] - out["flags"])
    bad = np.nonzero(d > 1e-6 * (np.abs(out["flags"]) + 1e-3))[0]
    print(rbb, "index==flags", np.array_equal(out["index"], out["flags"]), "bad rows", bad.size, bad[:20], "maxabs", d.max(), flush=True)
    if bad.size:
        print("  values flags", out["flags"][bad[:5]], "pairs", out["pairs"][bad[:5]], flush=True)
