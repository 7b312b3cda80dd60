"""Problem definitions shared by tests/mr_worker.py (each rank) and tests/test_gpu_multirank.py
(the oracle side): same seeded data on every rank, as the reference replicates data_ptr_."""
import numpy as np

import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

# name: (layout, kernel, kp_mode, dtype, imax)
CASES = {
    "dense_rbf": ("dense", "rbf", "auto", np.float64, 40),
    "dense_poly": ("dense", "polynomial", "auto", np.float64, 40),
    "dense_linear_pairwise": ("dense", "linear", "pairwise", np.float64, 40),
    "dense_linear_factored": ("dense", "linear", "factored", np.float64, 40),
    "sparse_linear": ("csr", "linear", "auto", np.float64, 40),
    "sparse_rbf": ("csr", "rbf", "auto", np.float64, 40),
    "sparse_poly": ("csr", "polynomial", "auto", np.float64, 40),
    "sparse_fp22_rbf": ("fp22", "rbf", "auto", np.float32, 10),
    "sparse_rbf_onthefly": ("csr", "rbf", "auto", np.float64, 40),
    "sparse_poly_onthefly": ("csr", "polynomial", "auto", np.float64, 40),
    "sparse_rbf_budget_split": ("csr", "rbf", "auto", np.float64, 40),
}
# sparse poly / rbf K·p algorithm per case (default: auto)
ALGO = {"sparse_rbf_onthefly": "onthefly", "sparse_poly_onthefly": "onthefly"}
# per-rank device-memory budgets (PLSSVM_MI_MEM_BUDGET, bytes): the ranks' own estimates straddle the
# budget — rank 0 would store the kernel expansion, rank 1 cannot — so only a group-wide decision keeps
# both on one path
BUDGET = {"sparse_rbf_budget_split": {1: "1"}}
# cases whose K·p stores no pairs (on the fly / densified)
UNSTORED = set(ALGO) | set(BUDGET)


def case_data(name):
    layout, kernel, kp_mode, dtype, imax = CASES[name]
    if layout == "dense":
        X, y = datagen.blobs(3000, 64, seed=3, cluster_std=4.0, dtype=dtype)
        return dict(X=X), y, 64
    csr, y = datagen.sparse_csr(6500, 5000, 20, seed=2, dtype=dtype)
    return dict(csr=csr), y, csr[4]


def make_case(name):
    layout, kernel, kp_mode, dtype, imax = CASES[name]
    data, y, d = case_data(name)
    prm = pm.Parameter(kernel, gamma=1.0 / d, coef0=1.0 if kernel == "polynomial" else 0.0, real_type=dtype)
    if "X" in data:
        prm.data = data["X"]
    elif layout == "fp22":
        from plssvm_sparse_fp22_amd.fp22 import pack

        rowptr, col, val, n, dd = data["csr"]
        prm.csr = (rowptr, col, pack(val), n, dd)
        prm.val_fmt = pm._abi.VAL_FP22
    else:
        prm.csr = data["csr"]
    prm.labels = y
    return prm, kp_mode, imax
