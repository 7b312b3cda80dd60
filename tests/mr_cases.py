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
    "sparse_f32_rbf_hfmt_split": ("csr", "rbf", "auto", np.float32, 10),
}
# sparse poly / rbf K·p algorithm per case (default: auto)
ALGO = {"sparse_rbf_onthefly": "onthefly", "sparse_poly_onthefly": "onthefly"}
# per-rank device-memory budgets (PLSSVM_MI_MEM_BUDGET, bytes): the ranks' own estimates straddle the
# budget — rank 0 would store the kernel expansion, rank 1 cannot — so only a group-wide decision keeps
# both on one path
BUDGET = {"sparse_rbf_budget_split": {1: "1"}}
# rows given LONG_ROW entries (beyond the row join's 256-entry LDS copy): the rank holding them builds its
# remainder by the column-join sort, which measures no bfloat16 bound, while the other rank's rows pass it —
# only a group-wide H storage keeps the sharded K·p's collectives identical on both ranks
LONG_ROWS = {"sparse_f32_rbf_hfmt_split": [5000]}
LONG_ROW = 300
# cases whose K·p stores no pairs (on the fly / densified)
UNSTORED = set(ALGO) | set(BUDGET)


def case_data(name):
    layout, kernel, kp_mode, dtype, imax = CASES[name]
    if layout == "dense":
        X, y = datagen.blobs(3000, 64, seed=3, cluster_std=4.0, dtype=dtype)
        return dict(X=X), y, 64
    csr, y = datagen.sparse_csr(6500, 5000, 20, seed=2, dtype=dtype)
    for i in LONG_ROWS.get(name, []):
        csr = _long_row(csr, i, LONG_ROW)
    return dict(csr=csr), y, csr[4]


def _long_row(csr, i, k):
    """csr with row i replaced by k seeded entries (ascending distinct features, values in the set's range)."""
    rowptr, col, val, n, d = csr
    rng = np.random.default_rng(1000 + i)
    c = np.sort(rng.choice(d, size=k, replace=False)).astype(col.dtype)
    v = rng.uniform(0.1, 1.0, k).astype(val.dtype)
    a, b = int(rowptr[i]), int(rowptr[i + 1])
    col2 = np.concatenate([col[:a], c, col[b:]])
    val2 = np.concatenate([val[:a], v, val[b:]])
    rp = rowptr.copy()
    rp[i + 1:] += k - (b - a)
    return rp, col2, val2, n, d


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
