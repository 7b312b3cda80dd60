"""Full-size parity ("full-size parity of configs 2-5 is row-sampled"): one K·p
of the HIP path at the BASELINE sizes, the bench's own synthetic data (bench.make_problem), against
an exact float64 recomputation of 256 random rows of Q~p on the CPU:

    (Q~p)_i = sum_j k(x_i, x_j) p_j + (QA_cost - q_i) sum_j p_j - sum_j q_j p_j + p_i / C

(all j < m = N - 1, q_j = k(x_j, x_m), QA_cost = k(x_m, x_m) + 1/C). Tolerance: 1e-12 (fp64) /
1e-4 (fp32) of the row's sum of |terms| (the same bar as the small-size tests).
Config 5 (2M x 100k FP22 RBF, FP22 input) runs at its full size on one GPU: the kernel expansion
stores O(nnz + multi-feature pairs), 1.37e9 remainder slots, where the Gram pattern needed eight
GPUs. Its 2M geometry (row blocks of 7,824 rows, windows of 32,768 partners, 15.6 % slot padding)
differs from the N = 400k set (same column occupancy, d = 20k), which stays as a second case.
"""
import numpy as np
import pytest
import scipy.sparse as sp

import bench
import plssvm_sparse_fp22_amd as pm

pytestmark = pytest.mark.gpu

ROWS = 256
CASES = [("dense_rbf_100k", None), ("csr_linear_1m", None), ("csr_rbf_1m", None), ("dense_linear_500k", None),
         ("fp22_rbf_2m", None),
         ("fp22_rbf_2m", 400_000)]


def kernel_rows(kernel, G, ni, nj, gamma, degree=3, coef0=0.0):
    if kernel == "linear":
        return G
    if kernel == "polynomial":
        return (gamma * G + coef0) ** degree
    return np.exp(-gamma * (ni[:, None] + nj[None, :] - 2.0 * G))


@pytest.mark.parametrize("config,points", CASES)
def test_full_size_row_sampled(config, points):
    cfg = bench.CONFIGS[config]
    kernel, dtype = cfg[0], cfg[3]
    p, n, d, y, extra = bench.make_problem(cfg, points, None, 0)
    m = n - 1
    rng = np.random.default_rng(11)
    pv = rng.uniform(1.0, 2.0, m).astype(dtype)
    rows = np.sort(rng.choice(m, ROWS, replace=False))
    with pm.CSVM(p) as svm:
        svm.setup_data_on_device()
        svm.generate_q()
        ret = svm.run_device_kernel(None, np.zeros(m, dtype=dtype), pv, 1.0)[rows].astype(np.float64)
    gamma = 1.0 / d
    p64 = pv.astype(np.float64)
    def q_and_kmm(g_last, n_last):
        if kernel == "linear":
            return g_last, n_last
        if kernel == "polynomial":
            return (gamma * g_last) ** 3, (gamma * n_last) ** 3
        return np.exp(-gamma * (nrm[:m] + n_last - 2.0 * g_last)), 1.0

    if "X" in extra:
        X = extra["X"].astype(np.float64)
        nrm = np.einsum("ij,ij->i", X, X)
        q, kmm = q_and_kmm(X[:m] @ X[m], nrm[m])
        if kernel == "linear":  # sum_j k_ij p_j = x_i . (X_m^T p), exact enough in float64
            ksum = X[rows] @ (X[:m].T @ p64)
            kabs = np.abs(X[rows]) @ (np.abs(X[:m]).T @ p64)
        else:
            Kr = kernel_rows(kernel, X[rows] @ X[:m].T, nrm[rows], nrm[:m], gamma)
            ksum, kabs = Kr @ p64, np.abs(Kr) @ p64
    else:
        rowptr, col, val, _, _ = extra["csr"]
        if p.val_fmt == pm._abi.VAL_FP22:  # the device sees the FP22-rounded values
            from plssvm_sparse_fp22_amd import fp22

            val = fp22.unpack(p.csr[2], val.size)
        Xs = sp.csr_matrix((val.astype(np.float64), col, rowptr), shape=(n, d))
        nrm = np.asarray(Xs.multiply(Xs).sum(axis=1)).ravel()
        q, kmm = q_and_kmm(Xs[:m] @ Xs[m].toarray().ravel(), nrm[m])
        if kernel == "linear":
            ksum = Xs[rows] @ (Xs[:m].T @ p64)
            kabs = abs(Xs[rows]) @ (abs(Xs[:m]).T @ p64)
        else:
            ksum, kabs = np.zeros(ROWS), np.zeros(ROWS)
            XmT = Xs[:m].T.tocsc()
            for a in range(0, ROWS, 32):  # 32 rows x m columns at a time
                G = (Xs[rows[a:a + 32]] @ XmT).toarray()
                Kr = kernel_rows(kernel, G, nrm[rows[a:a + 32]], nrm[:m], gamma)
                ksum[a:a + 32], kabs[a:a + 32] = Kr @ p64, np.abs(Kr) @ p64
    QA = kmm + 1.0
    sp_, sqp = p64.sum(), q @ p64
    want = ksum + (QA - q[rows]) * sp_ - sqp + p64[rows]
    scale = kabs + np.abs(QA - q[rows]) * sp_ + np.abs(q) @ p64 + p64[rows]
    tol = 1e-12 if dtype == np.float64 else 1e-4
    err = np.abs(ret - want) / scale
    assert err.max() <= tol, (config, float(err.max()), rows[np.argmax(err)])
