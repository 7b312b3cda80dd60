"""Sparse CG-trace cases: multi-iteration residual curves of every sparse K·p path
against the oracle, across the explicit-residual iteration (run % 50 == 49, OpenMP/csvm.cpp:119-132).

One seeded CSR set (1200 points x 300 features, 20 per row: most pairs share a feature, many share
several, so the kernel expansion's stored remainder H carries real weight), C = 10 (1000 for the fp32 rbf
cases, COST_CASE), imax = 60 and
eps = 1e-12 — below every fp32/fp64 CG's rounding floor, so every run (the reference's, the oracle's,
the HIP path's) takes exactly imax iterations and crosses the reset. Test infrastructure only (shared by
tests/golden/make_cg_trace_vectors.py and tests/test_gpu_cg_trace.py).
"""
import hashlib
import os

import numpy as np

from plssvm_sparse_fp22_amd import datagen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VECTORS = os.path.join(ROOT, "tests", "golden", "cg_traces")

N, D, K, SEED = 1200, 300, 20, 8
COST, IMAX, EPS = 10.0, 60, 1e-12
# the fp32 rbf cases (gamma 5e-4 for the bfloat16 bound: a nearly constant kernel) are too well conditioned at
# C = 10 — their recursive residual reaches 0 in fp32 after ~35-48 iterations. At C = 1000 their CG still moves
# after 60 iterations (delta / delta0 ~ 1e-12 at the reset), and eps = 1e-30 (eps^2 underflows to 0 in fp32:
# no stop) makes every run take exactly imax iterations across the reset.
EPS_CASE = {"rbf_f32_bf16_flags": 1e-30, "rbf_fp22_bf16_flags": 1e-30, "rbf_f32_realh": 1e-30}
COST_CASE = {"rbf_f32_bf16_flags": 1000.0, "rbf_fp22_bf16_flags": 1000.0, "rbf_f32_realh": 1000.0}

# name: kernel, real type, gamma, coef0, FP22 input, sparse algorithm, environment of the HIP run, layout checks
CASES = {
    # factored linear: the panelled SELL-64 passes (spmv.hpp), row-block CSR pass with the finalize fused
    "linear_f64": ("linear", np.float64, None, 0.0, False, "auto", {}, {}),
    "linear_f32": ("linear", np.float32, None, 0.0, False, "auto", {}, {}),
    # kernel expansion, real-typed H (fp64: exp_hbytes 8), indexed 4-slot chunks
    "rbf_f64_expansion": ("rbf", np.float64, 0.05, 0.0, False, "expansion", {}, {"exp_hbytes": 8}),
    "poly_f64_expansion": ("polynomial", np.float64, 0.05, 1.0, False, "expansion", {}, {"exp_hbytes": 8}),
    # kernel expansion in fp32 with bfloat16 H + flagged chunks (the layout of the 3-RBF / config-5 bench lines;
    # gamma small enough for the 2^-16 bound — up to ~6 shared features of |x| <= 1: max |H| / k = 6.6e-6 here;
    # the flags forced: few windows leave many empty cells here)
    "rbf_f32_bf16_flags": ("rbf", np.float32, 0.0005, 0.0, False, "expansion", {"PLSSVM_MI_EXP_ROWS": "flags"},
                           {"exp_hbytes": 2, "exp_layout": 2}),
    "rbf_fp22_bf16_flags": ("rbf", np.float32, 0.0005, 0.0, True, "expansion", {"PLSSVM_MI_EXP_ROWS": "flags"},
                            {"exp_hbytes": 2, "exp_layout": 2}),
    # the real-H fp32 layout (bound forced off)
    "rbf_f32_realh": ("rbf", np.float32, 0.0005, 0.0, False, "expansion", {"PLSSVM_MI_EXP_HFMT": "full"},
                      {"exp_hbytes": 4}),
    # the unstored paths
    "rbf_f64_onthefly": ("rbf", np.float64, 0.05, 0.0, False, "onthefly", {}, {}),
    "rbf_f64_densified": ("rbf", np.float64, 0.05, 0.0, False, "dense", {}, {}),
}


def build(name):
    """Returns dict(csr=(rowptr, col, val, n, d) in the case's real type (FP22: dequantised values),
    fp22=packed words or None, y, gamma, coef0, kernel, dtype)."""
    kernel, dtype, gamma, coef0, fp22, _, _, _ = CASES[name]
    (rowptr, col, val, n, d), y = datagen.sparse_csr(N, D, K, seed=SEED, dtype=np.float32 if dtype == np.float32
                                                     else np.float64)
    words = None
    if fp22:
        from plssvm_sparse_fp22_amd import fp22 as f22

        words = f22.pack(val)
        val = f22.unpack(words, val.size)
    dt = np.dtype(dtype).type
    g = dt(1.0) / dt(d) if gamma is None else dt(gamma)
    return dict(csr=(rowptr, col, val.astype(dtype), n, d), fp22=words, y=y.astype(dtype), gamma=g, coef0=dt(coef0),
                kernel=kernel, dtype=dtype, eps=EPS_CASE.get(name, EPS), cost=COST_CASE.get(name, COST))


def input_hash(s):
    h = hashlib.sha256()
    for a in s["csr"][:3]:
        h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.ascontiguousarray(s["y"]).tobytes())
    return h.hexdigest()


def q_explicit(s, with_abs=False):
    """The whole Q~ (m x m) in longdouble from float64 products of the case's values (csvm.cpp:230-258:
    k(x_i, x_j) + QA_cost - q_i - q_j + delta_ij / C). with_abs: also the matrix of the terms' magnitudes
    |k_ij| + |QA_cost| + |q_i| + |q_j| + delta_ij / C, which bounds the rounding of any evaluation order."""
    import scipy.sparse as sp

    rowptr, col, val, n, d = s["csr"]
    Xs = sp.csr_matrix((np.asarray(val, dtype=np.float64), col, rowptr), shape=(n, d))
    G = (Xs @ Xs.T).toarray().astype(np.longdouble)
    g, c0 = np.longdouble(float(s["gamma"])), np.longdouble(float(s["coef0"]))
    if s["kernel"] == "linear":
        Kf = G
    elif s["kernel"] == "polynomial":
        Kf = (g * G + c0) ** 3
    else:
        nrm = np.diag(G)
        Kf = np.exp(-g * (nrm[:, None] + nrm[None, :] - 2 * G))
    m = n - 1
    eye = np.eye(m, dtype=np.longdouble) / np.longdouble(s["cost"])
    qa = Kf[m, m] + np.longdouble(1.0 / s["cost"])
    Q = Kf[:m, :m] + qa - Kf[:m, m][:, None] - Kf[:m, m][None, :] + eye
    if not with_abs:
        return Q
    qv = np.abs(Kf[:m, m])
    return Q, np.abs(Kf[:m, :m]) + abs(qa) + qv[:, None] + qv[None, :] + eye


def trace_extended(s, Q=None):
    """learn()'s CG (x0 = 1, explicit residual every 50th iteration, OpenMP/csvm.cpp:82-170) in longdouble on
    the explicit Q~: where a fp32/fp64 trace leaves it, that CG has lost its orthogonality to rounding."""
    Q = q_explicit(s) if Q is None else Q
    m = Q.shape[0]
    yl = np.asarray(s["y"], dtype=np.longdouble)
    b = yl[:m] - yl[m]
    x = np.ones(m, dtype=np.longdouble)
    r = b - Q @ x
    dv = r.copy()
    delta = r @ r
    d0, tr = delta, [delta]
    for it in range(IMAX):
        Ad = Q @ dv
        a = delta / (dv @ Ad)
        x += a * dv
        r = b - Q @ x if it % 50 == 49 else r - a * Ad
        dn = r @ r
        tr.append(dn)
        if dn <= np.longdouble(s["eps"]) ** 2 * d0:
            break
        dv = dn / delta * dv + r
        delta = dn
    return np.array(tr, dtype=np.float64)
