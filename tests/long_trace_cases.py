"""Long CG-trace cases: residual curves compared with the OpenMP oracle over >= 60 iterations,
across the explicit-residual iteration run % 50 == 49 (OpenMP/csvm.cpp:113-160), on systems where the oracle
reproduces itself (1 vs 8 threads within 1e-9 relative) over the whole window.

Why the round-4 cases could not do this (tests/cg_trace_cases.py): there x0 = 1 starts the CG far out along the
top eigenvector of Q~, the first step removes 6-9 orders of magnitude of the residual, and every later iterate
carries the first step's rounding amplified by that factor; the 1-vs-8-thread traces separate after 3-5 iterations.
The systems here are built so that the curve is a smooth, slow descent that stays far above the rounding floor:

  * the last point (the one learn() eliminates, csvm.cpp:230-258) is the centroid of the others (here: the
    origin, every feature column has zero mean), so Q~ 1 carries no top-eigenvector component and r0 = b - Q~ 1
    is spread over the spectrum; labels are drawn independently of the features;
  * the Gram part has an EQUISPACED spectrum (no isolated extreme eigenvalues whose Ritz values converge early,
    which is where CG loses orthogonality and rounding starts to grow): dense sets are U diag(sigma) V^T with
    sigma^2 equispaced; sparse sets are row groups with disjoint feature blocks (each row dense in its group's
    features, the union of the groups' spectra equispaced), so pairs inside a group share every feature — the
    kernel expansion's stored remainder H carries real weight — and pairs across groups share none;
  * a condition number (kappa, C) for which 60-70 iterations reduce delta by 1e-2 .. 1e-5, not to the floor.

fp32: on data where the bfloat16 remainder bound holds (2 gamma |x|^2 <~ 4e-3) Q~'s entries are differences of
O(1) kernel values with an O(gamma |x|^2) result, so every fp32 evaluation loses ~log10(1 / (gamma |x|^2)) digits
per K·p — the oracle's own fp32 learn() leaves its fp64 curve by orders of magnitude within 3 iterations on every
such set (tests/golden/cg_traces_long/manifest.json: "f32_oracle_dev"). The fp32 cases therefore compare the HIP
curve with the fp64 oracle's; the manifest records how far the fp32 oracle itself strays.

Test infrastructure only (shared by tests/golden/make_long_trace_vectors.py and tests/test_gpu_cg_trace_long.py).
"""
import hashlib
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VECTORS = os.path.join(ROOT, "tests", "golden", "cg_traces_long")

N = 1200
IMAX = 70
EPS = 1e-30  # below every CG's floor, and eps^2 underflows in fp32: each run takes exactly IMAX iterations


def svd_set(n, d, seed, kappa):
    """Dense: rows 0..n-2 = U diag(sqrt(s2)) V^T (U orthonormal with zero column means, s2 equispaced in
    [1, kappa]), scaled to max |x| = 1; the last row is the origin = the centroid of the others."""
    rng = np.random.default_rng(seed)
    m = n - 1
    A = rng.standard_normal((m, d))
    A -= A.mean(axis=0)
    U, _ = np.linalg.qr(A)
    V, _ = np.linalg.qr(rng.standard_normal((d, d)))
    X = np.zeros((n, d))
    X[:m] = (U * np.sqrt(np.linspace(1.0, kappa, d))) @ V.T
    X /= np.abs(X).max()
    X = X.astype(np.float32).astype(np.float64)  # exact in both real types, 4 B per value in the fixture
    y = np.where(rng.random(n) < 0.5, -1.0, 1.0)
    return X, y


def group_set(n, d, fpg, seed, kappa):
    """Sparse: the n-1 rows in d // fpg groups, group g dense in its own fpg features (a zero-mean block with a
    prescribed spectrum; the union over the groups equispaced in [1/kappa, 1]), rows shuffled, max |x| = 1; the last
    row empty (the origin). Returns CSR (rowptr int64, col int32, val float64, n, d) and labels."""
    rng = np.random.default_rng(seed)
    m = n - 1
    G = d // fpg
    s2 = np.linspace(1.0 / kappa, 1.0, G * fpg)[rng.permutation(G * fpg)].reshape(G, fpg)
    bounds = np.linspace(0, m, G + 1).astype(int)
    X = np.zeros((n, d))
    for g in range(G):
        r0, r1 = bounds[g], bounds[g + 1]
        A = rng.standard_normal((r1 - r0, fpg))
        A -= A.mean(axis=0)
        U, _ = np.linalg.qr(A)
        V, _ = np.linalg.qr(rng.standard_normal((fpg, fpg)))
        X[r0:r1, g * fpg:(g + 1) * fpg] = (U * np.sqrt(s2[g])) @ V.T
    X /= np.abs(X).max()
    X[:m] = X[rng.permutation(m)]
    y = np.where(rng.random(n) < 0.5, -1.0, 1.0)
    nz = X != 0
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum(nz.sum(1))
    return (rowptr, np.nonzero(nz)[1].astype(np.int32), X[nz], n, d), y


# name: kernel, real type, data recipe, gamma rule, coef0, C, sparse algorithm, environment, layout checks.
# gamma rule ("dist", c): gamma = c / mean ||x_i - x_j||^2 (the kernel's curvature over the set);
#            ("x2", g2): 2 gamma max x^2 = g2 (the bfloat16 remainder bound's scale)
CASES = {
    # dense MFMA pairwise tiles (kp_tiles.hip), the configs[1] path
    "rbf_f64_dense": ("rbf", np.float64, ("svd", 256, 11, 1e4), ("dist", 0.01), 0.0, 1e5, "auto", {}, {}),
    "linear_f64_dense": ("linear", np.float64, ("svd", 256, 12, 1e4), None, 0.0, 87.0, "auto", {}, {}),
    # factored linear SELL-64 passes (spmv.hpp)
    "linear_f64_sparse": ("linear", np.float64, ("group", 300, 10, 13, 1e3), None, 0.0, 1e3, "auto", {}, {}),
    "linear_f32_sparse": ("linear", np.float32, ("group", 300, 10, 13, 1e3), None, 0.0, 1e3, "auto", {}, {}),
    # kernel expansion, real-typed H
    "rbf_f64_expansion": ("rbf", np.float64, ("group", 300, 10, 14, 1e3), ("dist", 0.01), 0.0, 3e4, "expansion", {},
                          {"exp_hbytes": 8, "centered": 1}),
    # kernel expansion in fp32, bfloat16 H, flagged chunks (the 3-RBF / config-5 layout)
    "rbf_f32_bf16_flags": ("rbf", np.float32, ("group", 300, 3, 15, 1e3), ("x2", 4e-3), 0.0, 1e6, "expansion",
                           {"PLSSVM_MI_EXP_ROWS": "flags"}, {"exp_hbytes": 2, "exp_layout": 2, "centered": 1}),
    # the same set and layout with pair flags (round 5: cells padded to 2 slots, expand.hip "pair flags")
    "rbf_f32_bf16_pairs": ("rbf", np.float32, ("group", 300, 3, 15, 1e3), ("x2", 4e-3), 0.0, 1e6, "expansion",
                           {"PLSSVM_MI_EXP_ROWS": "pairs"}, {"exp_hbytes": 2, "exp_layout": 4, "centered": 1}),
    # the same with 2 features per group (pairs share 2 features) and with 10 (gamma from the curvature rule)
    "rbf_f32_bf16_flags_b": ("rbf", np.float32, ("group", 300, 2, 16, 1e3), ("x2", 4e-3), 0.0, 1e6, "expansion",
                             {"PLSSVM_MI_EXP_ROWS": "flags"}, {"exp_hbytes": 2, "exp_layout": 2, "centered": 1}),
    "rbf_f32_bf16_flags_c": ("rbf", np.float32, ("group", 300, 10, 17, 1e3), ("dist", 0.001), 0.0, 1e6, "expansion",
                             {"PLSSVM_MI_EXP_ROWS": "flags"}, {"exp_hbytes": 2, "exp_layout": 2, "centered": 1}),
    # round 6: fp32 bfloat16 cases whose fp64 curve DESCENDS by 2-3 orders over the window (C = 3e5;
    # the C = 1e6 cases above descend by less than one, non-monotonically) while the oracle still reproduces itself
    "rbf_f32_bf16_desc": ("rbf", np.float32, ("group", 300, 10, 18, 1e3), ("dist", 0.001), 0.0, 3e5, "expansion",
                          {"PLSSVM_MI_EXP_ROWS": "flags"}, {"exp_hbytes": 2, "exp_layout": 2, "centered": 1}),
    "rbf_f32_bf16_desc_pairs": ("rbf", np.float32, ("group", 300, 3, 19, 1e3), ("x2", 4e-3), 0.0, 3e5, "expansion",
                                {"PLSSVM_MI_EXP_ROWS": "pairs"}, {"exp_hbytes": 2, "exp_layout": 4, "centered": 1}),
}


def build(name):
    kernel, dtype, recipe, grule, coef0, cost, _, _, _ = CASES[name]
    if recipe[0] == "svd":
        X, y = svd_set(N, recipe[1], recipe[2], recipe[3])
        csr = None
        nrm = (X ** 2).sum(1)
        vmax2 = float((X ** 2).max())
    else:
        csr, y = group_set(N, recipe[1], recipe[2], recipe[3], recipe[4])
        X = None
        rowptr, _, val, n, _ = csr
        nrm = np.bincount(np.repeat(np.arange(n), np.diff(rowptr)), weights=val ** 2, minlength=n)
        vmax2 = float((val ** 2).max())
    dt = np.dtype(dtype).type
    if grule is None:
        gamma = 0.0
    elif grule[0] == "dist":
        gamma = grule[1] / (2 * float(nrm.mean()))
    else:
        gamma = grule[1] / (2 * vmax2)
    s = dict(kernel=kernel, dtype=dtype, y=y.astype(dtype), gamma=dt(gamma), coef0=dt(coef0), cost=cost, eps=EPS)
    if X is not None:
        s["X"] = X.astype(dtype)
    else:
        s["csr"] = (csr[0], csr[1], csr[2].astype(dtype), csr[3], csr[4])
    return s


def load(name):
    """The case with its inputs read from the committed fixture (the GPU tests: LAPACK's QR inside the recipe need
    not give the same bits on another machine; tests/test_long_trace_vectors.py checks recipe == fixture here)."""
    kernel, dtype, _, _, _, cost, _, _, _ = CASES[name]
    g = np.load(os.path.join(VECTORS, name + ".npz"))
    dt = np.dtype(dtype).type
    s = dict(kernel=kernel, dtype=dtype, y=g["in_y"].astype(dtype), gamma=dt(g["in_gamma"][0]),
             coef0=dt(g["in_coef0"][0]), cost=cost, eps=EPS)
    if "in_X" in g:
        s["X"] = g["in_X"].astype(dtype)
    else:
        s["csr"] = (g["in_rowptr"], g["in_col"], g["in_val"].astype(dtype), N, int(g["in_d"][0]))
    return s


def input_arrays(s):
    a = dict(in_y=np.asarray(s["y"]), in_gamma=np.array([s["gamma"]]), in_coef0=np.array([s["coef0"]]))
    if "X" in s:
        a["in_X"] = np.asarray(s["X"], np.float32)
    else:
        a.update(in_rowptr=s["csr"][0], in_col=s["csr"][1], in_val=np.asarray(s["csr"][2]),
                 in_d=np.array([s["csr"][4]]))
    return a


def input_hash(s):
    h = hashlib.sha256()
    for a in ([s["X"]] if "X" in s else s["csr"][:3]):
        h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.ascontiguousarray(s["y"]).tobytes())
    return h.hexdigest()


def dense_of(s):
    if "X" in s:
        return np.asarray(s["X"], np.float64)
    import scipy.sparse as sp

    rowptr, col, val, n, d = s["csr"]
    return sp.csr_matrix((np.asarray(val, np.float64), col, rowptr), shape=(n, d)).toarray()


def q_explicit(s):
    """Q~ (m x m, longdouble) from float64 products of the case's values (csvm.cpp:230-258)."""
    X = dense_of(s)
    G = (X @ X.T).astype(np.longdouble)
    g, c0 = np.longdouble(float(s["gamma"])), np.longdouble(float(s["coef0"]))
    if s["kernel"] == "linear":
        Kf = G
    elif s["kernel"] == "polynomial":
        Kf = (g * G + c0) ** 3
    else:
        nrm = np.diag(G)
        Kf = np.exp(-g * (nrm[:, None] + nrm[None, :] - 2 * G))
    m = X.shape[0] - 1
    qa = Kf[m, m] + np.longdouble(1.0 / s["cost"])
    return Kf[:m, :m] + qa - Kf[:m, m][:, None] - Kf[:m, m][None, :] + np.eye(m, dtype=np.longdouble) / np.longdouble(
        s["cost"])


def trace_extended(s):
    """learn()'s CG (x0 = 1, r = b - Q~x explicitly when run % 50 == 49, OpenMP/csvm.cpp:82-170) in longdouble."""
    Q = q_explicit(s)
    m = Q.shape[0]
    yl = np.asarray(s["y"], dtype=np.longdouble)
    b = yl[:m] - yl[m]
    x = np.ones(m, dtype=np.longdouble)
    r = b - Q @ x
    dv = r.copy()
    delta = r @ r
    tr = [delta]
    for it in range(IMAX):
        Ad = Q @ dv
        a = delta / (dv @ Ad)
        x += a * dv
        r = b - Q @ x if it % 50 == 49 else r - a * Ad
        dn = r @ r
        tr.append(dn)
        dv = dn / delta * dv + r
        delta = dn
    return np.array(tr, dtype=np.float64)
