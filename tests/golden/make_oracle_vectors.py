#!/usr/bin/env python3
"""Generates tests/golden/oracle_vectors/ with the C oracle (oracle/: the reference OpenMP path
restated, pinned by the reference fixtures in tests/test_oracle.py). Test infrastructure only.

For every set of tests/golden_sets.py x {linear, polynomial, rbf} x {f32, f64} it records
  q, QA_cost                  generate_q + QA_cost (csvm.cpp:230-245)
  kp_add_p1, kp_add_m1        ret = 0 + add * Q~ p for p ~ U(1, 2) (seed 5), add = +1 / -1
  alpha, rho, trace, iters    learn() with C = 1, eps = 1e-6 (tighter than the reference default 1e-3,
                              so the delta trace runs more iterations), imax = min(num_features, 64)
  alpha_t8, trace_t8, iters_t8  the same learn() on 8 OpenMP threads: the reference's own run-to-run
                              spread (its atomics reorder the sums), the noise floor of the CG checks
  trace_ld                    the same CG in extended precision (numpy longdouble on the explicit Q~):
                              where the reference's fp32/fp64 trace leaves it, the reference itself has
                              lost the CG's orthogonality and later entries are rounding-path dependent
in <set>__<kernel>__<f32|f64>.npz (plain arrays, no pickles), and manifest.json with the
parameters and a sha256 of each input. The oracle runs single-threaded, so the vectors are
deterministic (its OpenMP atomics make multi-threaded sums order-dependent).

usage (build container, ~1 minute): python tests/golden/make_oracle_vectors.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import golden_sets as gs  # noqa: E402
from oracle import pyoracle  # noqa: E402


def oracle_data(s, dtype):
    if s["kind"] == "dense":
        return pyoracle.Data(s["X"], dtype=dtype)
    rowptr, col, val, n, d = s["csr"]
    return pyoracle.Data(rowptr=rowptr, col=col, val=val, n=n, d=d, dtype=dtype)


def trace_extended(s, kernel, args, y, imax, eps):
    """CG of learn() (x0 = 1, explicit residual every 50th iteration) in longdouble on the explicit
    Q~ (K from float64 products: its rounding is far below the CG's own amplification)."""
    if s["kind"] == "dense":
        X = np.asarray(s["X"], dtype=np.float64)
        G = X @ X.T
    else:
        import scipy.sparse as sp

        rowptr, col, val, n, d = s["csr"]
        Xs = sp.csr_matrix((np.asarray(val, dtype=np.float64), col, rowptr), shape=(n, d))
        G = (Xs @ Xs.T).toarray()
    G = G.astype(np.longdouble)
    g, c0 = np.longdouble(args["gamma"]), np.longdouble(args["coef0"])
    if kernel == "linear":
        Kf = G
    elif kernel == "polynomial":
        Kf = (g * G + c0) ** args["degree"]
    else:
        nrm = np.diag(G)
        Kf = np.exp(-g * (nrm[:, None] + nrm[None, :] - 2 * G))
    m = G.shape[0] - 1
    Q = Kf[:m, :m] + (Kf[m, m] + 1) - Kf[:m, m][:, None] - Kf[:m, m][None, :] + np.eye(m, dtype=np.longdouble)
    yl = np.asarray(y, dtype=np.longdouble)
    b = yl[:m] - yl[m]
    x = np.ones(m, dtype=np.longdouble)
    r = b - Q @ x
    dv = r.copy()
    delta = r @ r
    d0, tr = delta, [delta]
    for it in range(imax):
        Ad = Q @ dv
        a = delta / (dv @ Ad)
        x += a * dv
        r = b - Q @ x if it % 50 == 49 else r - a * Ad
        dn = r @ r
        tr.append(dn)
        if dn <= np.longdouble(eps) ** 2 * d0:
            break
        dv = dn / delta * dv + r
        delta = dn
    return np.array(tr, dtype=np.float64)


def vectors(name, kernel, dtype):
    s = gs.build(name, dtype)
    data = oracle_data(s, dtype)
    args = gs.params(s, kernel, dtype)
    imax = min(s["d"], gs.IMAX_CAP)
    ref = pyoracle.learn(kernel, data, s["y"], cost=1.0, eps=gs.EPS, imax=imax, nthreads=1, **args)
    ref8 = pyoracle.learn(kernel, data, s["y"], cost=1.0, eps=gs.EPS, imax=imax, nthreads=8, **args)
    q = pyoracle.generate_q(kernel, data, **args)
    m = s["n"] - 1
    p = gs.p_vector(m, dtype)
    kp = {}
    for tag, add in (("p1", 1.0), ("m1", -1.0)):
        kp[tag] = pyoracle.kp(kernel, data, q, ref["QA_cost"], 1.0, add, p, nthreads=1, **args)
    arrays = dict(q=q, QA_cost=np.array([ref["QA_cost"]], dtype=dtype), kp_add_p1=kp["p1"], kp_add_m1=kp["m1"],
                  alpha=ref["alpha"], rho=np.array([ref["rho"]], dtype=dtype), trace=ref["trace"],
                  iters=np.array([ref["iters"]], dtype=np.int64), alpha_t8=ref8["alpha"], trace_t8=ref8["trace"],
                  iters_t8=np.array([ref8["iters"]], dtype=np.int64),
                  trace_ld=trace_extended(s, kernel, args, s["y"], imax, gs.EPS))
    meta = dict(set=name, kernel=kernel, dtype=np.dtype(dtype).name, n=int(s["n"]), d=int(s["d"]),
                layout=s["kind"] if s["fp22"] is None else "fp22", degree=args["degree"],
                gamma=float(args["gamma"]), coef0=float(args["coef0"]), cost=1.0, eps=gs.EPS, imax=imax,
                p_seed=gs.P_SEED, input_sha256=gs.input_hash(s), iters=int(ref["iters"]))
    return arrays, meta


def main():
    pyoracle.build()
    os.makedirs(gs.VECTORS, exist_ok=True)
    manifest = {}
    for name in gs.SETS:
        for kernel in gs.KERNELS:
            for tag, dtype in gs.DTYPES.items():
                k = gs.key(name, kernel, tag)
                arrays, meta = vectors(name, kernel, dtype)
                np.savez_compressed(os.path.join(gs.VECTORS, k + ".npz"), **arrays)
                manifest[k] = meta
                print(k, "iters", meta["iters"], flush=True)
    with open(os.path.join(gs.VECTORS, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
