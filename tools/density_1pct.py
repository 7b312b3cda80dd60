#!/usr/bin/env python3
"""Sparse RBF at 1 % density: the stored structures cannot fit, auto must fall back to
the densified MFMA path and produce a correct K·p (no OOM).

N x d = 200k x 50k (config 3's width) at 1 % = 500 features per row, fp32, gamma = 1/d: ~90 % of the
pairs share two or more features, so the kernel expansion's remainder and the Gram pattern would both
be ~all 2e10 pairs (terabytes); X densified is 40 GB. One K·p on sampled rows against a float64
recomputation (tolerance 1e-4 of sum |k_ij p_j|, the fp32 bar). Prints one JSON line.
With the on-the-fly path (PLSSVM_MI_SPARSE_ONTHEFLY) auto picks it instead of the densified tiles when its
estimate is lower; --algo forces one (auto | onthefly | dense).
usage: python tools/density_1pct.py [N] [d] [k] [--algo A] [--dtype f32|f64] [--reps R]
"""
import json
import os
import sys
import time

import numpy as np
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import plssvm_sparse_fp22_amd as pm  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("n", type=int, nargs="?", default=200_000)
    ap.add_argument("d", type=int, nargs="?", default=50_000)
    ap.add_argument("k", type=int, nargs="?", default=500)
    ap.add_argument("--algo", default="auto", choices=["auto", "onthefly", "dense"])
    ap.add_argument("--dtype", default="f32", choices=["f32", "f64"])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--kernel", default="rbf", choices=["rbf", "polynomial"])
    a = ap.parse_args()
    n, d, k = a.n, a.d, a.k
    dt = np.float32 if a.dtype == "f32" else np.float64
    rng = np.random.default_rng(12)
    t0 = time.time()
    col = np.empty((n, k), dtype=np.int32)
    for i in range(n):
        col[i] = np.sort(rng.choice(d, k, replace=False))
    val = rng.uniform(-1.0, 1.0, (n, k)).astype(dt)
    rowptr = np.arange(0, (n + 1) * k, k, dtype=np.int64)
    col, val = col.reshape(-1), val.reshape(-1)
    gen_s = time.time() - t0
    prm = pm.Parameter(a.kernel, gamma=1.0 / d, coef0=1.0, real_type=dt)
    prm.csr = (rowptr, col, val, n, d)
    m = n - 1
    p = rng.uniform(1.0, 2.0, m).astype(dt)
    with pm.CSVM(prm, sparse_algo=a.algo) as svm:
        t0 = time.time()
        svm.setup_data_on_device()
        setup_s = time.time() - t0
        info = svm.info()
        got = svm.kp_part(p, "kernel")
        t0 = time.time()
        for _ in range(a.reps):
            got2 = svm.kp_part(p, "kernel")
        kp_s = (time.time() - t0) / a.reps
        assert np.array_equal(got, got2), "K·p not bitwise reproducible"
    rows = np.sort(rng.choice(m, 64, replace=False))
    X = sp.csr_matrix((val.astype(np.float64), col, rowptr), shape=(n, d))
    nrm = np.asarray(X.multiply(X).sum(axis=1)).ravel()
    G = (X[rows] @ X[:m].T).toarray()
    if a.kernel == "rbf":
        K = np.exp(-(1.0 / d) * np.maximum(nrm[rows, None] + nrm[None, :m] - 2.0 * G, 0.0))
    else:
        K = ((1.0 / d) * G + 1.0) ** 3
    want = K @ p.astype(np.float64)
    scale = K @ np.abs(p.astype(np.float64))
    err = float(np.max(np.abs(got[rows] - want) / scale))
    tol = 1e-4 if dt == np.float32 else 1e-12
    out = {"N": n, "d": d, "nnz_per_row": k, "density": k / d, "dtype": a.dtype, "kernel": a.kernel,
           "sparse_algo": info["sparse_algo"],
           "sparse_algo_name": {1: "pattern", 2: "expansion", 3: "densified", 4: "onthefly"}.get(info["sparse_algo"]),
           "device_bytes": info.get("device_bytes"), "gen_s": round(gen_s, 1), "setup_s": round(setup_s, 1),
           "kp_s": round(kp_s, 4), "dense_equiv_tflops": 2.0 * d * m * (m + 1) / 2 / kp_s / 1e12,
           "max_rel_err": err, "tol": tol, "ok": bool(err <= tol and info["sparse_algo"] in (3, 4))}
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
