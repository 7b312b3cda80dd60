#!/usr/bin/env python3
"""Sparse RBF at 1 % density: the stored structures cannot fit, auto must fall back to
the densified MFMA path and produce a correct K·p (no OOM).

N x d = 200k x 50k (config 3's width) at 1 % = 500 features per row, fp32, gamma = 1/d: ~90 % of the
pairs share two or more features, so the kernel expansion's remainder and the Gram pattern would both
be ~all 2e10 pairs (terabytes); X densified is 40 GB. One K·p on sampled rows against a float64
recomputation (tolerance 1e-4 of sum |k_ij p_j|, the fp32 bar). Prints one JSON line.
usage: python tools/density_1pct.py [N] [d] [k]
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
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 50_000
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 500
    rng = np.random.default_rng(12)
    t0 = time.time()
    col = np.empty((n, k), dtype=np.int32)
    for i in range(n):
        col[i] = np.sort(rng.choice(d, k, replace=False))
    val = rng.uniform(-1.0, 1.0, (n, k)).astype(np.float32)
    rowptr = np.arange(0, (n + 1) * k, k, dtype=np.int64)
    col, val = col.reshape(-1), val.reshape(-1)
    gen_s = time.time() - t0
    prm = pm.Parameter("rbf", gamma=1.0 / d, real_type=np.float32)
    prm.csr = (rowptr, col, val, n, d)
    m = n - 1
    p = rng.uniform(1.0, 2.0, m).astype(np.float32)
    with pm.CSVM(prm) as svm:
        t0 = time.time()
        svm.setup_data_on_device()
        setup_s = time.time() - t0
        info = svm.info()
        t0 = time.time()
        got = svm.kp_part(p, "kernel")
        kp_s = time.time() - t0
    rows = np.sort(rng.choice(m, 64, replace=False))
    X = sp.csr_matrix((val.astype(np.float64), col, rowptr), shape=(n, d))
    nrm = np.asarray(X.multiply(X).sum(axis=1)).ravel()
    G = (X[rows] @ X[:m].T).toarray()
    K = np.exp(-(1.0 / d) * np.maximum(nrm[rows, None] + nrm[None, :m] - 2.0 * G, 0.0))
    want = K @ p.astype(np.float64)
    scale = K @ np.abs(p.astype(np.float64))
    err = float(np.max(np.abs(got[rows] - want) / scale))
    out = {"N": n, "d": d, "nnz_per_row": k, "density": k / d, "sparse_algo": info["sparse_algo"],
           "sparse_algo_name": {1: "pattern", 2: "expansion", 3: "densified"}.get(info["sparse_algo"]),
           "device_bytes": info.get("device_bytes"), "gen_s": round(gen_s, 1), "setup_s": round(setup_s, 1),
           "kp_s": round(kp_s, 2), "kp_tflops_fp32": 2.0 * d * m * (m + 1) / 2 / kp_s / 1e12,
           "max_rel_err": err, "tol": 1e-4, "ok": bool(err <= 1e-4 and info["sparse_algo"] == 3)}
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
