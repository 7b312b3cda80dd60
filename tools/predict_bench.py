#!/usr/bin/env python3
"""predict / update_w throughput on BASELINE-shaped models (SURVEY §8(f)2 measurement; run on the GPU box).

* dense RBF, config 2's model: 100k support vectors x 256 fp64, 100k predict points: the GEMM
  G = X Z^T (2 d n np FLOP) on rocBLAS + the kernel/alpha epilogue; reported against the fp64 MFMA peak;
* sparse RBF, config 3-RBF's model: 1M support vectors x 50k CSR fp32 (5e7 entries), 4096 CSR points:
  through the kernel expansion (the model's column moments once, then per point its features' moment
  sums and the support vectors sharing two or more features with it), beside the brute-force kernel
  (every support vector entry gathered per 64 points, PLSSVM_MI_PRED_BRUTE);
* linear update_w on config 3 (the SELL CSC pass, w = sum alpha_i x_i).
Times include the host transfers of the points and results (the C ABI takes host buffers); alpha is
random (the model's alphas do not change the work). Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import plssvm_sparse_fp22_amd as pm  # noqa: E402
from plssvm_sparse_fp22_amd import datagen  # noqa: E402


def timed(fn, reps=3):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    return (time.perf_counter() - t0) / reps, out


def main():
    res = {}
    rng = np.random.default_rng(7)
    # dense RBF (config 2 model)
    n, d, npts = 100_000, 256, 100_000
    X, y = datagen.blobs(n, d, seed=2)
    Z, _ = datagen.blobs(npts, d, seed=9)
    p = pm.Parameter("rbf", gamma=1.0 / d, real_type=np.float64)
    p.data, p.labels = X, y
    with pm.CSVM(p) as svm:
        svm.setup_data_on_device()
        alpha = rng.standard_normal(n)
        s, _ = timed(lambda: svm.predict_values(Z, alpha=alpha, bias=0.1))
    flop = 2.0 * d * n * npts
    res["dense_rbf_100k"] = {"support_vectors": n, "d": d, "points": npts, "dtype": "f64", "seconds": s,
                             "points_per_s": npts / s, "gemm_TFLOPs": flop / s / 1e12,
                             "frac_of_fp64_mfma_peak": flop / s / 78.6e12}
    # sparse RBF (config 3-RBF model) and linear update_w (config 3)
    n, d, k, npts = 1_000_000, 50_000, 50, 4096
    csr, y = datagen.sparse_csr(n, d, k, seed=3, dtype=np.float32)
    zc, _ = datagen.sparse_csr(npts, d, k, seed=11, dtype=np.float32)
    for kern in ("rbf", "linear"):
        p = pm.Parameter(kern, gamma=1.0 / d, real_type=np.float32)
        p.csr, p.labels = csr, y
        with pm.CSVM(p) as svm:
            svm.setup_data_on_device()
            alpha = rng.standard_normal(n).astype(np.float32)
            if kern == "rbf":
                s, _ = timed(lambda: svm.predict_values(zc, alpha=alpha, bias=0.1), reps=3)
                os.environ["PLSSVM_MI_PRED_BRUTE"] = "1"
                sb, _ = timed(lambda: svm.predict_values(zc, alpha=alpha, bias=0.1), reps=1)
                del os.environ["PLSSVM_MI_PRED_BRUTE"]
                nnz = int(csr[0][-1])
                res["csr_rbf_1m"] = {"support_vectors": n, "d": d, "nnz": nnz, "points": npts, "dtype": "f32",
                                     "path": "kernel expansion (moments + multi-feature partners per point)",
                                     "seconds": s, "points_per_s": npts / s,
                                     "brute_force_seconds": sb, "brute_force_points_per_s": npts / sb}
            else:
                s, _ = timed(lambda: svm.update_w(alpha), reps=5)
                nnz = int(csr[0][-1])
                res["csr_linear_1m_update_w"] = {"nnz": nnz, "seconds": s, "GBps_incl_host_copies": nnz * 6.0 / s / 1e9}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
