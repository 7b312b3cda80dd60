"""GPU parity against the committed oracle golden vectors (tests/golden/oracle_vectors/, written by
tests/golden/make_oracle_vectors.py from the C oracle), through the C ABI.

Every {set} x {linear, polynomial, rbf} x {f32, f64}: the inputs are rebuilt from their seeded
recipe and checked against the recorded sha256 first; then q, QA_cost, Q~p for add = +1 / -1
(generate_q / run_device_kernel) and learn() (alpha, rho, the CG delta trace) are compared.
The FP22 set goes in as packed FP22 words in f32 contexts (the FP22 path) and as its dequantised
values in f64 contexts (FP22 input is float-only, include/plssvm_mi355x.h).

Tolerances: q and K·p <= 1e-12 (f64) / 1e-4 (f32) of max|.|. The CG checks use
the two references recorded with the vectors: the same learn() on 8 OpenMP threads (the
reference's own run-to-run spread: its atomics reorder the sums) and the same CG in extended
precision. On these systems (x0 = 1, C = 1: the first iterations remove 8-10 orders of magnitude of
residual) the reference's own fp64 trace leaves the extended-precision one after 2-5 iterations —
beyond that point every fp32/fp64 CG, the reference's included, follows its own rounding path. So:
  delta trace: on the prefix where the reference is accurate (within R of extended precision),
       the HIP trace is within R + 10 x (reference 1-vs-8-thread spread) of the reference, and the
       HIP trace stays accurate at least as long (minus one iteration); R = 1e-6 (f64, north_star),
       1e-3 (f32);
  solution (f64): the explicit residual |b - Q~ x|^2 of the HIP alphas, through the device K·p, is
       at most 10 x that of the reference's alphas (or of eps^2 delta_0);
  alpha: where the reference trace is accurate to the end, alphas within A * max|alpha| + 10 x the
       reference's 1-vs-8-thread spread, A = 1e-7 (f64) / 2e-2 (f32) (alpha_m = -sum alpha: sqrt(m) x).
"""
import json
import os

import numpy as np
import pytest

import golden_sets as gs
import plssvm_sparse_fp22_amd as pm

pytestmark = pytest.mark.gpu

MANIFEST = json.load(open(os.path.join(gs.VECTORS, "manifest.json")))
TOL = {"float64": 1e-12, "float32": 1e-4}


def make_svm(s, meta, dtype):
    p = pm.Parameter(meta["kernel"], degree=meta["degree"], gamma=meta["gamma"], coef0=meta["coef0"],
                     cost=meta["cost"], epsilon=meta["eps"], real_type=dtype)
    if s["kind"] == "dense":
        p.data = s["X"]
    elif s["fp22"] is not None and dtype == np.float32:
        rowptr, col, _, n, d = s["csr"]
        p.csr = (rowptr, col, s["fp22"], n, d)
        p.val_fmt = pm._abi.VAL_FP22
    else:
        p.csr = s["csr"]
    p.labels = s["y"]
    return pm.CSVM(p)


def close(got, want, tol, what):
    scale = max(float(np.abs(want).max()), 1e-300)
    np.testing.assert_allclose(got, want, rtol=0, atol=tol * scale, err_msg=what)


@pytest.mark.parametrize("key", sorted(MANIFEST))
def test_hip_matches_oracle_golden(key):
    meta = MANIFEST[key]
    dtype = np.dtype(meta["dtype"]).type
    s = gs.build(meta["set"], dtype)
    assert gs.input_hash(s) == meta["input_sha256"], "input recipe drifted from the committed vectors"
    g = np.load(os.path.join(gs.VECTORS, key + ".npz"))
    tol = TOL[meta["dtype"]]
    with make_svm(s, meta, dtype) as svm:
        svm.setup_data_on_device()
        q = svm.generate_q()
        close(q, g["q"], tol, f"{key}: q")
        assert abs(float(svm.QA_cost) - float(g["QA_cost"][0])) <= tol * max(1.0, abs(float(g["QA_cost"][0])))
        p = gs.p_vector(meta["n"] - 1, dtype)
        for tag, add in (("p1", 1.0), ("m1", -1.0)):
            ret = svm.run_device_kernel(None, np.zeros(meta["n"] - 1, dtype=dtype), p, add)
            close(ret, g[f"kp_add_{tag}"], tol, f"{key}: K·p add={add}")
        svm.learn(imax=meta["imax"])
        b = (s["y"][:-1] - s["y"][-1]).astype(dtype)
        check_cg(key, dtype, svm, g, b, meta["eps"])


def stable_prefix(t, ref, R):
    n = min(len(t), len(ref))
    bad = np.nonzero(np.abs(t[:n] / ref[:n] - 1) > R)[0]
    return int(bad[0]) if bad.size else n


def check_cg(key, dtype, svm, g, b, eps):
    R, A = (1e-6, 1e-7) if dtype == np.float64 else (1e-3, 2e-2)
    t1, t8, tld = g["trace"], g["trace_t8"], g["trace_ld"]
    ns = stable_prefix(t1, tld, R)
    assert ns >= 1 and len(svm.trace) >= ns, (key, ns, len(svm.trace))
    noise = np.maximum.accumulate(np.abs(t8[:ns] / t1[:ns] - 1))
    dev = np.abs(svm.trace[:ns] / t1[:ns] - 1)
    assert np.all(dev <= R + 10 * noise), (key, dev, noise)
    assert stable_prefix(svm.trace, tld, 2 * R) >= ns - 1, (key, svm.trace, tld, ns)
    if dtype == np.float64:
        def residual(alpha):
            r = b.copy()
            svm.run_device_kernel(None, r, alpha[:-1], -1.0)
            return float(r @ r)

        assert residual(svm.alpha) <= 10 * max(residual(g["alpha"]), eps * eps * t1[0]), key
    if ns == len(t1) == len(svm.trace):
        a1 = g["alpha"]
        tol = A * np.abs(a1).max() + 10 * np.abs(g["alpha_t8"] - a1).max()
        np.testing.assert_allclose(svm.alpha[:-1], a1[:-1], rtol=0, atol=tol, err_msg=f"{key}: alpha")
        # alpha_m = -sum(alpha): its error is a sum of m per-entry errors
        assert abs(svm.alpha[-1] - a1[-1]) <= np.sqrt(len(a1)) * tol, (key, svm.alpha[-1], a1[-1])
