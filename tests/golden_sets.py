"""The input sets of the committed oracle golden vectors (tests/golden/oracle_vectors/).

SURVEY.md §8(c): {config-1 500x4 blobs, 5x4, 500x200, 3000x64 blobs, 2000x5000 CSR @ 1 %, the same
FP22-dequantised} x {linear, polynomial (degree 3, gamma 1/d, coef0 0), rbf (gamma 1/d)} x
{fp32, fp64}. Every set is rebuilt from a seeded recipe (or a reference fixture file); the manifest
records a sha256 of the inputs so a drifting generator is caught before any comparison.
Test infrastructure only (shared by tests/golden/make_oracle_vectors.py and the golden tests).
"""
import hashlib
import os

import numpy as np

import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIXTURES = os.path.join(ROOT, "tests", "golden", "reference_fixtures")
VECTORS = os.path.join(ROOT, "tests", "golden", "oracle_vectors")

SETS = ["config1_500x4", "5x4", "500x200", "blobs_3000x64", "csr_2000x5000", "fp22_2000x5000"]
KERNELS = ["linear", "polynomial", "rbf"]
DTYPES = {"f32": np.float32, "f64": np.float64}
P_SEED = 5  # p ~ U(1, 2) for the K·p vectors
IMAX_CAP = 64  # learn(): imax = min(num_features, 64) (5000 CG iterations of the oracle are too slow)
EPS = 1e-6  # learn(): tighter than the reference default 1e-3 (more CG iterations), far above rounding noise


def build(name, dtype):
    """Returns dict(kind='dense'|'csr', X | csr, y, n, d, fp22: packed words or None)."""
    if name == "config1_500x4":
        X, y = datagen.blobs(500, 4, seed=1, dtype=dtype)
        return dict(kind="dense", X=X, y=y, n=500, d=4, fp22=None)
    if name in ("5x4", "500x200"):
        X, y = pm.parse_libsvm(os.path.join(FIXTURES, f"{name}.libsvm"), dtype=dtype)
        return dict(kind="dense", X=np.ascontiguousarray(X), y=y, n=X.shape[0], d=X.shape[1], fp22=None)
    if name == "blobs_3000x64":
        X, y = datagen.blobs(3000, 64, seed=7, dtype=dtype)
        return dict(kind="dense", X=X, y=y, n=3000, d=64, fp22=None)
    if name in ("csr_2000x5000", "fp22_2000x5000"):
        (rowptr, col, val, n, d), y = datagen.sparse_csr(2000, 5000, 50, seed=9, dtype=np.float32)
        words = None
        if name.startswith("fp22"):
            from plssvm_sparse_fp22_amd import fp22

            words = fp22.pack(val)
            val = fp22.unpack(words, val.size)
        return dict(kind="csr", csr=(rowptr, col, val.astype(dtype), n, d), y=y.astype(dtype), n=n, d=d,
                    fp22=words)
    raise KeyError(name)


def input_hash(s):
    h = hashlib.sha256()
    if s["kind"] == "dense":
        h.update(np.ascontiguousarray(s["X"]).tobytes())
    else:
        for a in s["csr"][:3]:
            h.update(np.ascontiguousarray(a).tobytes())
    h.update(np.ascontiguousarray(s["y"]).tobytes())
    return h.hexdigest()


def params(s, kernel, dtype):
    dt = np.dtype(dtype).type
    return dict(degree=3, gamma=dt(1.0) / dt(s["d"]), coef0=dt(0.0))


def p_vector(m, dtype):
    return np.random.default_rng(P_SEED).uniform(1.0, 2.0, m).astype(dtype)


def key(name, kernel, tag):
    return f"{name}__{kernel}__{tag}"
