"""GPU parity of update_w / predict (gpu_csvm::update_w / predict, src/plssvm/backends/gpu_csvm.cpp:52-127,
327-350) against the reference's own predict fixtures and the oracle's predict restatement
(openmp::csvm::predict, src/plssvm/backends/OpenMP/csvm.cpp:174-240).

Fixture: tests/data/models/500x200.libsvm.{linear,polynomial,rbf}.model applied to
tests/data/libsvm/500x200.libsvm.test must give tests/data/predict/500x200.libsvm.predict.
Tolerances: fp64 decision values 1e-10 relative to max|value| (rocBLAS / LDS dot-product order vs
the oracle's sequential fma chains), fp32 1e-4.
"""
import numpy as np
import pytest

from conftest import fixture_path
import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen, parse_libsvm, parse_model

pytestmark = pytest.mark.gpu

TOL = {np.float64: 1e-10, np.float32: 1e-4}


def model_svm(model, d, dtype=np.float64, sparse=False):
    SV = model["SV"]
    if SV.shape[1] < d:
        SV = np.pad(SV, ((0, 0), (0, d - SV.shape[1])))
    p = pm.Parameter(model["kernel"], degree=model.get("degree", 3), gamma=model.get("gamma", 1.0 / d),
                     coef0=model.get("coef0", 0.0), real_type=dtype)
    if sparse:
        p.csr = dense_to_csr(SV.astype(dtype))
    else:
        p.data = SV.astype(dtype)
    return pm.CSVM(p), SV


def dense_to_csr(X):
    rowptr = np.concatenate([[0], np.cumsum((X != 0).sum(axis=1))]).astype(np.int64)
    rr, cc = np.nonzero(X)
    return rowptr, cc.astype(np.int32), X[rr, cc], X.shape[0], X.shape[1]


@pytest.mark.parametrize("sparse", [False, True])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_predict_reference_fixture(oracle, kernel, sparse):
    Z, _ = parse_libsvm(fixture_path("500x200.libsvm.test"))
    expected = np.loadtxt(fixture_path("500x200.libsvm.predict"))
    model = parse_model(fixture_path(f"500x200.libsvm.{kernel}.model"))
    svm, SV = model_svm(model, Z.shape[1], sparse=sparse)
    points = dense_to_csr(Z) if sparse else Z
    vals = svm.predict_values(points, alpha=model["alpha"], bias=-model["rho"])
    assert np.array_equal(np.where(vals > 0, 1.0, -1.0), expected)
    ref = oracle.predict(kernel, SV, model["alpha"], model["rho"], Z, degree=model.get("degree", 3),
                         gamma=model.get("gamma", 1.0), coef0=model.get("coef0", 0.0))
    np.testing.assert_allclose(vals, ref, rtol=0, atol=TOL[np.float64] * np.abs(ref).max())
    assert np.array_equal(svm.predict(points, alpha=model["alpha"], bias=-model["rho"]), expected)
    svm.close()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_learn_then_predict_dense(oracle, kernel, dtype):
    X, y = datagen.blobs(1500, 24, seed=11, dtype=dtype)
    Z, yz = datagen.blobs(300, 24, seed=12, dtype=dtype)
    p = pm.Parameter(kernel, gamma=1.0 / 24, coef0=1.0 if kernel == "polynomial" else 0.0, real_type=dtype)
    p.data, p.labels = X, y
    with pm.CSVM(p) as svm:
        svm.learn(imax=60)
        vals = svm.predict_values(Z)
        ref = oracle.predict(kernel, X, svm.alpha, -svm.bias, Z, gamma=dtype(1.0 / 24),
                             coef0=dtype(1.0 if kernel == "polynomial" else 0.0))
        np.testing.assert_allclose(vals, ref, rtol=0, atol=TOL[dtype] * np.abs(ref).max())
        # csvm::accuracy on the training data and on held-out points == the oracle's labels' accuracy
        ref_train = oracle.predict(kernel, X, svm.alpha, -svm.bias, X, gamma=dtype(1.0 / 24),
                                   coef0=dtype(1.0 if kernel == "polynomial" else 0.0))
        assert abs(svm.accuracy() - np.mean(np.where(ref_train > 0, 1, -1) == y)) <= 1.0 / 1500
        assert abs(svm.accuracy(Z, yz) - np.mean(np.where(ref > 0, 1, -1) == yz)) <= 1.0 / 300


@pytest.mark.parametrize("fp22", [False, True])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_predict_sparse(oracle, kernel, fp22):
    dtype = np.float32 if fp22 else np.float64
    n, d = 3000, 2000
    csr, y = datagen.sparse_csr(n, d, 20, seed=21, dtype=dtype)
    zc, _ = datagen.sparse_csr(150, d, 20, seed=22, dtype=dtype)
    alpha = np.random.default_rng(3).standard_normal(n).astype(dtype)
    p = pm.Parameter(kernel, gamma=1.0 / d, coef0=0.5, real_type=dtype)
    dec = (lambda v: oracle.fp22_unpack(oracle.fp22_pack(v), v.size)) if fp22 else (lambda v: v)
    if fp22:
        p.csr = (csr[0], csr[1], oracle.fp22_pack(csr[2]), n, d)
        p.val_fmt = pm._abi.VAL_FP22
    else:
        p.csr = csr
    with pm.CSVM(p) as svm:
        zval = oracle.fp22_pack(zc[2]) if fp22 else zc[2]
        vals = svm.predict_values((zc[0], zc[1], zval, zc[3], zc[4]), alpha=alpha, bias=0.25,
                                  val_fmt=pm._abi.VAL_FP22 if fp22 else None)
        Xd = (csr[0], csr[1], dec(csr[2]).astype(dtype), n, d)
        Zd = (zc[0], zc[1], dec(zc[2]).astype(dtype), 150, d)
        ref = oracle.predict(kernel, densify(Xd), alpha, -0.25, densify(Zd), gamma=dtype(1.0 / d), coef0=dtype(0.5))
        np.testing.assert_allclose(vals, ref, rtol=0, atol=TOL[dtype] * np.abs(ref).max())
        if kernel == "linear":
            w = svm.update_w(alpha)
            np.testing.assert_allclose(w, densify(Xd).T @ alpha, rtol=0, atol=TOL[dtype] * np.abs(w).max())


def densify(c):
    rowptr, col, val, n, d = c
    X = np.zeros((n, d), dtype=val.dtype)
    for i in range(n):
        X[i, col[rowptr[i]:rowptr[i + 1]]] = val[rowptr[i]:rowptr[i + 1]]
    return X


def test_update_w_dense():
    X, y = datagen.blobs(700, 40, seed=5)
    alpha = np.random.default_rng(1).standard_normal(700)
    p = pm.Parameter("linear")
    p.data = X
    with pm.CSVM(p) as svm:
        np.testing.assert_allclose(svm.update_w(alpha), X.T @ alpha, rtol=1e-12, atol=1e-12 * np.abs(X.T @ alpha).max())


def test_predict_edge_cases():
    X, y = datagen.blobs(200, 8, seed=6)
    p = pm.Parameter("rbf", gamma=0.125)
    p.data, p.labels = X, y
    with pm.CSVM(p) as svm:
        svm.learn()
        assert svm.predict_values(np.zeros((0, 8))).shape == (0,)
        with pytest.raises(pm.BackendError, match="must match the number of features per predict point"):
            svm.predict_values(np.zeros((3, 7)))
        one = svm.predict_values(X[:1])
        many = svm.predict_values(X)
        np.testing.assert_allclose(one[0], many[0], rtol=1e-13)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_predict_sparse_expansion_matches_brute_force(kernel, dtype, monkeypatch):
    """sparse poly / rbf predict through the kernel expansion (moments + the support vectors sharing two or
    more features with the point) against the brute-force kernel (PLSSVM_MI_PRED_BRUTE): 800k support
    vectors (two passes of the per-point row bitmap) and a dense-ish set whose repeat rows overflow the
    per-pass list (the path then falls back to brute force by itself)"""
    rng = np.random.default_rng(4)
    for n, d, k, npts in [(800_000, 20_000, 10, 200), (6000, 60, 20, 50)]:
        csr, _ = datagen.sparse_csr(n, d, k, seed=31, dtype=dtype)
        zc, _ = datagen.sparse_csr(npts, d, k, seed=32, dtype=dtype)
        alpha = rng.standard_normal(n).astype(dtype)
        p = pm.Parameter(kernel, gamma=1.0 / d, coef0=0.5, real_type=dtype)
        p.csr = csr
        with pm.CSVM(p) as svm:
            svm.setup_data_on_device()
            assert svm.info()["sparse_algo"] == pm._abi.SPARSE_EXPANSION
            got = svm.predict_values(zc, alpha=alpha, bias=0.25)
            monkeypatch.setenv("PLSSVM_MI_PRED_BRUTE", "1")
            want = svm.predict_values(zc, alpha=alpha, bias=0.25)
            monkeypatch.delenv("PLSSVM_MI_PRED_BRUTE")
        np.testing.assert_allclose(got, want, rtol=0, atol=TOL[dtype] * np.abs(want).max(), err_msg=f"n={n}")
