"""CPU tests: pin the C oracle (oracle/) to the reference's own fixtures and known-answer method.

The reference cannot be compiled here ({fmt}/fast_float are absent and may not be stubbed), so
the oracle is pinned by (1) the golden learn() result 5x4.libsvm -> 5x4.libsvm.model, (2) the
predict fixtures for all three kernels, (3) a numpy restatement of the reference's test
comparator compare::generate_q / compare::device_kernel_function
(tests/backends/compare.hpp:103-156) at the reference's tolerance (128 eps relative,
tests/utility.hpp:117-136).
"""
import numpy as np
import pytest

from conftest import fixture_path
from plssvm_sparse_fp22_amd import datagen
from plssvm_sparse_fp22_amd.io import parse_libsvm, parse_model


def ref_near(a, b, scale=1.0):
    """util::gtest_assert_floating_point_near (tests/utility.hpp:117-136), vectorised."""
    a = np.asarray(a)
    b = np.asarray(b)
    eps = 128 * scale * np.finfo(a.dtype).eps
    diff = np.abs(a.astype(np.float64) - b.astype(np.float64))
    norm = np.abs(a.astype(np.float64)) + np.abs(b.astype(np.float64))
    return (a == b) | (diff < np.maximum(np.finfo(a.dtype).tiny, eps * norm))


def np_kernel(kernel, a, b, degree, gamma, coef0):
    """compare::kernel_function: the plain definitions of include/plssvm/kernel_types.hpp:63-85."""
    if kernel == "linear":
        return a @ b
    if kernel == "polynomial":
        return (gamma * (a @ b) + coef0) ** degree
    return np.exp(-gamma * np.sum((a - b) ** 2, axis=-1))


def compare_generate_q(kernel, X, degree, gamma, coef0):
    return np.array([np_kernel(kernel, X[-1], X[i], degree, gamma, coef0) for i in range(X.shape[0] - 1)],
                    dtype=X.dtype)


def compare_device_kernel(kernel, X, x, q, QA_cost, cost, add, degree, gamma, coef0):
    """compare::device_kernel_function (tests/backends/compare.hpp:132-156), row-vectorised, in fp64."""
    m = x.shape[0]
    Xd = X.astype(np.float64)
    r = np.zeros(m)
    for i in range(m):
        kij = np_kernel(kernel, Xd[i][None, :], Xd[: i + 1], degree, gamma, coef0) if kernel == "rbf" else \
            np_kernel(kernel, Xd[: i + 1], Xd[i], degree, gamma, coef0)
        temp = kij + QA_cost - q[i] - q[: i + 1]
        r[i] += np.dot(temp[:i], x[:i]) * add + (temp[i] + 1.0 / cost) * x[i] * add
        r[:i] += temp[:i] * x[i] * add
    return r


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_learn_reproduces_golden_5x4_model(oracle, dtype):
    X, y = parse_libsvm(fixture_path("5x4.libsvm"), dtype=dtype)
    model = parse_model(fixture_path("5x4.libsvm.model"))
    r = oracle.learn("linear", oracle.Data(X, dtype=dtype), y, cost=1.0, eps=1e-3, nthreads=1)
    # match model SV rows (printed with {:e}) to data rows
    order = [int(np.argmin(np.abs(X - sv).sum(axis=1))) for sv in model["SV"]]
    assert sorted(order) == list(range(5))
    if dtype == np.float64:
        assert abs(r["rho"] - model["rho"]) <= 1e-9 * abs(model["rho"])
        np.testing.assert_allclose(r["alpha"][order], model["alpha"], rtol=1e-9, atol=1e-12)
    else:
        # the golden model is an fp64 run; fp32 CG drifts (alpha <= 2e-2 rel in fp32)
        assert abs(r["rho"] - model["rho"]) <= 2e-2 * abs(model["rho"])
        np.testing.assert_allclose(r["alpha"][order], model["alpha"], rtol=2e-2, atol=1e-3)
    assert r["iters"] == 3 and r["trace"].shape == (4,)


@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_kernel_function_pinned_by_predict_fixture(oracle, kernel):
    Z, _ = parse_libsvm(fixture_path("500x200.libsvm.test"))
    expected = np.loadtxt(fixture_path("500x200.libsvm.predict"))
    m = parse_model(fixture_path(f"500x200.libsvm.{kernel}.model"))
    SV = m["SV"]
    if SV.shape[1] < Z.shape[1]:
        SV = np.pad(SV, ((0, 0), (0, Z.shape[1] - SV.shape[1])))
    out = oracle.predict(kernel, SV, m["alpha"], m["rho"], Z, degree=m.get("degree", 3), gamma=m.get("gamma", 1.0),
                         coef0=m.get("coef0", 0.0))
    assert np.array_equal(np.where(out > 0, 1.0, -1.0), expected)
    assert np.all(out * expected > 0)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_q_and_kp_match_reference_comparator(oracle, dtype, kernel):
    X, y = parse_libsvm(fixture_path("500x200.libsvm"), dtype=dtype)
    X = X[:300]
    d = X.shape[1]
    gamma = dtype(1) / dtype(d)
    degree, coef0, cost = 3, dtype(0), dtype(1)
    data = oracle.Data(X, dtype=dtype)
    q = oracle.generate_q(kernel, data, degree=degree, gamma=gamma, coef0=coef0)
    q_ref = compare_generate_q(kernel, X.astype(np.float64), degree, float(gamma), float(coef0)).astype(dtype)
    # numpy's dot is not the reference's sequential fma chain: compare at the chain's error scale
    tol = (1e-12 if dtype == np.float64 else 2e-5) * np.abs(q_ref).max()
    assert ref_near(q, q_ref).mean() > 0.95
    np.testing.assert_allclose(q, q_ref, rtol=0, atol=tol)
    QA = dtype(np_kernel(kernel, X[-1].astype(np.float64), X[-1].astype(np.float64), degree, float(gamma),
                         float(coef0))) + dtype(1) / cost
    rng = np.random.default_rng(7)
    x = rng.uniform(1.0, 2.0, size=X.shape[0] - 1).astype(dtype)
    for add in (-1.0, 1.0):
        got = oracle.kp(kernel, data, q, QA, cost, add, x, degree=degree, gamma=gamma, coef0=coef0, nthreads=4)
        want = compare_device_kernel(kernel, X, x.astype(np.float64), q.astype(np.float64), float(QA), float(cost),
                                     add, degree, float(gamma), float(coef0))
        # reference tolerance 128 eps relative; fp32 accumulation over m terms needs the scale of sum|terms|
        scale = 1.0 if dtype == np.float64 else 4.0
        assert ref_near(got, want.astype(dtype), scale=scale).mean() > 0.99
        np.testing.assert_allclose(got, want, rtol=(1e-11 if dtype == np.float64 else 2e-4), atol=0)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_csr_oracle_bitwise_equals_dense(oracle, dtype, kernel):
    csr, y = datagen.sparse_csr(257, 300, 12, seed=11, dtype=dtype)
    X = datagen.densify(csr)
    dense = oracle.Data(X, dtype=dtype)
    sparse = oracle.Data(rowptr=csr[0], col=csr[1], val=csr[2], n=csr[3], d=csr[4], dtype=dtype)
    g = dtype(1) / dtype(300)
    qd = oracle.generate_q(kernel, dense, gamma=g, coef0=dtype(1))
    qs = oracle.generate_q(kernel, sparse, gamma=g, coef0=dtype(1))
    assert np.array_equal(qd, qs)
    p = np.random.default_rng(1).uniform(1, 2, 256).astype(dtype)
    kd = oracle.kp(kernel, dense, qd, dtype(2.5), dtype(1.5), 1.0, p, gamma=g, coef0=dtype(1), nthreads=1)
    ks = oracle.kp(kernel, sparse, qs, dtype(2.5), dtype(1.5), 1.0, p, gamma=g, coef0=dtype(1), nthreads=1)
    assert np.array_equal(kd, ks)


def test_cg_properties_and_reset(oracle):
    """CG on a blobs set past 50 iterations: the every-50th explicit residual keeps delta consistent."""
    X, y = datagen.blobs(300, 64, seed=5)
    r = oracle.learn("rbf", oracle.Data(X), y, cost=100.0, eps=1e-10, imax=120, nthreads=1)
    assert r["iters"] >= 51  # crosses the run % 50 == 49 explicit-residual iteration
    assert r["trace"][-1] <= 1e-20 * r["trace"][0]  # stop test delta <= eps^2 delta0
    # alpha sums to zero by construction (alpha[m] = -sum)
    assert abs(r["alpha"].sum()) < 1e-9


def test_fp22_codec(oracle):
    rng = np.random.default_rng(0)
    v = np.concatenate([rng.normal(size=10000).astype(np.float32), np.float32([0, -0.0, 1, -1, 3.4e38, 1e-40,
                                                                               np.inf, -np.inf])])
    w = oracle.fp22_pack(v)
    assert w.size == ((v.size + 15) // 16) * 11
    u = oracle.fp22_unpack(w, v.size)
    fin = np.isfinite(v) & (np.abs(v) > 1e-37)
    rel = np.abs(u[fin] - v[fin]) / np.abs(v[fin])
    assert rel.max() <= 2.0 ** -14
    assert np.isinf(u[-2]) and u[-2] > 0 and np.isinf(u[-1]) and u[-1] < 0
    # idempotent: decode(encode(x)) is a fixed point
    assert np.array_equal(oracle.fp22_unpack(oracle.fp22_pack(u), v.size), u)
    nan = oracle.fp22_unpack(oracle.fp22_pack(np.float32([np.nan])), 1)
    assert np.isnan(nan[0])


def test_parser_sparse_fixture():
    X, y = parse_libsvm(fixture_path("5x4.sparse.libsvm"))
    want = np.array([[0, 0, 0, 0], [0, 0, 0.51687296029754564, 0], [0, 1.01405596624706053, 0, 0],
                     [0, 0.60276937379453293, 0, -0.13086851759108944], [0, 0, 0.298499933047586044, 0]])
    assert np.array_equal(X, want)
    assert np.array_equal(y, [1, 1, -1, -1, -1])
    (rowptr, col, val, n, d), _ = parse_libsvm(fixture_path("5x4.sparse.libsvm"), sparse=True)
    assert n == 5 and d == 4 and list(rowptr) == [0, 0, 1, 2, 4, 5]
    assert np.array_equal(datagen.densify((rowptr, col, val, n, d)), want)


def test_product_fp22_codec_matches_oracle(oracle):
    from plssvm_sparse_fp22_amd import fp22

    rng = np.random.default_rng(4)
    v = np.concatenate([rng.normal(size=4099).astype(np.float32) * 10, np.float32([np.inf, -np.inf, 0, -0.0])])
    assert np.array_equal(fp22.pack(v), oracle.fp22_pack(v))
    assert np.array_equal(fp22.unpack(fp22.pack(v), v.size), oracle.fp22_unpack(oracle.fp22_pack(v), v.size))
    assert np.isnan(fp22.unpack(fp22.pack(np.float32([np.nan])), 1)[0])


def test_factored_csr_baseline_equals_the_pairwise_oracle(oracle):
    """The CPU baseline's O(nnz) factored linear K·p (bench.py cpu_baseline_factored) is the same product as
    the oracle's pairwise restatement of the reference kernel (exact up to rounding)."""
    from plssvm_sparse_fp22_amd import datagen

    for dt, tol in ((np.float64, 1e-13), (np.float32, 1e-5)):
        (rowptr, col, val, n, d), _ = datagen.sparse_csr(3000, 400, 20, seed=4, dtype=dt)
        data = oracle.Data(rowptr=rowptr, col=col, val=val, n=n, d=d, dtype=dt)
        q = oracle.generate_q("linear", data)
        p = np.random.default_rng(1).uniform(1, 2, n - 1).astype(dt)
        want = oracle.kp("linear", data, q, dt(2.5), 1.0, -1.0, p)
        got = oracle.kp_csr_factored(data, q, dt(2.5), 1.0, -1.0, p, fast=False)
        assert np.abs(got - want).max() <= tol * np.abs(want).max()
