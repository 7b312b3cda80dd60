"""GPU parity: the HIP path (through the C ABI) against the C oracle and the reference fixtures.

Tolerances: fp64 K·p <= 1e-12 relative to max|K·p|, alpha/rho <= 1e-9 rel,
CG delta trace <= 1e-6 rel per iteration; fp32 K·p <= 1e-4 of max|K·p| (norm-trick RBF and a
different summation order), alpha <= 2e-2 rel, delta <= 1e-3 rel on the first iterations.
"""
import numpy as np
import pytest

from conftest import fixture_path
import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

pytestmark = pytest.mark.gpu

KERNELS = ["linear", "polynomial", "rbf"]
DTYPES = [np.float64, np.float32]
KP_TOL = {np.float64: 1e-12, np.float32: 1e-4}


def make_svm(X, y, kernel, dtype, cost=1.0, gamma=None, degree=3, coef0=0.0, kp_mode="auto"):
    p = pm.Parameter(kernel, degree=degree, gamma=gamma if gamma is not None else 1.0 / X.shape[1], coef0=coef0,
                     cost=cost, real_type=dtype)
    p.data = np.ascontiguousarray(X, dtype=dtype)
    p.labels = None if y is None else np.asarray(y, dtype=dtype)
    return pm.CSVM(p, kp_mode=kp_mode)


def oracle_args(svm):
    p = svm.params
    dt = svm.dtype.type
    return dict(degree=p.degree, gamma=dt(p.gamma), coef0=dt(p.coef0))


def check_kp(oracle, X, kernel, dtype, kp_mode="auto", seed=0):
    svm = make_svm(X, None, kernel, dtype, kp_mode=kp_mode)
    svm.setup_data_on_device()
    q = svm.generate_q()
    data = oracle.Data(X, dtype=dtype)
    q_ref = oracle.generate_q(kernel, data, **oracle_args(svm))
    np.testing.assert_allclose(q, q_ref, rtol=KP_TOL[dtype], atol=KP_TOL[dtype] * max(1e-30, np.abs(q_ref).max()))
    m = X.shape[0] - 1
    rng = np.random.default_rng(seed)
    x = rng.uniform(1.0, 2.0, m).astype(dtype)
    for add in (-1.0, 1.0):
        ret = np.zeros(m, dtype=dtype)
        svm.run_device_kernel(None, ret, x, add)
        want = oracle.kp(kernel, data, q_ref, svm.QA_cost, dtype(1.0), add, x, **oracle_args(svm))
        scale = max(np.abs(want).max(), 1e-30)
        np.testing.assert_allclose(ret, want, rtol=0, atol=KP_TOL[dtype] * scale,
                                   err_msg=f"{kernel} {np.dtype(dtype).name} add={add} shape={X.shape}")
    svm.close()


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("kernel", KERNELS)
def test_kp_reference_fixture_500x200(oracle, kernel, dtype):
    X, _ = pm.parse_libsvm(fixture_path("500x200.libsvm"), dtype=dtype)
    check_kp(oracle, X, kernel, dtype)


@pytest.mark.parametrize("shape", [(2, 1), (3, 5), (129, 7), (130, 17), (257, 64), (700, 33), (1025, 3)])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("kernel", KERNELS)
def test_kp_ragged_shapes(oracle, kernel, dtype, shape):
    rng = np.random.default_rng(shape[0] * 31 + shape[1])
    X = rng.uniform(-1, 1, size=shape).astype(dtype)
    check_kp(oracle, X, kernel, dtype, seed=shape[0])


@pytest.mark.parametrize("dtype", DTYPES)
def test_kp_linear_factored_mode(oracle, dtype):
    X, _ = datagen.blobs(777, 45, seed=3, dtype=dtype)
    check_kp(oracle, X, "linear", dtype, kp_mode="factored")


def test_mfma_layout_asymmetric_integer_data(oracle):
    """Exact small-integer data: any swapped MFMA row/col map breaks bitwise equality of the linear K·p."""
    rng = np.random.default_rng(5)
    for dtype in DTYPES:
        X = rng.integers(-3, 4, size=(300, 24)).astype(dtype)
        svm = make_svm(X, None, "linear", dtype)
        svm.setup_data_on_device()
        q = svm.generate_q()
        x = rng.integers(1, 3, size=299).astype(dtype)
        ret = np.zeros(299, dtype=dtype)
        svm.run_device_kernel(None, ret, x, 1.0)
        want = oracle.kp("linear", oracle.Data(X, dtype=dtype), q, svm.QA_cost, dtype(1), 1.0, x)
        assert np.array_equal(ret, want), np.abs(ret - want).max()
        svm.close()


@pytest.mark.parametrize("dtype", DTYPES)
def test_kp_bitwise_reproducible(dtype):
    X, _ = datagen.blobs(600, 40, seed=9, dtype=dtype)
    svm = make_svm(X, None, "rbf", dtype)
    svm.setup_data_on_device()
    svm.generate_q()
    x = np.linspace(1, 2, 599).astype(dtype)
    a = svm.run_device_kernel(None, np.zeros(599, dtype), x, 1.0)
    b = svm.run_device_kernel(None, np.zeros(599, dtype), x, 1.0)
    assert np.array_equal(a, b)


@pytest.mark.parametrize("dtype", DTYPES)
def test_learn_reproduces_golden_5x4_model(dtype):
    X, y = pm.parse_libsvm(fixture_path("5x4.libsvm"), dtype=dtype)
    model = pm.parse_model(fixture_path("5x4.libsvm.model"))
    svm = make_svm(X, y, "linear", dtype)
    svm.learn()
    order = [int(np.argmin(np.abs(X - sv).sum(axis=1))) for sv in model["SV"]]
    tol = 1e-9 if dtype == np.float64 else 2e-2
    assert abs(svm.rho - model["rho"]) <= tol * abs(model["rho"])
    np.testing.assert_allclose(svm.alpha[order], model["alpha"], rtol=tol, atol=tol * 1e-3)
    assert svm.iters == 3


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("kernel", KERNELS)
def test_learn_matches_oracle_config1(oracle, kernel, dtype):
    """Config 1: generate_data.py-style blobs 500x4 (seeded); full learn(), imax = d = 4."""
    X, y = datagen.blobs(500, 4, seed=1, dtype=dtype)
    svm = make_svm(X, y, kernel, dtype)
    svm.learn()
    ref = oracle.learn(kernel, oracle.Data(X, dtype=dtype), y, **oracle_args(svm))
    assert svm.iters == ref["iters"]
    if dtype == np.float64:
        np.testing.assert_allclose(svm.trace, ref["trace"], rtol=1e-6)
        np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=1e-9, atol=1e-9 * np.abs(ref["alpha"]).max())
        assert abs(svm.rho - ref["rho"]) <= 1e-9 * max(1.0, abs(ref["rho"]))
    else:
        np.testing.assert_allclose(svm.trace[:3], ref["trace"][:3], rtol=1e-3)
        np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=2e-2, atol=2e-2 * np.abs(ref["alpha"]).max())


def test_learn_config2_scaled_down(oracle):
    """Config 2 shape (dense RBF, d = 256, fp64, C = 1, eps = 1e-3) at N = 3000: residual curve to 1e-6."""
    X, y = datagen.blobs(3000, 256, seed=2, cluster_std=4.0)
    svm = make_svm(X, y, "rbf", np.float64)
    svm.learn()
    ref = oracle.learn("rbf", oracle.Data(X), y, gamma=1.0 / 256)
    assert svm.iters == ref["iters"]
    np.testing.assert_allclose(svm.trace, ref["trace"], rtol=1e-6)
    np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=1e-9, atol=1e-9 * np.abs(ref["alpha"]).max())


@pytest.mark.parametrize("kernel,cost,std",[("linear", 1e4, 4.0), ("polynomial", 1e4, 1.0), ("rbf", 100.0, 1.0)])
def test_cg_trace_across_explicit_residual(oracle, kernel, cost, std):
    """> 50 iterations (run % 50 == 49 recomputes r = b - Q~x, OpenMP/csvm.cpp:130-139).

    These systems are ill-conditioned (C >= 100), so rounding differences grow along the CG
    recurrence: the reference OpenMP kernel itself (atomics) gives traces that differ by > 1e-6
    between 1 and 8 threads after a few iterations. The bar is therefore 1e-6 on the first
    iterations where OpenMP itself is reproducible (its 1-vs-8-thread deviation < 1e-9); after
    that, the same iteration count (+-2) and the same converged solution."""
    X, y = datagen.blobs(300, 64, seed=5, cluster_std=std)
    svm = make_svm(X, y, kernel, np.float64, cost=cost)
    svm.setup_data_on_device()
    q = svm.generate_q()
    b = (y[:-1] - y[-1]).astype(np.float64)
    x = svm.solver_CG(b, 150, 1e-10, q)
    args = dict(degree=3, gamma=1.0 / 64, coef0=0.0)
    data = oracle.Data(X)
    ref_x, ref_t, ref_it = oracle.solve_cg(kernel, data, b, 150, 1e-10, q, svm.QA_cost, cost, nthreads=1, **args)
    _, ref_t8, _ = oracle.solve_cg(kernel, data, b, 150, 1e-10, q, svm.QA_cost, cost, nthreads=8, **args)
    assert ref_it > 50, "test must cross the explicit-residual iteration"
    assert abs(svm.iters - ref_it) <= 2
    n = min(len(svm.trace), len(ref_t), len(ref_t8))
    self_noise = np.maximum.accumulate(np.abs(ref_t8[:n] / ref_t[:n] - 1))
    dev = np.abs(svm.trace[:n] / ref_t[:n] - 1)
    reproducible = self_noise < 1e-9
    assert reproducible[:3].all()
    assert np.all(dev[reproducible] <= 1e-6), (dev, self_noise)
    # both converged (delta <= eps^2 delta0): solutions agree to the conditioning of the system
    np.testing.assert_allclose(x, ref_x, rtol=1e-3, atol=1e-3 * np.abs(ref_x).max())


@pytest.mark.parametrize("layout,kernel", [("dense", "rbf"), ("dense", "linear"), ("csr", "linear"),
                                           ("csr", "rbf")])
def test_cg_graph_blocks_bitwise_equal_to_launches(layout, kernel):
    """cg_step(130) replays iterations [0, 50) and [50, 100) — each with its explicit-residual
    iteration — from one captured hipGraph and runs [100, 130) as launches; 130 single cg_step(1)
    calls never use the graph. Same kernels, same order: x and the delta trace are bitwise equal."""
    if layout == "csr":
        csr, y = datagen.sparse_csr(1500, 300, 12, seed=13, dtype=np.float64)
    else:
        X, y = datagen.blobs(700, 40, seed=13, cluster_std=3.0)
    out = []
    for batched in (True, False):
        p = pm.Parameter(kernel, gamma=1.0 / (300 if layout == "csr" else 40), cost=100.0, real_type=np.float64)
        if layout == "csr":
            p.csr = csr
        else:
            p.data = np.ascontiguousarray(X)
        with pm.CSVM(p) as svm:
            svm.setup_data_on_device()
            svm.generate_q()
            svm.cg_begin((y[:-1] - y[-1]).astype(np.float64), eps=1e-300)
            if batched:
                it, _ = svm.cg_step(130)
            else:
                for _ in range(130):
                    it, _ = svm.cg_step(1)
            out.append(svm.cg_result(131))
    (xa, ta, ia), (xb, tb, ib) = out
    assert ia == ib == 130
    assert np.array_equal(xa, xb) and np.array_equal(ta, tb)


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("kernel,mode", [("rbf", "auto"), ("polynomial", "auto"), ("linear", "factored")])
def test_simulated_ranks_sum_to_full_kp(oracle, world, kernel, mode):
    """The multi-GPU work split on one GPU: each simulated rank computes only its super-blocks
    (pairwise) or rows (factored); the shares sum to the single-rank K·p (the RCCL all-reduce)."""
    X, _ = datagen.blobs(2600, 24, seed=4)
    m = X.shape[0] - 1
    x = np.linspace(1, 2, m)
    full = make_svm(X, None, kernel, np.float64, kp_mode=mode)
    full.setup_data_on_device()
    q = full.generate_q()
    want = full.run_device_kernel(None, np.zeros(m), x, 1.0)
    total = np.zeros(m)
    for r in range(world):
        p = pm.Parameter(kernel, gamma=1.0 / 24)
        p.data = X
        svm = pm.CSVM(p, kp_mode=mode, sim_rank=(r, world))
        svm.setup_data_on_device()
        svm.generate_q()
        total += svm.run_device_kernel(None, np.zeros(m), x, 1.0)
        svm.close()
    np.testing.assert_allclose(total, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


def test_state_errors():
    X, _ = datagen.blobs(50, 3, seed=2)
    svm = make_svm(X, None, "rbf", np.float64)
    with pytest.raises(pm.BackendError):
        svm.generate_q()
    svm.setup_data_on_device()
    with pytest.raises(pm.BackendError):
        svm.run_device_kernel(None, np.zeros(49), np.ones(49), 1.0)


def test_single_point_degenerate():
    X = np.array([[0.5, -0.25]])
    svm = make_svm(X, np.array([1.0]), "rbf", np.float64)
    svm.learn()
    assert svm.alpha.shape == (1,) and svm.alpha[0] == 0.0


@pytest.mark.parametrize("layout,kernel,kp_mode", [("dense", "rbf", "auto"), ("dense", "linear", "factored"),
                                                   ("csr", "linear", "auto"), ("csr", "rbf", "auto")])
def test_single_rank_rccl_group(layout, kernel, kp_mode):
    """A one-rank RCCL group (uid given) runs every per-K·p collective through RCCL on this GPU
    (all-reduce of the raw K·p / of w, all-gather of the factored rows): the K·p and a CG solve must
    equal the context without a communicator bit for bit — the collective code path on hardware."""
    n, d = 3000, 64
    if layout == "dense":
        X, y = datagen.blobs(n, d, seed=3)
    else:
        csr, y = datagen.sparse_csr(n, 5000, 20, seed=3, dtype=np.float64)
    outs = []
    for uid in (None, pm.unique_id()):
        p = pm.Parameter(kernel, gamma=1.0 / d, real_type=np.float64)
        if layout == "dense":
            p.data = X
        else:
            p.csr = csr
        p.labels = y
        svm = pm.CSVM(p, kp_mode=kp_mode, uid=uid)
        svm.setup_data_on_device()
        svm.generate_q()
        x = np.linspace(1, 2, n - 1)
        ret = svm.run_device_kernel(None, np.zeros(n - 1), x, 1.0)
        svm.learn(imax=40)
        outs.append((ret, np.array(svm.trace), svm.alpha.copy()))
        svm.close()
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("layout,kernel,kp_mode,algo", [("csr", "rbf", "auto", "auto"), ("csr", "polynomial", "auto", "auto"),
                                                        ("csr", "linear", "auto", "auto"),
                                                        ("csr", "rbf", "auto", "onthefly"), ("csr", "rbf", "auto", "pattern"),
                                                        ("dense", "rbf", "auto", "auto")])
def test_single_rank_rccl_group_sharded(layout, kernel, kp_mode, algo, monkeypatch):
    """The sharded CG's RCCL code (PLSSVM_MI_SHARD=1 in a one-rank RCCL group): dot partials all-gathered
    (the step's sum d / sum q d partials grouped with the next K·p's first collective), K·p inputs
    all-gathered, the expansion's w all-gather and moment all-reduce on the collective stream overlapping
    the moments pass and the remainder stream, reduce-scatter of the pattern / tile partial sums. With one
    rank every gathered sum is the local one, so K·p, the CG trace and the alphas must equal the context
    without a communicator bit for bit."""
    n, d = 3000, 64
    if layout == "dense":
        X, y = datagen.blobs(n, d, seed=3)
    else:
        csr, y = datagen.sparse_csr(n, 5000, 20, seed=3, dtype=np.float64)
    outs = []
    for uid in (None, pm.unique_id()):
        if uid is None:
            monkeypatch.delenv("PLSSVM_MI_SHARD", raising=False)
        else:
            monkeypatch.setenv("PLSSVM_MI_SHARD", "1")
        p = pm.Parameter(kernel, gamma=1.0 / d, coef0=1.0 if kernel == "polynomial" else 0.0, real_type=np.float64)
        if layout == "dense":
            p.data = X
        else:
            p.csr = csr
        p.labels = y
        svm = pm.CSVM(p, kp_mode=kp_mode, uid=uid, sparse_algo=algo)
        svm.setup_data_on_device()
        svm.generate_q()
        x = np.linspace(1, 2, n - 1)
        ret = svm.run_device_kernel(None, np.zeros(n - 1), x, 1.0)
        svm.learn(imax=60)  # crosses the every-50th explicit residual
        outs.append((ret, np.array(svm.trace), svm.alpha.copy()))
        svm.close()
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)


@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_single_rank_rccl_group_sharded_bf16(kernel, monkeypatch):
    """The sharded expansion with bfloat16 windows (fp32): the group gathers the rows'
    bfloat16 w and the ranks' S partials instead of w (expansion_kp_raw). With one rank the gathered
    partials are the local ones in dot2's grid order, so K·p, trace and alphas equal the context without a
    communicator bit for bit."""
    n, nf = 3000, 5000
    csr, y = datagen.sparse_csr(n, nf, 20, seed=3, dtype=np.float32)
    outs = []
    for uid in (None, pm.unique_id()):
        if uid is None:
            monkeypatch.delenv("PLSSVM_MI_SHARD", raising=False)
        else:
            monkeypatch.setenv("PLSSVM_MI_SHARD", "1")
        p = pm.Parameter(kernel, gamma=1.0 / nf, coef0=1.0 if kernel == "polynomial" else 0.0, real_type=np.float32)
        p.csr = csr
        p.labels = y
        svm = pm.CSVM(p, uid=uid, sparse_algo="expansion")
        svm.setup_data_on_device()
        assert svm.info()["exp_hbytes"] == 2
        svm.generate_q()
        x = np.linspace(1, 2, n - 1).astype(np.float32)
        ret = svm.run_device_kernel(None, np.zeros(n - 1, np.float32), x, 1.0)
        svm.learn(imax=60)
        outs.append((ret, np.array(svm.trace), svm.alpha.copy()))
        svm.close()
    for a, b in zip(outs[0], outs[1]):
        np.testing.assert_array_equal(a, b)
