"""GPU parity of the sparse paths (CSR / packed FP22) against the oracle's CSR restatement.

The reference has no sparse device path (its parser densifies, src/plssvm/parameter.cpp:66-87), so
parity is "same math as the dense OpenMP semantics on the densified (and FP22-dequantised) matrix":
the oracle's CSR functions are bitwise equal to its dense ones (tests/test_oracle.py).
Tolerances as in test_gpu_parity.py (fp64 1e-12 / fp32 1e-4 of max|K·p|).
"""
import numpy as np
import pytest

import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen

pytestmark = pytest.mark.gpu

TOL = {np.float64: 1e-12, np.float32: 1e-4}


def sparse_svm(csr, kernel, dtype, fp22=False, mode="auto", sim=None, gamma=None, coef0=1.0, y=None, cost=1.0,
               algo="auto"):
    rbf_form = 0
    if mode == "direct":  # rbf pairs as exp(-g |x_i - x_j|^2) - e_i e_j instead of the factored form
        mode, rbf_form = "auto", 1
    rowptr, col, val, n, d = csr
    p = pm.Parameter(kernel, gamma=gamma if gamma is not None else 1.0 / d, coef0=coef0, real_type=dtype, cost=cost)
    if fp22:
        from oracle import pyoracle

        p.csr = (rowptr, col, pyoracle.fp22_pack(val), n, d)
        p.val_fmt = pm._abi.VAL_FP22
    else:
        p.csr = (rowptr, col, val.astype(dtype), n, d)
    p.labels = y
    return pm.CSVM(p, kp_mode=mode, sim_rank=sim, rbf_form=rbf_form, sparse_algo=algo)


def oracle_data(oracle, csr, dtype, fp22=False):
    rowptr, col, val, n, d = csr
    if fp22:
        val = oracle.fp22_unpack(oracle.fp22_pack(val), val.size)
    return oracle.Data(rowptr=rowptr, col=col, val=val.astype(dtype), n=n, d=d, dtype=dtype)


def check_sparse_kp(oracle, csr, kernel, dtype, fp22=False, mode="auto", coef0=1.0, gamma=None, algo="auto"):
    svm = sparse_svm(csr, kernel, dtype, fp22=fp22, mode=mode, coef0=coef0, gamma=gamma, algo=algo)
    svm.setup_data_on_device()
    q = svm.generate_q()
    data = oracle_data(oracle, csr, dtype, fp22)
    g = dtype(gamma if gamma is not None else 1.0 / csr[4])
    q_ref = oracle.generate_q(kernel, data, gamma=g, coef0=dtype(coef0))
    np.testing.assert_allclose(q, q_ref, rtol=TOL[dtype], atol=TOL[dtype] * np.abs(q_ref).max())
    m = csr[3] - 1
    x = np.random.default_rng(m).uniform(1, 2, m).astype(dtype)
    for add in (-1.0, 1.0):
        ret = np.zeros(m, dtype=dtype)
        svm.run_device_kernel(None, ret, x, add)
        want = oracle.kp(kernel, data, q_ref, svm.QA_cost, dtype(1.0), add, x, gamma=g, coef0=dtype(coef0))
        np.testing.assert_allclose(ret, want, rtol=0, atol=TOL[dtype] * np.abs(want).max(),
                                   err_msg=f"{kernel} {np.dtype(dtype).name} fp22={fp22} mode={mode} algo={algo}")
    info = svm.info()
    svm.close()
    return info


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel,mode,algo", [("linear", "auto", "auto"), ("linear", "pairwise", "auto"),
                                              ("polynomial", "auto", "auto"), ("polynomial", "auto", "pattern"),
                                              ("rbf", "auto", "auto"), ("rbf", "auto", "pattern"),
                                              ("rbf", "direct", "auto")])
@pytest.mark.parametrize("shape", [(300, 500, 10), (2500, 3000, 20), (9000, 20000, 15)])
def test_sparse_kp(oracle, kernel, mode, algo, dtype, shape):
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=n + d, dtype=dtype)
    info = check_sparse_kp(oracle, csr, kernel, dtype, mode=mode, algo=algo)
    assert info["is_sparse"] == 1
    assert info["rbf_factored"] == (kernel == "rbf" and mode == "auto")
    if kernel != "linear":  # auto picks the kernel expansion on these sets (small 2 g x^2, degree 3)
        want = pm._abi.SPARSE_PATTERN if (algo == "pattern" or mode == "direct") else pm._abi.SPARSE_EXPANSION
        assert info["sparse_algo"] == want


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel,gamma,coef0", [("rbf", 0.5, 0.0), ("rbf", 3.0, 0.0), ("polynomial", 0.3, 1.5),
                                                ("polynomial", 0.05, -0.7)])
def test_sparse_expansion_large_arguments(oracle, kernel, gamma, coef0, dtype):
    """Larger 2 g x^2 (Taylor degree up to 16) and poly with coef0 != 0 (all binomial terms), dense-ish
    rows so that many pairs share several features (the stored remainder H carries real weight)."""
    csr, _ = datagen.sparse_csr(1500, 60, 12, seed=17, dtype=dtype)
    info = check_sparse_kp(oracle, csr, kernel, dtype, gamma=gamma, coef0=coef0)
    if info["sparse_algo"] == pm._abi.SPARSE_EXPANSION:
        assert info["pairs"] > 0 and info["exp_terms"] >= 1


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
@pytest.mark.parametrize("shape", [(300, 500, 10), (2500, 3000, 20)])
def test_sparse_densified_path(oracle, kernel, dtype, shape):
    """PLSSVM_MI_SPARSE_DENSE: X densified on the device, K·p on the dense MFMA tiles."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=n + 7, dtype=dtype)
    info = check_sparse_kp(oracle, csr, kernel, dtype, algo="dense")
    assert info["sparse_algo"] == pm._abi.SPARSE_DENSE and info["pair_slots"] == 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel,mode,gamma,coef0", [("rbf", "auto", None, 1.0), ("rbf", "direct", None, 1.0),
                                                     ("polynomial", "auto", None, 1.0),
                                                     ("polynomial", "auto", 0.05, -0.7), ("rbf", "auto", 3.0, 0.0)])
@pytest.mark.parametrize("shape", [(300, 500, 10), (2500, 3000, 20), (9000, 20000, 15), (3000, 50, 20)])
def test_sparse_onthefly_kp(oracle, kernel, mode, gamma, coef0, dtype, shape):
    """PLSSVM_MI_SPARSE_ONTHEFLY: s_ij re-formed from the CSR / CSC on every K·p. (3000, 50, 20): every
    column holds ~1200 rows, so one feature's segment of a partner window is longer than a wave."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=n + 3, dtype=dtype)
    info = check_sparse_kp(oracle, csr, kernel, dtype, mode=mode, gamma=gamma, coef0=coef0, algo="onthefly")
    assert info["sparse_algo"] == pm._abi.SPARSE_ONTHEFLY and info["pair_slots"] == 0
    if gamma is None:  # large g |x|^2 may leave the factored form's range: the direct form is used then
        assert info["rbf_factored"] == (kernel == "rbf" and mode == "auto")


def test_sparse_onthefly_ragged_and_linear_pairwise(oracle):
    """empty rows, a row with every feature (several 64-feature batches), uneven rows; the linear kernel
    in pairwise mode through the same pair kernel"""
    rng = np.random.default_rng(19)
    n, d = 1900, 333
    rows = []
    for i in range(n):
        kk = 0 if i % 97 == 0 else (d if i in (5, 1500) else int(rng.integers(1, 40)))
        rows.append(np.sort(rng.choice(d, size=kk, replace=False)))
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum([r.size for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(-1, 1, col.size)
    csr = (rowptr, col, val, n, d)
    for kernel in ("rbf", "polynomial"):
        info = check_sparse_kp(oracle, csr, kernel, np.float64, algo="onthefly")
        assert info["sparse_algo"] == pm._abi.SPARSE_ONTHEFLY
    check_sparse_kp(oracle, csr, "linear", np.float64, mode="pairwise", algo="onthefly")


@pytest.mark.parametrize("world", [2, 3])
def test_sparse_onthefly_simulated_ranks(world):
    """rank shares (rows split) sum to the single-rank K·p"""
    csr, _ = datagen.sparse_csr(6000, 3000, 25, seed=12, dtype=np.float64)
    m = csr[3] - 1
    x = np.linspace(1, 2, m)
    full = sparse_svm(csr, "rbf", np.float64, algo="onthefly")
    full.setup_data_on_device()
    full.generate_q()
    want = full.run_device_kernel(None, np.zeros(m), x, 1.0)
    full.close()
    total = np.zeros(m)
    for r in range(world):
        svm = sparse_svm(csr, "rbf", np.float64, sim=(r, world), algo="onthefly")
        svm.setup_data_on_device()
        svm.generate_q()
        total += svm.run_device_kernel(None, np.zeros(m), x, 1.0)
        svm.close()
    np.testing.assert_allclose(total, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


def test_sparse_onthefly_learn_fp22_and_reproducible(oracle):
    """learn() through the on-the-fly path (CG, rank-1 terms, bias); FP22 input == its decoded values bit for
    bit; repeated K·p launches give identical bits; the overlap part equals the Gram pattern's"""
    csr, y = datagen.sparse_csr(2000, 2500, 30, seed=8, dtype=np.float64)
    svm = sparse_svm(csr, "rbf", np.float64, y=y, coef0=0.0, algo="onthefly")
    svm.learn(imax=60)
    ref = oracle.learn("rbf", oracle_data(oracle, csr, np.float64), y, imax=60, gamma=1.0 / 2500)
    assert abs(svm.iters - ref["iters"]) <= 1
    n = min(len(svm.trace), len(ref["trace"]), 6)
    np.testing.assert_allclose(svm.trace[:n], ref["trace"][:n], rtol=1e-6)
    np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=1e-6, atol=1e-6 * np.abs(ref["alpha"]).max())
    svm.close()
    from plssvm_sparse_fp22_amd.fp22 import pack, unpack

    c32, _ = datagen.sparse_csr(5000, 2000, 25, seed=5, dtype=np.float32)
    dec = unpack(pack(c32[2]), c32[2].size)
    x = np.random.default_rng(4).uniform(1, 2, c32[3] - 1).astype(np.float32)
    outs = []
    for fp22 in (True, False, False):
        c = (c32[0], c32[1], c32[2] if fp22 else dec, c32[3], c32[4])
        s2 = sparse_svm(c, "rbf", np.float32, fp22=fp22, algo="onthefly")
        s2.setup_data_on_device()
        s2.generate_q()
        outs.append(s2.run_device_kernel(None, np.zeros(c32[3] - 1, np.float32), x, 1.0))
        if not fp22:
            outs.append(s2.kp_part(x, "overlap"))
        s2.close()
    np.testing.assert_array_equal(outs[0], outs[1])
    np.testing.assert_array_equal(outs[1], outs[3])
    np.testing.assert_array_equal(outs[2], outs[4])
    pat = sparse_svm((c32[0], c32[1], dec, c32[3], c32[4]), "rbf", np.float32, algo="pattern")
    pat.setup_data_on_device()
    want = pat.kp_part(x, "overlap")
    pat.close()
    np.testing.assert_allclose(outs[2], want, rtol=0, atol=1e-4 * np.abs(want).max())


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sparse_over_budget_onthefly_sampled(dtype, monkeypatch):
    """auto over the device budget at 1 % density (60k x 20k, 200 features per row): the setup's estimate
    picks the on-the-fly path over the densified tiles; 128 sampled rows of sum_j k_ij p_j against a float64
    recomputation (fp32 1e-4 / fp64 1e-12 of sum_j |k_ij p_j|)"""
    import scipy.sparse as sp

    n, d, k = 60_000, 20_000, 200
    rng = np.random.default_rng(31)
    col = np.concatenate([np.sort(rng.choice(d, k, replace=False)) for _ in range(n)]).astype(np.int32)
    val = rng.uniform(-1, 1, n * k)
    rowptr = np.arange(0, (n + 1) * k, k, dtype=np.int64)
    monkeypatch.setenv("PLSSVM_MI_MEM_BUDGET", "4096")
    prm = pm.Parameter("rbf", gamma=1.0 / d, real_type=dtype)
    prm.csr = (rowptr, col, val.astype(dtype), n, d)
    m = n - 1
    p = rng.uniform(1, 2, m).astype(dtype)
    with pm.CSVM(prm) as svm:
        svm.setup_data_on_device()
        assert svm.info()["sparse_algo"] == pm._abi.SPARSE_ONTHEFLY
        got = svm.kp_part(p, "kernel")
    rows = np.sort(rng.choice(m, 128, replace=False))
    X = sp.csr_matrix((val.astype(dtype).astype(np.float64), col, rowptr), shape=(n, d))
    nrm = np.asarray(X.multiply(X).sum(axis=1)).ravel()
    G = (X[rows] @ X[:m].T).toarray()
    K = np.exp(-(1.0 / d) * np.maximum(nrm[rows, None] + nrm[None, :m] - 2.0 * G, 0.0))
    want, scale = K @ p.astype(np.float64), K @ np.abs(p.astype(np.float64))
    err = np.max(np.abs(got[rows] - want) / scale)
    assert err <= (1e-4 if dtype == np.float32 else 1e-12), err


@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_sparse_over_budget_falls_back_to_densified(oracle, kernel, monkeypatch):
    """auto: a stored structure estimated above the device budget (PLSSVM_MI_MEM_BUDGET) is never built;
    the densified path runs instead, with the same results. A forced algorithm ignores the budget."""
    csr, _ = datagen.sparse_csr(3000, 400, 25, seed=4, dtype=np.float64)
    monkeypatch.setenv("PLSSVM_MI_MEM_BUDGET", "4096")
    info = check_sparse_kp(oracle, csr, kernel, np.float64)
    assert info["sparse_algo"] in (pm._abi.SPARSE_DENSE, pm._abi.SPARSE_ONTHEFLY)  # the setup's cost estimate
    info = check_sparse_kp(oracle, csr, kernel, np.float64, algo="expansion")
    assert info["sparse_algo"] == pm._abi.SPARSE_EXPANSION
    monkeypatch.delenv("PLSSVM_MI_MEM_BUDGET")
    info = check_sparse_kp(oracle, csr, kernel, np.float64)
    assert info["sparse_algo"] == pm._abi.SPARSE_EXPANSION


def test_sparse_densified_learn_and_fp22(oracle):
    """the densified path through learn() (CG, rank-1 terms, bias) and with packed FP22 input"""
    csr, y = datagen.sparse_csr(1500, 900, 30, seed=6, dtype=np.float64)
    svm = sparse_svm(csr, "rbf", np.float64, y=y, coef0=0.0, algo="dense")
    svm.learn(imax=40)
    ref = oracle.learn("rbf", oracle_data(oracle, csr, np.float64), y, imax=40, gamma=1.0 / 900)
    assert abs(svm.iters - ref["iters"]) <= 1
    n = min(len(svm.trace), len(ref["trace"]), 6)
    np.testing.assert_allclose(svm.trace[:n], ref["trace"][:n], rtol=1e-6)
    np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=1e-6, atol=1e-6 * np.abs(ref["alpha"]).max())
    svm.close()
    csr32, _ = datagen.sparse_csr(2000, 1200, 25, seed=5, dtype=np.float32)
    info = check_sparse_kp(oracle, csr32, "rbf", np.float32, fp22=True, algo="dense")
    assert info["sparse_algo"] == pm._abi.SPARSE_DENSE


@pytest.mark.parametrize("rbb,groups", [("4096", "1"), ("8192", "1"), ("32768", "1"), ("4096", "2"), ("8192", "3")])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sparse_expansion_stream_geometries(oracle, rbb, groups, dtype, monkeypatch):
    """every remainder-stream geometry (rows per block / window width, PLSSVM_MI_EXP_RBB; window groups
    with partial row sums, PLSSVM_MI_EXP_G) against the oracle, on data whose multi-feature pairs span
    several windows and blocks"""
    monkeypatch.setenv("PLSSVM_MI_EXP_RBB", rbb)
    monkeypatch.setenv("PLSSVM_MI_EXP_G", groups)
    csr, _ = datagen.sparse_csr(42000, 600, 10, seed=21, dtype=dtype)
    info = check_sparse_kp(oracle, csr, "rbf", dtype, gamma=0.1)
    assert info["sparse_algo"] == pm._abi.SPARSE_EXPANSION and info["pairs"] > 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_sparse_rbf_large_gamma_falls_back_to_direct(oracle, dtype):
    """g max|x|^2 far outside the factored form's range (e_i underflows): auto must pick the direct form."""
    csr, _ = datagen.sparse_csr(2500, 300, 20, seed=11, dtype=dtype)
    info = check_sparse_kp(oracle, csr, "rbf", dtype, gamma=50.0)
    assert info["rbf_factored"] == 0


@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_sparse_gram_bitwise_reproducible(kernel):
    """integer LDS accumulation: repeated K·p launches give identical bits"""
    csr, _ = datagen.sparse_csr(9000, 2000, 30, seed=3, dtype=np.float32)
    svm = sparse_svm(csr, kernel, np.float32)
    svm.setup_data_on_device()
    svm.generate_q()
    m = csr[3] - 1
    x = np.random.default_rng(1).standard_normal(m).astype(np.float32)
    outs = []
    for _ in range(3):
        ret = np.zeros(m, dtype=np.float32)
        svm.run_device_kernel(None, ret, x, 1.0)
        outs.append(ret)
    svm.close()
    assert all(np.array_equal(outs[0], o) for o in outs[1:])


@pytest.mark.parametrize("kernel", ["linear", "rbf", "polynomial"])
def test_sparse_fp22(oracle, kernel):
    csr, _ = datagen.sparse_csr(3000, 4000, 25, seed=5, dtype=np.float32)
    info = check_sparse_kp(oracle, csr, kernel, np.float32, fp22=True)
    assert info["val_fmt"] == pm._abi.VAL_FP22


def test_sparse_ragged_rows(oracle):
    """empty rows, a dense row, duplicate-free but uneven rows, d not a multiple of anything."""
    rng = np.random.default_rng(9)
    n, d = 700, 333
    rows = []
    for i in range(n):
        k = 0 if i % 97 == 0 else (d if i == 5 else int(rng.integers(1, 30)))
        rows.append(np.sort(rng.choice(d, size=k, replace=False)))
    rowptr = np.zeros(n + 1, np.int64)
    rowptr[1:] = np.cumsum([r.size for r in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(-1, 1, col.size)
    csr = (rowptr, col, val, n, d)
    for kernel in ("rbf", "polynomial", "linear"):
        check_sparse_kp(oracle, csr, kernel, np.float64)
        check_sparse_kp(oracle, csr, kernel, np.float64, mode="pairwise" if kernel == "linear" else "auto")


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("kernel,mode", [("rbf", "auto"), ("linear", "auto")])
def test_sparse_simulated_ranks(world, kernel, mode):
    csr, _ = datagen.sparse_csr(6000, 5000, 20, seed=2, dtype=np.float64)
    m = csr[3] - 1
    x = np.linspace(1, 2, m)
    full = sparse_svm(csr, kernel, np.float64, mode=mode)
    full.setup_data_on_device()
    full.generate_q()
    want = full.run_device_kernel(None, np.zeros(m), x, 1.0)
    total = np.zeros(m)
    for r in range(world):
        svm = sparse_svm(csr, kernel, np.float64, mode=mode, sim=(r, world))
        svm.setup_data_on_device()
        svm.generate_q()
        total += svm.run_device_kernel(None, np.zeros(m), x, 1.0)
        svm.close()
    np.testing.assert_allclose(total, want, rtol=1e-12, atol=1e-12 * np.abs(want).max())


@pytest.mark.parametrize("kernel", ["linear", "rbf"])
def test_sparse_learn_matches_oracle(oracle, kernel):
    csr, y = datagen.sparse_csr(2000, 2500, 30, seed=8, dtype=np.float64)
    svm = sparse_svm(csr, kernel, np.float64, y=y, coef0=0.0)
    svm.learn(imax=60)
    ref = oracle.learn(kernel, oracle_data(oracle, csr, np.float64), y, imax=60, gamma=1.0 / 2500)
    assert abs(svm.iters - ref["iters"]) <= 1
    n = min(len(svm.trace), len(ref["trace"]), 6)
    np.testing.assert_allclose(svm.trace[:n], ref["trace"][:n], rtol=1e-6)
    np.testing.assert_allclose(svm.alpha, ref["alpha"], rtol=1e-6, atol=1e-6 * np.abs(ref["alpha"]).max())


@pytest.mark.parametrize("kernel,mode", [("rbf", "auto"), ("rbf", "direct"), ("polynomial", "auto"),
                                         ("linear", "pairwise"), ("linear", "auto")])
def test_sparse_fp22_equals_decoded_input(kernel, mode):
    """FP22 input == the same matrix given as decoded fp32, bit for bit, at a size with several Gram row
    blocks and windows (rows >= 4096; a device-side FP22 decode in the Gram build once broke exactly there)."""
    from plssvm_sparse_fp22_amd.fp22 import pack, unpack

    n, d, k = 20000, 4000, 50
    csr, _ = datagen.sparse_csr(n, d, k, seed=5, dtype=np.float32)
    dec = unpack(pack(csr[2]), csr[2].size)
    x = np.random.default_rng(4).uniform(1, 2, n - 1).astype(np.float32)
    outs = []
    for fp22 in (True, False):
        c = (csr[0], csr[1], csr[2] if fp22 else dec, n, d)
        svm = sparse_svm(c, kernel, np.float32, fp22=fp22, mode=mode)
        svm.setup_data_on_device()
        q = svm.generate_q()
        ret = svm.run_device_kernel(None, np.zeros(n - 1, np.float32), x, 1.0)
        outs.append((q, ret))
        svm.close()
    assert np.all(np.isfinite(outs[0][1]))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("kernel,fp22", [("rbf", False), ("linear", False), ("rbf", True), ("linear", True)])
def test_coo_setup_equals_csr(kernel, fp22):
    """COO triplets in random order (plssvm_mi_setup_coo) == the same matrix as CSR, bit for bit."""
    n, d = 5000, 3000
    csr, _ = datagen.sparse_csr(n, d, 15, seed=9, dtype=np.float32)
    rowptr, col, val = csr[0], csr[1], csr[2]
    row = np.repeat(np.arange(n, dtype=np.int64), np.diff(rowptr))
    perm = np.random.default_rng(2).permutation(col.size)
    x = np.random.default_rng(3).uniform(1, 2, n - 1).astype(np.float32)
    outs = []
    for layout in ("csr", "coo"):
        p = pm.Parameter(kernel, gamma=1.0 / d, real_type=np.float32)
        if layout == "csr":
            p.csr = (rowptr, col, pack_fp22(val) if fp22 else val, n, d)
        else:
            p.coo = (row[perm], col[perm], pack_fp22(val[perm]) if fp22 else val[perm], n, d)
        if fp22:
            p.val_fmt = pm._abi.VAL_FP22
        with pm.CSVM(p) as svm:
            svm.setup_data_on_device()
            q = svm.generate_q()
            outs.append((q, svm.run_device_kernel(None, np.zeros(n - 1, np.float32), x, 1.0)))
    np.testing.assert_array_equal(outs[0][0], outs[1][0])
    np.testing.assert_array_equal(outs[0][1], outs[1][1])


def pack_fp22(v):
    from plssvm_sparse_fp22_amd.fp22 import pack

    return pack(v)


def test_coo_rejects_duplicates_and_bad_indices():
    p = pm.Parameter("rbf", real_type=np.float64)
    p.coo = (np.array([0, 1, 1], np.int64), np.array([2, 0, 0], np.int32), np.ones(3), 3, 4)
    with pm.CSVM(p) as svm, pytest.raises(pm.BackendError, match="duplicate COO entry"):
        svm.setup_data_on_device()
    p.coo = (np.array([0, 5], np.int64), np.array([1, 1], np.int32), np.ones(2), 3, 4)
    with pm.CSVM(p) as svm, pytest.raises(pm.BackendError, match="row index out of range"):
        svm.setup_data_on_device()


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("kernel,shape,sim", [("rbf", (20000, 3000, 20), None), ("polynomial", (6000, 800, 30), None),
                                              ("rbf", (20000, 3000, 20), (1, 3)), ("rbf", (3000, 50, 20), None)])
def test_expansion_row_join_equals_sort_join(kernel, shape, sim, dtype, monkeypatch):
    """The remainder's symmetric rows built per row (the default row join: LDS bitmap of the rows met in
    the row's feature columns, H from a merge of the two rows) against the column-join sort
    (PLSSVM_MI_EXP_JOIN=sort: every incidence generated, radix-sorted, reduced by key): the same pairs
    (info.pairs) and the same K·p overlap sums within a tolerance: the row join's rbf H is the product
    recurrence (no expm1 of s, no cancellation) while the sort join forms phi(s) - sum phi(a_f), so the two H
    agree to fp64 rounding of the cancelling form, not to the last bit (the expansion predict,
    exp_pred_point_kernel, also forms phi(s) - sum phi(a_f) — the same H up to that rounding).
    (3000 x 50 @ 40 %: dense-ish rows whose repeats overflow a pass, so passes are split.) "row" is the
    one-pass join (partners written into fixed slot ranges per row, no count pass), "twopass" the count pass
    + write pass (PLSSVM_MI_EXP_RJ=twopass) — the same H kernel over the same partners, so bit for bit the same
    K·p —
    "smallcap" the one-pass join with 8 slots per row (PLSSVM_MI_EXP_RJ_CAP=8: rows beyond it are redone by
    the two passes with the counted sizes), "capped" the row join limited to one pass per row
    (PLSSVM_MI_EXP_RJ_PMAX=1; default 256) — a rank with a row that needs more passes builds its rows by
    the sort join instead, with the same result."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=17, dtype=np.float64)
    m = n - 1
    x = np.random.default_rng(3).uniform(1, 2, m).astype(dtype)
    out = {}
    envs = {"sort": ("PLSSVM_MI_EXP_JOIN", "sort"), "capped": ("PLSSVM_MI_EXP_RJ_PMAX", "1"),
            "twopass": ("PLSSVM_MI_EXP_RJ", "twopass"), "smallcap": ("PLSSVM_MI_EXP_RJ_CAP", "8")}
    for join in ("row", "sort", "capped", "twopass", "smallcap"):
        for k, _ in envs.values():
            monkeypatch.delenv(k, raising=False)
        if join in envs:
            monkeypatch.setenv(*envs[join])
        with sparse_svm(csr, kernel, dtype, sim=sim, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            assert info["sparse_algo"] == pm._abi.SPARSE_EXPANSION
            out[join] = (svm.kp_part(x, "overlap"), info["pairs"], info["pair_slots"])
    tol = 1e-14 if dtype == np.float64 else 1e-6
    b = out["sort"][0].astype(np.float64)
    for join in ("row", "capped", "twopass", "smallcap"):
        assert out[join][1] == out["sort"][1] and out[join][2] == out["sort"][2], join
        a = out[join][0].astype(np.float64)
        assert np.abs(a - b).max() <= tol * max(np.abs(b).max(), 1e-300), (join, np.abs(a - b).max())
    for join in ("twopass", "smallcap"):
        np.testing.assert_array_equal(out[join][0], out["row"][0], err_msg=join)


@pytest.mark.parametrize("gamma,want_hbytes", [(None, 2), (0.2, 4)])
def test_expansion_bf16_remainder_bound(gamma, want_hbytes, monkeypatch):
    """Remainder storage (expand.hip "H storage"): in a float context H is stored as bfloat16
    when every stored |H_ij| is at most 2^-16 of its pair's kernel value (1 + E(s) for rbf), so rounding H
    (relative error <= 2^-9) moves each pair's term by at most 2^-24 of that kernel value — below the float
    rounding of the kernel value itself. Checked: the default layout is bfloat16 on the BASELINE-like set and
    the real type when the bound fails (large gamma: H comparable to the kernel value); the kernel sums
    sum_j k_ij p_j (all terms positive) of both layouts agree to 2^-20 relative, and the overlap sums to
    2^-9 of sum_j |H_ij| w_j + float rounding."""
    csr, _ = datagen.sparse_csr(20000, 3000, 20, seed=17, dtype=np.float32)
    m = csr[3] - 1
    x = np.random.default_rng(5).uniform(1, 2, m).astype(np.float32)
    out = {}
    for fmt in ("auto", "full"):
        if fmt == "full":
            monkeypatch.setenv("PLSSVM_MI_EXP_HFMT", "full")
        else:
            monkeypatch.delenv("PLSSVM_MI_EXP_HFMT", raising=False)
        with sparse_svm(csr, "rbf", np.float32, gamma=gamma, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            out[fmt] = (info["exp_hbytes"], svm.kp_part(x, "kernel").astype(np.float64),
                        svm.kp_part(x, "overlap").astype(np.float64))
    assert out["full"][0] == 4
    assert out["auto"][0] == want_hbytes
    a, b = out["auto"][1], out["full"][1]
    assert np.all(np.abs(a - b) <= 2.0 ** -20 * np.abs(b)), np.max(np.abs(a - b) / np.abs(b))
    if want_hbytes == 4:  # same layout: bitwise
        np.testing.assert_array_equal(out["auto"][2], out["full"][2])


@pytest.mark.parametrize("rbb,groups,sim", [("auto", "0", None), ("4096", "1", None), ("8192", "3", None),
                                             ("32768", "2", None), ("auto", "0", (1, 3)), ("auto", "0", (2, 8))])
@pytest.mark.parametrize("shape", [(140000, 3000, 20), (150000, 200000, 6)])
def test_expansion_row_flags_equal_row_index(rbb, groups, sim, shape, monkeypatch):
    """Flagged chunks (expand.hip: no per-chunk row index; bit 14 of a chunk's first bfloat16 H marks a row's
    first chunk of a window, rows without partners in a window get a zero dummy chunk, the kernel numbers rows
    by a ballot of the flags) against the indexed 4-slot chunks: the same stored values in the same order, so
    the K·p and its overlap part are equal bit for bit — across accumulator classes, window groups and
    simulated ranks, with three partner windows (m > 2 x 65536), and on a very sparse set (150000 x 200000 @ 6
    per row) where nearly every (row, window) cell is empty (dummies; auto would keep the row index there)."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=23, dtype=np.float32)
    x = np.random.default_rng(9).uniform(-1, 2, n - 1).astype(np.float32)
    if rbb != "auto":
        monkeypatch.setenv("PLSSVM_MI_EXP_RBB", rbb)
        monkeypatch.setenv("PLSSVM_MI_EXP_G", groups)
    out = {}
    for rows in ("index", "flags"):
        monkeypatch.setenv("PLSSVM_MI_EXP_ROWS", rows)
        with sparse_svm(csr, "rbf", np.float32, sim=sim, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            assert info["exp_hbytes"] == 2
            out[rows] = (info["exp_layout"], svm.kp_part(x, "kernel"), svm.kp_part(x, "overlap"))
    assert out["index"][0] == 1 and out["flags"][0] == 2
    np.testing.assert_array_equal(out["flags"][1], out["index"][1])
    np.testing.assert_array_equal(out["flags"][2], out["index"][2])


@pytest.mark.parametrize("rbb,groups,sim", [("auto", "0", None), ("4096", "1", None), ("8192", "3", None),
                                             ("32768", "2", None), ("auto", "0", (1, 3)), ("auto", "0", (2, 8))])
@pytest.mark.parametrize("shape", [(140000, 3000, 20), (150000, 200000, 6), (60000, 1500, 12)])
def test_expansion_row_pairs_equal_row_flags(rbb, groups, sim, shape, monkeypatch):
    """Pair flags (round 5, info exp_layout 4: bit 14 of H0 / H2 marks a row starting at a chunk's slot 0 / 2, cells
    padded to 2 slots instead of 4, a window's stream of a wave padded to whole chunks at its end) against the chunk
    flags: the same stored values and products, the row sums formed as prefix differences per slot pair instead of
    per chunk — equal to 2^-20 of the rows' overlap magnitude (the bfloat16 bound's cancellation, expand.hip), fewer
    slots, across accumulator classes, window groups, simulated ranks, three partner windows, a set whose cells are
    nearly all empty (2-slot dummies) and a small-cell set (60000 x 1500 @ 12: cells of 1-3 entries)."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=23, dtype=np.float32)
    x = np.random.default_rng(9).uniform(-1, 2, n - 1).astype(np.float32)
    if rbb != "auto":
        monkeypatch.setenv("PLSSVM_MI_EXP_RBB", rbb)
        monkeypatch.setenv("PLSSVM_MI_EXP_G", groups)
    out = {}
    for rows in ("flags", "pairs"):
        monkeypatch.setenv("PLSSVM_MI_EXP_ROWS", rows)
        with sparse_svm(csr, "rbf", np.float32, sim=sim, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            assert info["exp_hbytes"] == 2
            out[rows] = (info["exp_layout"], info["pair_slots"], svm.kp_part(x, "kernel").astype(np.float64),
                         svm.kp_part(x, "overlap").astype(np.float64), svm.kp_part(np.abs(x), "overlap").astype(np.float64))
            # bitwise reproducible run to run
            np.testing.assert_array_equal(svm.kp_part(x, "overlap").astype(np.float64), out[rows][3])
    assert out["flags"][0] == 2 and out["pairs"][0] == 4
    assert out["pairs"][1] <= out["flags"][1]
    # scale: the overlap of |x| (plus 2^-10 of its largest row) and the fp32 rounding of the compared values themselves
    # (both are rounded to float once: a row's two results may differ in their last bits)
    mag = np.abs(out["flags"][4]) + 2.0 ** -10 * np.abs(out["flags"][4]).max()
    for q in (2, 3):
        tol = 2.0 ** -20 * mag + 2.0 ** -22 * np.abs(out["flags"][q])
        assert np.all(np.abs(out["pairs"][q] - out["flags"][q]) <= tol), (q, np.max(np.abs(out["pairs"][q] - out["flags"][q]) - tol))


def test_expansion_row_flags_default_and_oracle(oracle):
    """The default layout on a BASELINE-like set is a flagged one (chunk flags, or pair flags where they save >= 3 %
    of the slots), and its K·p equals the oracle (fp32 bar)."""
    csr, _ = datagen.sparse_csr(20000, 3000, 20, seed=17, dtype=np.float32)
    with sparse_svm(csr, "rbf", np.float32, algo="expansion") as svm:
        svm.setup_data_on_device()
        assert svm.info()["exp_layout"] in (2, 4)
    check_sparse_kp(oracle, csr, "rbf", np.float32, algo="expansion")


@pytest.mark.parametrize("rows", ["index", "flags", "pairs"])
def test_expansion_dot2_equals_fma_path(oracle, rows, monkeypatch):
    """The bfloat16 remainder's chunk products as two v_dot2_f32_bf16 instructions (inline assembly with a
    hand-placed hazard wait, expand.hip EXP_DOT2) against the FMA chain of the same kernel
    (PLSSVM_MI_EXP_DOT2=0), in both chunk layouts (row index / row-start flags): a chunk's four H and the four
    partners' w differ in every lane here (seeded real data, distinct rows), so a register mix-up between the
    two halves (the ROCm 7.2 builtin lowering that made the assembly necessary fed the first half's H to both)
    moves the sums far beyond rounding. Bar: the products are exact in fp32 in both paths, only the summation
    of a chunk's four products differs — 2^-20 of the row's overlap magnitude. Both also match the oracle."""
    monkeypatch.setenv("PLSSVM_MI_EXP_ROWS", rows)
    csr, _ = datagen.sparse_csr(30000, 2000, 24, seed=29, dtype=np.float32)
    m = csr[3] - 1
    x = np.random.default_rng(7).uniform(-2, 2, m).astype(np.float32)
    out = {}
    for dot2 in ("1", "0"):
        monkeypatch.setenv("PLSSVM_MI_EXP_DOT2", dot2)
        with sparse_svm(csr, "rbf", np.float32, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            assert info["exp_hbytes"] == 2 and info["exp_layout"] == {"index": 1, "flags": 2, "pairs": 4}[rows], info
            assert info["pairs"] > 100000
            if dot2 == "1" and info["exp_dot2"] == 0:  # built without the dot kernel, nothing to compare
                pytest.skip("libplssvm_mi355x built without EXP_DOT2 (toolchain other than the one it was verified on)")
            assert info["exp_dot2"] == (1 if dot2 == "1" else 0), info
            out[dot2] = (svm.kp_part(x, "overlap").astype(np.float64), svm.kp_part(np.abs(x), "overlap").astype(np.float64))
    a, b = out["1"][0], out["0"][0]
    mag = np.abs(out["0"][1])
    scale = np.maximum(mag, np.abs(b)) + 2.0 ** -10 * mag.max()
    err = np.abs(a - b) / scale
    assert err.max() <= 2.0 ** -20, err.max()
    info = check_sparse_kp(oracle, csr, "rbf", np.float32, algo="expansion")
    assert info["exp_hbytes"] == 2


@pytest.mark.parametrize("kernel,dtype,algo,fp22", [("rbf", np.float32, "expansion", False), ("rbf", np.float32, "expansion", True),
                                                    ("rbf", np.float64, "expansion", False),
                                                    ("polynomial", np.float64, "pattern", False),
                                                    ("rbf", np.float32, "onthefly", False), ("rbf", np.float64, "dense", False),
                                                    ("linear", np.float64, "auto", False), ("linear", np.float32, "auto", True)])
def test_csc_device_equals_host(kernel, dtype, algo, fp22, monkeypatch):
    """The setup's CSC (colptr, rows ascending per column, values, each CSR entry's CSC position) sorted on the device
    (the default: a stable radix sort by column) and by the host counting sort (PLSSVM_MI_CSC=host, the path for
    nnz >= 2^31): the same arrays, so every structure built from them and every K·p is bit for bit the same —
    on a ragged set with empty rows, empty columns and one long row, for every sparse path (kernel expansion with
    its row join, the Gram pattern's column join and its incidence split, on the fly, densified, factored linear
    SELL plans) and FP22 input; and the device sort failing out of memory (PLSSVM_MI_CSC=oom) falls back to the
    host sort with the same result."""
    n, d = 4000, 1500
    rng = np.random.default_rng(29)
    rows = []
    for i in range(n):
        k = 0 if i % 97 == 5 else (200 if i == 1234 else int(rng.integers(1, 30)))
        cols = np.sort(rng.choice(d - 100, size=k, replace=False)) if k else np.zeros(0, np.int64)  # columns >= 1400 empty
        rows.append(cols)
    rowptr = np.zeros(n + 1, dtype=np.int64)
    rowptr[1:] = np.cumsum([len(c) for c in rows])
    col = np.concatenate(rows).astype(np.int32)
    val = rng.uniform(0.05, 1.0, col.size)
    csr = (rowptr, col, val, n, d)
    m = n - 1
    x = np.random.default_rng(7).uniform(1, 2, m).astype(dtype)
    out = {}
    # "oom": the device sort runs out of memory after its first temporaries (test hook) and setup falls back to the
    # host counting sort — the same arrays again
    for where in ("device", "host", "oom"):
        if where != "device":
            monkeypatch.setenv("PLSSVM_MI_CSC", where)
        else:
            monkeypatch.delenv("PLSSVM_MI_CSC", raising=False)
        with sparse_svm(csr, kernel, dtype, fp22=fp22, algo=algo) as svm:
            svm.setup_data_on_device()
            svm.generate_q()
            info = svm.info()
            ret = np.zeros(m, dtype=dtype)
            svm.run_device_kernel(None, ret, x, 1.0)
            out[where] = (ret, info["sparse_algo"], info["pairs"], info["pair_slots"])
    np.testing.assert_array_equal(out["device"][0], out["host"][0])
    assert out["device"][1:] == out["host"][1:]
    np.testing.assert_array_equal(out["oom"][0], out["host"][0])
    assert out["oom"][1:] == out["host"][1:]


def test_expansion_row_join_column_split_table(monkeypatch):
    """More rows than one bitmap pass of the row join (2^20 partner rows): every row takes two passes over its
    columns, which start at the same partner rows for every row, so the setup finds those positions in each column
    once (exp_colsplit_kernel) instead of two binary searches per feature and pass. PLSSVM_MI_EXP_COLSPLIT=0 keeps
    the searches: the same pairs and bit for bit the same K·p (1.1M rows x 20k features, 4 per row)."""
    csr, _ = datagen.sparse_csr(1_100_001, 20000, 4, seed=41, dtype=np.float32)
    m = csr[3] - 1
    x = np.random.default_rng(9).uniform(1, 2, m).astype(np.float32)
    out = {}
    for mode in ("table", "search"):
        if mode == "search":
            monkeypatch.setenv("PLSSVM_MI_EXP_COLSPLIT", "0")
        else:
            monkeypatch.delenv("PLSSVM_MI_EXP_COLSPLIT", raising=False)
        with sparse_svm(csr, "rbf", np.float32, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            out[mode] = (svm.kp_part(x, "overlap"), info["pairs"], info["pair_slots"])
    assert out["table"][1:] == out["search"][1:] and out["table"][1] > 0
    np.testing.assert_array_equal(out["table"][0], out["search"][0])


@pytest.mark.parametrize("kernel,dtype,shape", [("rbf", np.float32, (140000, 3000, 20)), ("rbf", np.float64, (20000, 2000, 16)),
                                                ("polynomial", np.float64, (3000, 50, 20)),
                                                ("rbf", np.float32, (1_100_001, 20000, 4))])
def test_expansion_lower_triangle_join_bitwise(kernel, dtype, shape, monkeypatch):
    """The lower-triangle row join (round 5: each row joins only its partners j < i — every column read up to the
    row's own entry — H once per unordered pair, the upper lists by a stable radix sort of the pairs by partner)
    against the full row join (PLSSVM_MI_EXP_LT=0): the same symmetric rows, H bit for bit (H_ij = H_ji), so the same
    pairs, slots and K·p bits — incl. dense-ish rows (3000 x 50 @ 40 %) and 1.1M rows, whose lower lists span two
    bitmap passes (the column split table below row i, row i's own CSC position as the last bound)."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=31, dtype=dtype)
    x = np.random.default_rng(4).uniform(-1, 2, n - 1).astype(dtype)
    out = {}
    for lt in ("1", "0"):
        monkeypatch.setenv("PLSSVM_MI_EXP_LT", lt)
        with sparse_svm(csr, kernel, dtype, algo="expansion", coef0=1.0) as svm:
            svm.setup_data_on_device()
            info = svm.info()
            assert info["sparse_algo"] == pm._abi.SPARSE_EXPANSION
            out[lt] = (info["exp_lt"], info["pairs"], info["pair_slots"], info["exp_hbytes"],
                       svm.kp_part(x, "kernel"), svm.kp_part(x, "overlap"))
    assert out["1"][0] == 1 and out["0"][0] == 0
    assert out["1"][1:4] == out["0"][1:4]
    np.testing.assert_array_equal(out["1"][4], out["0"][4])
    np.testing.assert_array_equal(out["1"][5], out["0"][5])


@pytest.mark.parametrize("shape", [(20000, 3000, 20), (3000, 50, 20)])
def test_expansion_float_h_equals_fp64_h(shape, monkeypatch):
    """Round 5: in a float context the rbf remainder H is evaluated in float (exp_rowjoin_h_kernel<float, true>: the
    product recurrence of the shared features' expm1 has no cancellation) — against the fp64 evaluation
    (PLSSVM_MI_EXP_H64=1): the same pairs and slots, the same H storage decision, and the overlap sums within float
    rounding of their magnitude (2^-20 of the |x| overlap; the dense-ish 3000 x 50 @ 40 % set shares up to ~20 features
    per pair, so H there is far from the two-feature E_a E_b)."""
    n, d, k = shape
    csr, _ = datagen.sparse_csr(n, d, k, seed=29, dtype=np.float32)
    x = np.random.default_rng(5).uniform(-1, 2, n - 1).astype(np.float32)
    out = {}
    for h64 in ("0", "1"):
        monkeypatch.setenv("PLSSVM_MI_EXP_H64", h64)
        with sparse_svm(csr, "rbf", np.float32, algo="expansion") as svm:
            svm.setup_data_on_device()
            info = svm.info()
            out[h64] = (info["pairs"], info["pair_slots"], info["exp_hbytes"], svm.kp_part(x, "overlap").astype(np.float64),
                        svm.kp_part(np.abs(x), "overlap").astype(np.float64))
    assert out["0"][:3] == out["1"][:3]
    mag = np.abs(out["1"][4]) + 2.0 ** -10 * np.abs(out["1"][4]).max()
    dev = np.abs(out["0"][3] - out["1"][3])
    assert np.all(dev <= 2.0 ** -20 * mag + 2.0 ** -22 * np.abs(out["1"][3])), dev.max()
