"""C-ABI edge cases and the centered finalize's switching logic.

* A NULL rowptr (n > 1) must come back as PLSSVM_MI_ERR_ARG with the reference's message, not a crash.
* The centered rank-1 finalize (`plssvm_mi_info.centered`) is used only while the device q is the
  engine's own k(x_i, x_m): a caller's different q takes the plain finalize, and a caller's QA_cost
  (plssvm_mi_set_qa_cost) keeps its difference from k_mm + 1/C. Each of the three cases is compared with
  PLSSVM_MI_CTR=0 (the plain finalize throughout) and with the fp64 oracle's Q~p for the same q and QA_cost, at the
  fp32 bar (1e-4 of max|Q~p|), for rbf and poly on the kernel expansion. learn() is compared the same way.
"""
import ctypes

import numpy as np
import pytest

import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import _abi, datagen

pytestmark = pytest.mark.gpu


def test_setup_csr_null_rowptr_is_an_error():
    lib = _abi.lib()
    ctx = ctypes.c_void_p()
    assert lib.plssvm_mi_create(4, 2, 3, 0.1, 0.0, 1.0, 0, ctypes.byref(ctx)) == 0
    try:
        col = (ctypes.c_int32 * 4)(0, 1, 0, 1)
        val = (ctypes.c_float * 4)(1, 2, 3, 4)
        rc = lib.plssvm_mi_setup_csr(ctx, None, col, val, 0, 3, 2)
        assert rc == -1, rc  # PLSSVM_MI_ERR_ARG
        assert b"empty" in lib.plssvm_mi_last_error(ctx).lower()
        rc = lib.plssvm_mi_setup_coo(ctx, None, col, val, 0, 4, 3, 2)
        assert rc < 0
    finally:
        lib.plssvm_mi_destroy(ctx)


def _svm(csr, kernel, dtype):
    rowptr, col, val, n, d = csr
    p = pm.Parameter(kernel, gamma=1.0 / d, coef0=0.5, real_type=dtype)
    p.csr = (rowptr, col, val.astype(dtype), n, d)
    return pm.CSVM(p)


@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_centered_finalize_switching(oracle, kernel, monkeypatch):
    dt = np.float32
    csr, y = datagen.sparse_csr(4000, 3000, 12, seed=21, dtype=dt)
    rowptr, col, val, n, d = csr
    m = n - 1
    data64 = oracle.Data(rowptr=rowptr, col=col, val=val.astype(dt).astype(np.float64), n=n, d=d, dtype=np.float64)
    g = float(dt(1.0 / d))
    q64 = oracle.generate_q(kernel, data64, gamma=g, coef0=0.5)
    rng = np.random.default_rng(5)
    pv = rng.uniform(1, 2, m).astype(dt)
    qpert = (q64 * (1 + 1e-3 * rng.standard_normal(m))).astype(dt)
    res = {}
    for ctr in ("1", "0"):
        monkeypatch.setenv("PLSSVM_MI_CTR", ctr)
        with _svm(csr, kernel, dt) as svm:
            svm.setup_data_on_device()
            qg = svm.generate_q()
            qa = float(svm.QA_cost)
            out = {}
            out["gen"] = svm.run_device_kernel(None, np.zeros(m, dt), pv, 1.0).astype(np.float64)
            assert svm.info()["centered"] == (1 if ctr == "1" else 0)
            out["caller_q"] = svm.run_device_kernel(qpert, np.zeros(m, dt), pv, 1.0).astype(np.float64)
            assert svm.info()["centered"] == 0  # a q other than the generated one: the plain finalize
            svm.run_device_kernel(qg, np.zeros(m, dt), pv, 1.0)  # the generated q again: centered again
            assert svm.info()["centered"] == (1 if ctr == "1" else 0)
            svm.set_QA_cost(qa + 0.25)
            out["qa"] = svm.run_device_kernel(None, np.zeros(m, dt), pv, 1.0).astype(np.float64)
            res[ctr] = (out, qa)
    qa = res["1"][1]
    want = {
        "gen": oracle.kp(kernel, data64, q64, qa, 1.0, 1.0, pv.astype(np.float64), gamma=g, coef0=0.5),
        "caller_q": oracle.kp(kernel, data64, qpert.astype(np.float64), qa, 1.0, 1.0, pv.astype(np.float64), gamma=g,
                              coef0=0.5),
        "qa": oracle.kp(kernel, data64, q64, qa + 0.25, 1.0, 1.0, pv.astype(np.float64), gamma=g, coef0=0.5),
    }
    for case, w in want.items():
        tol = 1e-4 * np.abs(w).max()
        for ctr in ("1", "0"):
            err = np.abs(res[ctr][0][case] - w).max()
            assert err <= tol, (kernel, case, ctr, err / np.abs(w).max())
        assert np.abs(res["1"][0][case] - res["0"][0][case]).max() <= tol, (kernel, case)


@pytest.mark.parametrize("kernel", ["rbf", "polynomial"])
def test_centered_learn_equals_plain(oracle, kernel, monkeypatch):
    dt = np.float32
    csr, y = datagen.sparse_csr(3000, 2000, 10, seed=22, dtype=dt)
    rowptr, col, val, n, d = csr
    data64 = oracle.Data(rowptr=rowptr, col=col, val=val.astype(dt).astype(np.float64), n=n, d=d, dtype=np.float64)
    ref = oracle.learn(kernel, data64, y.astype(np.float64), eps=1e-3, imax=30, gamma=float(dt(1.0 / d)), coef0=0.5)
    got = {}
    for ctr in ("1", "0"):
        monkeypatch.setenv("PLSSVM_MI_CTR", ctr)
        with _svm(csr, kernel, dt) as svm:
            svm.params.labels = y
            svm.learn(imax=30)
            got[ctr] = np.asarray(svm.alpha, dtype=np.float64)
    scale = np.abs(ref["alpha"]).max()
    for ctr in ("1", "0"):
        assert np.abs(got[ctr] - ref["alpha"]).max() <= 2e-2 * scale, (kernel, ctr)


@pytest.mark.parametrize("kernel", ["rbf", "linear"])
def test_graph_replay_off_equals_on(kernel, monkeypatch):
    """PLSSVM_MI_GRAPH=0 launches every CG iteration instead of replaying captured 50-iteration blocks: the same
    kernels in the same order, so learn() gives the same bits (imax = 120 crosses two captured blocks)."""
    csr, y = datagen.sparse_csr(3000, 1500, 10, seed=23, dtype=np.float64)
    out = {}
    for g in ("1", "0"):
        monkeypatch.setenv("PLSSVM_MI_GRAPH", g)
        rowptr, col, val, n, d = csr
        p = pm.Parameter(kernel, gamma=1.0 / d, real_type=np.float64, epsilon=1e-30, cost=1e3)
        p.csr = csr
        p.labels = y
        with pm.CSVM(p) as svm:
            svm.learn(imax=120)
            out[g] = (np.asarray(svm.trace).copy(), svm.alpha.copy(), svm.iters)
    assert out["1"][2] == out["0"][2]
    np.testing.assert_array_equal(out["1"][0], out["0"][0])
    np.testing.assert_array_equal(out["1"][1], out["0"][1])


def test_setup_timing_lines(capfd, monkeypatch):
    """PLSSVM_MI_TIMING=1 prints the setup's phase times to stderr ("[plssvm_mi] <phase> <seconds>")."""
    monkeypatch.setenv("PLSSVM_MI_TIMING", "1")
    csr, y = datagen.sparse_csr(3000, 1500, 10, seed=24, dtype=np.float32)
    with _svm(csr, "rbf", np.float32) as svm:
        svm.setup_data_on_device()
    err = capfd.readouterr().err
    assert "[plssvm_mi]" in err and "expansion" in err, err[-2000:]
