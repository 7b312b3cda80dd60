"""The one-reduction CG (Chronopoulos-Gear; PLSSVM_MI_OPT_CG_VARIANT, blas1.hip cg1_*) judged with the long residual
curves: the same 61-iteration windows, across the run-49 explicit residual, on the systems where
the OpenMP oracle reproduces itself to 1e-9 (tests/long_trace_cases.py, fixtures tests/golden/cg_traces_long/).

The recurrence differs from the reference's solver_CG (OpenMP/csvm.cpp:82-170) — the product Q~r instead of Q~d,
s = Q~d by a recurrence, r.r and r.Q~r after ONE collective — so the curve it must match is the oracle's, at the
reference recurrence's own bars: every delta_k (k <= 60) within 1e-6 (fp64) / 1e-3 of the fp64 oracle (fp32), alphas
after 70 iterations within 1e-6 / 2e-2. Three transports:

* one GPU, no group (G = 1): every long-trace case;
* a one-rank RCCL group with the sharded CG (PLSSVM_MI_SHARD=1): the collective path, through RCCL on this GPU;
* a world-2 host-staged group (tests/cg1_worker.py, two processes on this GPU over gloo): two ranks' partials
  gathered and summed in rank order, the variant taken by auto (a sharded group of several ranks).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import long_trace_cases as lc
import plssvm_sparse_fp22_amd as pm

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
MANIFEST = json.load(open(os.path.join(lc.VECTORS, "manifest.json")))
WINDOW = 61


def _svm(s, name, monkeypatch, **kw):
    kernel, dtype, _, _, _, _, algo, env, _ = lc.CASES[name]
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    p = pm.Parameter(kernel, degree=3, gamma=float(s["gamma"]), coef0=float(s["coef0"]), cost=s["cost"],
                     epsilon=s["eps"], real_type=dtype)
    if "X" in s:
        p.data = s["X"]
    else:
        p.csr = s["csr"]
    p.labels = s["y"]
    return pm.CSVM(p, sparse_algo=algo, **kw)


def _judge(name, s, t, alpha, iters):
    g = np.load(os.path.join(lc.VECTORS, name + ".npz"))
    f64 = s["dtype"] == np.float64
    assert iters == lc.IMAX == int(g["iters"][0])
    ref = g["trace"] if f64 else g["trace64"]
    aref = (g["alpha"] if f64 else g["alpha64"]).astype(np.float64)
    R = 1e-6 if f64 else 1e-3
    dev = np.abs(np.asarray(t, np.float64)[:WINDOW] / ref[:WINDOW] - 1)
    m = lc.N - 1
    adev = float(np.abs(np.asarray(alpha, np.float64)[:m] - aref[:m]).max()) / float(np.abs(aref[:m]).max())
    print(f"\n{name}: one-reduction CG vs oracle over {WINDOW} iterations: max {dev.max():.3e} (bar {R:g}); "
          f"alpha {adev:.3e}")
    assert np.all(dev <= R), (name, np.nonzero(dev > R)[0][:5], dev.max())
    assert adev <= (1e-6 if f64 else 2e-2), (name, adev)


@pytest.mark.parametrize("name", sorted(lc.CASES))
def test_one_reduction_cg_long_trace(name, monkeypatch):
    s = lc.load(name)
    assert lc.input_hash(s) == MANIFEST[name]["input_sha256"]
    with _svm(s, name, monkeypatch, cg_variant="one_reduction") as svm:
        svm.learn(imax=lc.IMAX)
        _judge(name, s, svm.trace, svm.alpha, svm.iters)


@pytest.mark.parametrize("name", sorted(lc.CASES))
def test_one_reduction_cg_long_trace_rccl_group(name, monkeypatch):
    s = lc.load(name)
    monkeypatch.setenv("PLSSVM_MI_SHARD", "1")
    with _svm(s, name, monkeypatch, cg_variant="one_reduction", uid=pm.unique_id()) as svm:
        svm.learn(imax=lc.IMAX)
        _judge(name, s, svm.trace, svm.alpha, svm.iters)


def _free_port():
    so = socket.socket()
    so.bind(("127.0.0.1", 0))
    port = so.getsockname()[1]
    so.close()
    return port


@pytest.mark.parametrize("name", sorted(lc.CASES))
def test_one_reduction_cg_long_trace_world2(name, tmp_path):
    s = lc.load(name)
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    variant = "auto" if "csr" in s else "one_reduction"  # dense groups replicate the CG: auto keeps the reference's
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "cg1_worker.py"), name, str(r), "2", str(port),
                               str(tmp_path), variant], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{outs[r][-3000:]}"
    res = [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(2)]
    np.testing.assert_array_equal(res[0]["trace"], res[1]["trace"])
    np.testing.assert_array_equal(res[0]["alpha"], res[1]["alpha"])
    _judge(name, s, res[0]["trace"], res[0]["alpha"], int(res[0]["iters"]))
