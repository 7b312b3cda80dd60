"""The engine's multi-rank path executed for real on one GPU (A10 partial).

Two processes (tests/mr_worker.py), one context each on the box's GPU, form a world-2 group with
plssvm_mi_comm_init_host: each exchange is the reference's own device_reduction transport
(gpu_csvm.cpp:366-386: synchronise, D2H, combine on the host, H2D) with the host combine done over
gloo (all-gather, sum in rank order). Everything else is the real multi-GPU path, identical to the
RCCL one: the partition of the implicit matrix (super-block ranges / row blocks / row chunks), each
rank's share of the K·p kernels, the exchange, and the replicated device-resident CG.
(RCCL itself refuses two ranks on one device; its collective calls are covered by the one-rank
RCCL group in test_gpu_parity.py::test_single_rank_rccl_group.)

Both ranks' q, K·p (add = -1, +1), kernel part, CG delta trace, alpha and bias are compared with the
oracle (fp64: K·p 1e-12 of max, trace 1e-6 per iteration, alpha 1e-9 of max; fp32/FP22: K·p 1e-4 vs
the fp32 oracle, and trace / alpha / bias vs the fp64 oracle within 1e-3 / 2e-2 or twice the fp32
oracle's own distance from the fp64 one, whichever is larger) and with each other (bit for bit:
the CG is replicated).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from mr_cases import ALGO, BUDGET, CASES, LONG_ROWS, UNSTORED, case_data

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def run_group(case, world, tmp_path):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="4")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mr_worker.py"), case, str(r), str(world), str(port),
                               str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(world)]
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
    return [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("case", sorted(CASES))
def test_world2_group_matches_oracle(oracle, case, tmp_path):
    layout, kernel, kp_mode, dtype, imax = CASES[case]
    world = 2
    res = run_group(case, world, tmp_path)
    data, y, d = case_data(case)
    if "X" in data:
        od = oracle.Data(data["X"], dtype=dtype)
    else:
        rowptr, col, val, n, dd = data["csr"]
        if layout == "fp22":
            val = oracle.fp22_unpack(oracle.fp22_pack(val), val.size)
        od = oracle.Data(rowptr=rowptr, col=col, val=val.astype(dtype), n=n, d=dd, dtype=dtype)
    dt = np.dtype(dtype).type
    args = dict(degree=3, gamma=dt(1.0 / d), coef0=dt(1.0 if kernel == "polynomial" else 0.0))
    q_ref = oracle.generate_q(kernel, od, **args)
    m = od.n - 1
    x = np.random.default_rng(21).uniform(1, 2, m).astype(dtype)
    f64 = dtype == np.float64
    ktol, ttol, atol_ = (1e-12, 1e-6, 1e-9) if f64 else (1e-4, 1e-3, 2e-2)
    ref = oracle.learn(kernel, od, y, imax=imax, **args)
    if not f64:
        # fp32: compare with the fp64 oracle on the same (fp32-representable) inputs; the bar is the
        # larger of the fixed fp32 tolerance and twice the fp32 oracle's own distance from it (an fp32 CG
        # that removes most of the residual in one step is rounding-bound: here the fp32 oracle's
        # alpha_m is 5 % off the fp64 one)
        od64 = oracle.Data(rowptr=od.rowptr, col=od.col, val=od.X.astype(np.float64), n=od.n, d=od.d,
                           dtype=np.float64) if od.csr else oracle.Data(od.X.astype(np.float64))
        args64 = {k: (np.float64(v) if k != "degree" else v) for k, v in args.items()}
        ref32 = ref
        ref = oracle.learn(kernel, od64, y.astype(np.float64), imax=imax, **args64)
        n8 = min(len(ref32["trace"]), len(ref["trace"]))
        ttol = max(ttol, 2 * float(np.abs(ref32["trace"][:n8] / ref["trace"][:n8] - 1).max()))
        amax = float(np.abs(ref["alpha"]).max())
        atol_ = max(atol_, 2 * float(np.abs(ref32["alpha"] - ref["alpha"]).max()) / amax)
        atol_m = 2 * abs(float(ref32["alpha"][m]) - float(ref["alpha"][m]))

    # the split is real: every rank owns a non-empty, disjoint part of the work
    if layout == "dense" and kp_mode != "factored":
        assert sum(int(r["tiles_local"]) for r in res) == int(res[0]["tiles_total"])
        assert all(int(r["tiles_local"]) > 0 for r in res)
    if layout != "dense" and kernel != "linear" and case not in UNSTORED:  # stored pairs (the on-the-fly path stores none)
        assert all(int(r["pairs"]) > 0 for r in res)
    # one K·p algorithm for the whole group, also when the ranks' own estimates straddle the budget
    assert len({int(r["sparse_algo"]) for r in res}) == 1, [int(r["sparse_algo"]) for r in res]
    # one H storage for the whole group (the sharded K·p gathers bfloat16 or real w by it): a rank whose rows
    # cannot take the bfloat16 bound (LONG_ROWS: the column-join sort) keeps both ranks on real H
    assert len({int(r["exp_hbytes"]) for r in res}) == 1, [int(r["exp_hbytes"]) for r in res]
    if case in LONG_ROWS:
        assert int(res[0]["exp_hbytes"]) == np.dtype(dtype).itemsize
    if case in BUDGET:
        import plssvm_sparse_fp22_amd as pm

        assert int(res[0]["sparse_algo"]) in (pm._abi.SPARSE_ONTHEFLY, pm._abi.SPARSE_DENSE)
    for rank, r in enumerate(res):
        assert int(r["world"]) == world
        np.testing.assert_allclose(r["q"], q_ref, rtol=ktol, atol=ktol * np.abs(q_ref).max())
        for add, key in ((-1.0, "kp_minus"), (1.0, "kp_plus")):
            want = oracle.kp(kernel, od, q_ref, dt(r["QA"]), dt(1.0), add, x, **args)
            np.testing.assert_allclose(r[key], want, rtol=0, atol=ktol * np.abs(want).max(),
                                       err_msg=f"{case} rank {rank} add={add}")
        assert int(r["iters"]) == ref["iters"], (case, rank, int(r["iters"]), ref["iters"])
        # fp32: compare the trace while the residual is above the fp32 rounding floor (delta/delta0 >= 1e-6,
        # i.e. |r|/|r0| >= 1e-3); below it every fp32 CG, the reference's included, follows its own rounding
        live = np.ones(len(ref["trace"]), bool) if f64 else ref["trace"] / ref["trace"][0] >= 1e-6
        np.testing.assert_allclose(r["trace"][:len(live)][live], ref["trace"][live], rtol=ttol,
                                   err_msg=f"{case} rank {rank}")
        np.testing.assert_allclose(r["alpha"][:m], ref["alpha"][:m], rtol=atol_, atol=atol_ * np.abs(ref["alpha"]).max())
        # alpha_m = -sum(alpha) (csvm.cpp:258) carries the summed error of all m alphas
        tol_m = atol_ * np.abs(ref["alpha"]).max() if f64 else max(atol_ * np.abs(ref["alpha"]).max(), atol_m)
        assert abs(float(r["alpha"][m]) - float(ref["alpha"][m])) <= tol_m, (case, rank)
        tol_b = atol_ * max(1.0, abs(float(ref["bias"]))) if f64 else max(atol_ * max(1.0, abs(float(ref["bias"]))),
                                                                         2 * abs(float(ref32["bias"]) - float(ref["bias"])))
        assert abs(float(r["bias"]) - float(ref["bias"])) <= tol_b, (case, rank)
    # replicated CG: identical bits on every rank
    for key in ("kp_plus", "kpart", "alpha", "trace"):
        np.testing.assert_array_equal(res[0][key], res[1][key])
