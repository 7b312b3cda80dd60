"""One process driving several GPUs: the csvm<T> adapter's device group (include/plssvm_mi355x_group.hpp).

The reference's hip::csvm<T>(params) takes every visible GPU in one process (src/plssvm/backends/HIP/csvm.hip.cpp:
53-55; one OpenMP thread per device, gpu_csvm.cpp:136-155). plssvm-train now does the same: one host thread and one
context per GPU, joined in one row-block group. On the one-GPU box the group runs as two (or three) contexts on
device 0 over the in-process host exchange (RCCL refuses two ranks on one GPU): `--devices 0,0`.

* plssvm-train --devices 0,0 reproduces the reference's 5x4 model fixture and the oracle's learn() on config 1
  (alphas 1e-9, the printed residual curve 1e-6), dense and --sparse, and writes the same model as one device up to
  the reduction order of the split (1e-12);
* the failure protocol (tests/group_check.cpp): a rank failing before its collective, or inside the library, while
  its peer waits in the exchange ends both calls — the failing rank's code and message reach the caller, the
  waiting rank returns PLSSVM_MI_ERR_RCCL — within seconds, the group then refuses calls and is destroyed cleanly;
* without a failure both ranks' K·p are the same bits.
"""
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_path
from test_cli import EXE, TRACE_RE, _write_libsvm, read_model

pytestmark = pytest.mark.gpu
CHECK = os.path.join(ROOT, "plssvm_sparse_fp22_amd", "bin", "plssvm-group-check")


def _train(path, out, *extra):
    return subprocess.run([EXE, *extra, path, str(out)], capture_output=True, text=True, check=True, timeout=120)


def _key(row):  # a data row as the model file prints it ("{:e}" per feature)
    return tuple(float(f"{v:e}") for v in row)


def _alpha_by_sv(model):
    return {_key(sv): a for sv, a in zip(model["SV"], model["alpha"])}


@pytest.mark.parametrize("extra", [[], ["--sparse"]])
@pytest.mark.parametrize("devices", ["0,0", "0,0,0"])
def test_train_group_reproduces_golden_model(tmp_path, devices, extra):
    r = _train(fixture_path("5x4.libsvm"), tmp_path / "g.model", "--devices", devices, *extra)
    assert f"Found {devices.count(',') + 1} HIP device(s):" in r.stdout
    got, want = read_model(str(tmp_path / "g.model")), read_model(fixture_path("5x4.libsvm.model"))
    assert abs(got["rho"] - want["rho"]) <= 1e-9 * abs(want["rho"])
    g, w = _alpha_by_sv(got), _alpha_by_sv(want)
    assert g.keys() == w.keys()
    for k in w:
        assert abs(g[k] - w[k]) <= 1e-9 * max(1.0, abs(w[k]))


@pytest.mark.parametrize("kernel", ["0", "2"])
@pytest.mark.parametrize("extra", [[], ["--sparse"]])
def test_train_group_config1_equals_oracle_and_one_device(tmp_path, oracle, kernel, extra):
    from plssvm_sparse_fp22_amd import datagen

    X, y = datagen.blobs(500, 4, seed=1)
    path = str(tmp_path / "c1.libsvm")
    _write_libsvm(path, X, y)
    r2 = _train(path, tmp_path / "two.model", "-t", kernel, "--devices", "0,0", *extra)
    _train(path, tmp_path / "one.model", "-t", kernel, "--device", "0", "-q", *extra)
    kname = "linear" if kernel == "0" else "rbf"
    ref = oracle.learn(kname, oracle.Data(np.ascontiguousarray(X)), y, eps=1e-3)
    lines = TRACE_RE.findall(r2.stdout)
    assert len(lines) == ref["iters"] > 0
    for k, line in enumerate(lines):
        assert abs(float(line[2]) - ref["trace"][k]) <= 1e-6 * ref["trace"][k]
    two, one = read_model(str(tmp_path / "two.model")), read_model(str(tmp_path / "one.model"))
    a2, a1 = _alpha_by_sv(two), _alpha_by_sv(one)
    # the model lists support vectors by label; map the oracle's alphas through the data rows
    aref = {_key(X[i]): ref["alpha"][i] for i in range(X.shape[0])}
    assert a2.keys() == aref.keys()
    for k, v in aref.items():
        assert abs(a2[k] - v) <= 1e-9 * max(1.0, abs(v)), (k, a2[k], v)
        assert abs(a2[k] - a1[k]) <= 1e-12 * max(1.0, abs(v))
    assert abs(two["rho"] - ref["rho"]) <= 1e-9 * max(1.0, abs(ref["rho"]))


def _check(mode):
    out = subprocess.run([CHECK, mode], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.stdout, out.stderr[-2000:])
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_group_ranks_equal_without_failure():
    res = _check("none")
    assert res["world"] == 2 and res["host"] == 1
    assert res["rc0"] == 0 and res["rc1"] == 0
    assert res["ranks"] == "equal" and np.isfinite(res["sum"])


@pytest.mark.parametrize("mode,code,text", [("early", -6, ""), ("library", -1, "unknown")])
def test_group_failure_raises_on_every_rank_without_hanging(mode, code, text):
    res = _check(mode)
    assert res["world"] == 2 and res["host"] == 1
    assert res["fail_rank"] == 1 and res["fail_code"] == code, res
    assert text in res["msg"].lower(), res
    assert res["rc1"] == code
    assert res["rc0"] == -3, res  # the waiting rank was released from its exchange: PLSSVM_MI_ERR_RCCL
    assert res["refused"] == 1
    assert res["seconds"] < 60
