"""plssvm-train (C++ host executable over the C ABI): the reference's CLI smoke test
(`plssvm-train --help`, tests/CMakeLists.txt:115-116) on CPU, and the golden 5x4 model on the GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT, fixture_path

EXE = os.path.join(ROOT, "plssvm_sparse_fp22_amd", "bin", "plssvm-train")


def test_help():
    out = subprocess.run([EXE, "--help"], capture_output=True, text=True, check=True).stdout
    for flag in ("--kernel_type", "--degree", "--gamma", "--coef0", "--cost", "--epsilon", "--backend", "--quiet"):
        assert flag in out


def test_bad_backend_and_missing_input():
    r = subprocess.run([EXE, "-b", "cuda", fixture_path("5x4.libsvm")], capture_output=True, text=True)
    assert r.returncode != 0 and "backend" in r.stderr
    r = subprocess.run([EXE], capture_output=True, text=True)
    assert r.returncode != 0


def read_model(path):
    from plssvm_sparse_fp22_amd.io import parse_model

    return parse_model(path)


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--sparse"]])
def test_train_reproduces_golden_model(tmp_path, extra):
    out = tmp_path / "5x4.model"
    subprocess.run([EXE, "-q", *extra, fixture_path("5x4.libsvm"), str(out)], check=True)
    got, want = read_model(str(out)), read_model(fixture_path("5x4.libsvm.model"))
    assert got["kernel"] == "linear" and got["nr_sv"] == [2, 3]
    assert abs(got["rho"] - want["rho"]) <= 1e-9 * abs(want["rho"])
    # same support vectors with the same alphas (the reference's order of negatives follows OpenMP threads)
    key = lambda sv: tuple(np.round(sv, 5))
    g = {key(sv): a for sv, a in zip(got["SV"], got["alpha"])}
    w = {key(sv): a for sv, a in zip(want["SV"], want["alpha"])}
    assert g.keys() == w.keys()
    for k in w:
        assert abs(g[k] - w[k]) <= 1e-9 * max(1.0, abs(w[k]))
    head = open(out).read().splitlines()[:8]
    assert head[0] == "svm_type c_svc" and head[1] == "kernel_type linear" and head[-1] == "SV"


PRED = os.path.join(ROOT, "plssvm_sparse_fp22_amd", "bin", "plssvm-predict")


def test_predict_help_and_missing_files():
    out = subprocess.run([PRED, "--help"], capture_output=True, text=True, check=True).stdout
    assert "test_file model_file [output_file]" in out
    for flag in ("--backend", "--target_platform", "--quiet"):
        assert flag in out
    r = subprocess.run([PRED, fixture_path("500x200.libsvm.test")], capture_output=True, text=True)
    assert r.returncode != 0 and "missing model file" in r.stderr
    r = subprocess.run([PRED, "-b", "cuda", fixture_path("500x200.libsvm.test"), fixture_path("500x200.libsvm.rbf.model")],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "backend" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("extra", [[], ["--sparse"]])
@pytest.mark.parametrize("kernel", ["linear", "polynomial", "rbf"])
def test_predict_reproduces_reference_prediction_file(tmp_path, kernel, extra):
    """tests/data/models/500x200.libsvm.<kernel>.model on tests/data/libsvm/500x200.libsvm.test gives the
    reference's tests/data/predict/500x200.libsvm.predict line for line (main_predict.cpp:80 writes
    fmt::join(labels, "\n") without a final newline; the fixture file has one)."""
    out = tmp_path / "p.predict"
    r = subprocess.run([PRED, *extra, fixture_path("500x200.libsvm.test"), fixture_path(f"500x200.libsvm.{kernel}.model"),
                        str(out)], capture_output=True, text=True, check=True)
    got = open(out).read()
    assert not got.endswith("\n")
    assert got.split("\n") == open(fixture_path("500x200.libsvm.predict")).read().rstrip("\n").split("\n")
    assert "Accuracy = " in r.stdout and "(classification)" in r.stdout


@pytest.mark.gpu
def test_train_then_predict_round_trip(tmp_path):
    model = tmp_path / "m.model"
    subprocess.run([EXE, "-q", "-t", "2", fixture_path("500x200.libsvm"), str(model)], check=True)
    r = subprocess.run([PRED, fixture_path("500x200.libsvm"), str(model), str(tmp_path / "p")], capture_output=True,
                       text=True, check=True)
    acc = float(r.stdout.split("Accuracy = ")[1].split("%")[0])
    assert acc > 90.0


@pytest.mark.gpu
def test_train_binary_input_equals_libsvm(tmp_path):
    """plssvm-train on the PLSSVMB1 binary form of 5x4.libsvm writes the same model as on the text file."""
    from plssvm_sparse_fp22_amd import io

    X, y = io.parse_libsvm(fixture_path("5x4.libsvm"), sparse=True)
    b = tmp_path / "5x4.bin"
    io.write_binary(b, X, y, io.BIN_F64)
    m1, m2 = tmp_path / "a.model", tmp_path / "b.model"
    subprocess.run([EXE, "-q", "--sparse", fixture_path("5x4.libsvm"), str(m1)], check=True)
    subprocess.run([EXE, "-q", str(b), str(m2)], check=True)
    assert open(m1).read() == open(m2).read()


TRACE_RE = re.compile(r"^Start Iteration (\d+) \(max: (\d+)\) with current residuum (\S+) \(target: (\S+)\)\. Done in (\d+)ms\.$",
                      re.M)
DONE_RE = re.compile(r"^Finished after (\d+) iterations with a residuum of (\S+) \(target: (\S+)\) and an average "
                     r"iteration time of (\d+)ms\.$", re.M)


def _write_libsvm(path, X, y):
    with open(path, "w") as f:
        for xi, yi in zip(X, y):
            f.write(f"{int(yi)} " + " ".join(f"{k}:{v!r}" for k, v in enumerate(xi.tolist())) + "\n")


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["5x4", "config1_500x4", "blobs_3000x256_rbf"])
def test_train_prints_the_reference_residual_trace(tmp_path, case, oracle):
    """plssvm-train without -q prints the reference solver_CG's lines (OpenMP/csvm.cpp:115-117,161-166):
    'Start Iteration k (max: imax) with current residuum delta (target: eps^2 delta0).' per iteration and
    the 'Finished after ...' summary. The printed residual curve equals the oracle's delta trace (fp64,
    1e-6 per iteration), the iteration count and the stop target likewise. The RBF set (config 2's shape
    at N = 3000) runs enough iterations to cross batched polls."""
    from plssvm_sparse_fp22_amd import datagen, io

    kernel = "linear"
    if case == "5x4":
        path = fixture_path("5x4.libsvm")
        X, y = io.parse_libsvm(path)
    else:
        if case == "config1_500x4":
            X, y = datagen.blobs(500, 4, seed=1)
        else:
            X, y = datagen.blobs(3000, 256, seed=2, cluster_std=4.0)
            kernel = "rbf"
        path = str(tmp_path / "train.libsvm")
        _write_libsvm(path, X, y)
        X2, y2 = io.parse_libsvm(path)
        assert np.array_equal(X2, X) and np.array_equal(y2, y)
    r = subprocess.run([EXE, "-t", "2" if kernel == "rbf" else "0", path, str(tmp_path / "m.model")],
                       capture_output=True, text=True, check=True)
    ref = oracle.learn(kernel, oracle.Data(np.ascontiguousarray(X)), y, eps=1e-3)
    lines = TRACE_RE.findall(r.stdout)
    assert len(lines) == ref["iters"] > 0, r.stdout[-3000:]
    target = 1e-6 * ref["trace"][0]
    for k, (it, imax, delta, tgt, _) in enumerate(lines):
        assert int(it) == k + 1 and int(imax) == X.shape[1]
        assert abs(float(delta) - ref["trace"][k]) <= 1e-6 * ref["trace"][k], (k, delta, ref["trace"][k])
        assert abs(float(tgt) - target) <= 1e-6 * target
    done = DONE_RE.findall(r.stdout)
    assert len(done) == 1
    assert int(done[0][0]) == ref["iters"]
    assert abs(float(done[0][1]) - ref["trace"][-1]) <= 1e-6 * ref["trace"][-1]
    assert "Setup for solving the optimization problem done in" in r.stdout
    assert "Solved minimization problem (r = b - Ax) using CG in" in r.stdout


def test_quiet_train_prints_nothing_on_cpu_error():
    """-q gates every line (parameter_train.cpp:60,124): an error still goes to stderr only."""
    r = subprocess.run([EXE, "-q", "/nonexistent.libsvm"], capture_output=True, text=True)
    assert r.returncode != 0 and r.stdout == ""
