"""bench.py's JSON line on the GPU (the driver's contract): the headline workload at its BASELINE size,
a roofline fraction that is a fraction, and the time-to-solution record. Runs bench.py as a child process
(bounded steps) and checks the line it prints."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_bench(*args, timeout=240):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                         text=True, timeout=timeout)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.gpu
def test_headline_line_contract():
    r = run_bench("--no-extra", "--no-cpu", "--steps", "3", "--warmup", "1")
    assert r["unit"] == "CG iterations/s" and r["value"] > 0 and r["n_gpus"] == 1
    assert r["steps"] == 3 and r["warmup"] == 1 and r["higher_is_better"] is True
    cfg = r["config"]
    assert (cfg["N"], cfg["d"], cfg["kernel"], cfg["layout"]) == (100_000, 256, "rbf", "dense")
    assert r["dtype"] == "f64"
    roof = r["roofline"]
    assert roof["bound"] == "mfma" and roof["unit"] == "TFLOP/s"
    # 2 d m (m + 1) / 2 FLOP per launch over the measured launch time: a real fraction of spec
    assert roof["alg_flop_per_launch"] == pytest.approx(2 * 256 * 99_999 * 100_000 / 2)
    assert 0.5 < roof["frac"] < 1.0
    learn = r["learn"]
    assert learn["converged"] and learn["cg_iters"] >= 1 and learn["learn_s"] > 0


@pytest.mark.gpu
def test_sparse_extra_line_contract():
    r = run_bench("--config", "csr_linear_1m", "--no-cpu", "--steps", "3", "--warmup", "1")
    cfg = r["config"]
    assert (cfg["N"], cfg["d"], cfg["layout"]) == (1_000_000, 50_000, "csr")
    roof = r["roofline"]
    assert roof["bound"] == "hbm" and 0.3 < roof["frac"] < 1.0


@pytest.mark.gpu
def test_dense_linear_500k_line_contract():
    """BASELINE configs[3] (dense linear 500k x 1024 fp32, the MFMA row) at its full size on one GPU: the record the
    default line carries as extra.dense_linear_500k"""
    r = run_bench("--config", "dense_linear_500k", "--no-cpu", "--steps", "1", "--warmup", "0", "--kp-reps", "1")
    cfg = r["config"]
    assert (cfg["N"], cfg["d"], cfg["kernel"], cfg["layout"], cfg["kp_mode"]) == (500_000, 1024, "linear", "dense",
                                                                                 "pairwise")
    assert r["dtype"] == "f32"
    roof = r["roofline"]
    assert roof["bound"] == "mfma" and roof["kernel"] == "kp_tile_kernel"
    assert roof["alg_flop_per_launch"] == pytest.approx(2 * 1024 * 499_999 * 500_000 / 2)
    assert 0.5 < roof["frac"] < 1.0
