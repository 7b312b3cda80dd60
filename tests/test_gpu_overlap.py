"""Full-size parity of the sparse poly/RBF per-pair work (VERDICT r1 "sparse-RBF parity blind spot").

The checks in test_gpu_fullsize.py compare the whole K·p, whose fp32 scale is dominated by the
separable part: the overlapping pairs' terms are ~5e-7 of it at config 3-RBF, so those checks would
pass with the pair kernel writing zeros. Here the overlap sum O_i (PLSSVM_MI_PART_OVERLAP: the exact
per-pair work of the sparse kernel, nothing separable) is compared on 256 sampled rows against a
float64 restatement (tests/overlap_check.py), relative to sum_j |c_ij p_j|: 1e-4 in fp32, 1e-12 in fp64.

Reference: every pair's kernel value is part of the result (svm_kernel.hip.hpp:206-268).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from overlap_check import check

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))

CASES = [
    ("csr_rbf_1m", None, np.float32, None),     # BASELINE configs[2] with RBF at full size: 1M x 50k
    ("fp22_rbf_2m", None, np.float32, None),     # configs[4] (FP22 input) at full size: 2M x 100k on one GPU
    ("fp22_rbf_2m", None, np.float64, None),     # the same set in fp64 (remainder stream 1.37e9 slots x 10 B)
    ("fp22_rbf_2m", 400_000, np.float32, None),  # configs[4] at N = 400k, same column occupancy
    ("csr_rbf_1m", None, np.float64, None),      # fp64 at full size (the kernel expansion fits)
    ("csr_rbf_1m", 400_000, np.float32, "polynomial"),
    ("csr_rbf_1m", 200_000, np.float64, "polynomial"),
]
ALGOS = ["auto", "pattern"]  # auto = the kernel expansion on these sets; pattern = the stored Gram pattern


def _case_id(c):
    return f"{c[0]}-{c[1]}-{np.dtype(c[2]).name}-{c[3] or 'cfg'}"


@pytest.mark.parametrize("algo", ALGOS)
@pytest.mark.parametrize("config,points,dtype,kernel", CASES, ids=[_case_id(c) for c in CASES])
def test_overlap_sum_full_size(config, points, dtype, kernel, algo):
    if algo == "pattern" and config == "fp22_rbf_2m" and points is None:
        pytest.skip("the Gram pattern of the 2M set (~300 GB) does not fit one GPU; the expansion runs it")
    if algo == "pattern" and dtype == np.float64 and points is None:
        points = 400_000  # the fp64 pattern of the full set (2.5e10 pairs x 10 B) does not fit one GPU
    err, tol, info = check(config, points, dtype, kernel, sparse_algo=algo)
    assert info["pairs"] > 0
    want = pm_algo(algo)
    assert info["sparse_algo"] == want
    print(f"overlap {config} N={points} {np.dtype(dtype).name} {kernel} {algo}: err {err:.3e} (tol {tol:g})")
    assert err <= tol, (config, points, np.dtype(dtype).name, kernel, algo, err)


def pm_algo(algo):
    import plssvm_sparse_fp22_amd as pm

    return pm._abi.SPARSE_PATTERN if algo == "pattern" else pm._abi.SPARSE_EXPANSION


def _ablated(env, dts, algo):
    env = dict(os.environ, **env)
    out = subprocess.run([sys.executable, os.path.join(HERE, "overlap_check.py"), "csr_rbf_1m", "200000", dts, algo],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    return json.loads(out.stdout.strip().splitlines()[-1])


def test_overlap_check_sees_an_ablated_pattern_kernel():
    """The check run on the timing-only ablation PLSSVM_MI_GRAM_ABLATE=2 of the Gram-pattern kernel (the
    pair function replaced by a linear stand-in, no exp) must fail: the test sees the per-pair work."""
    res = _ablated({"PLSSVM_MI_GRAM_ABLATE": "2"}, "f32", "pattern")
    # O_i is a signed sum (~2 % of sum |terms| here): the ablation's ~28 % per-term error shows as ~6e-3
    assert res["err"] > 10 * res["tol"], res
    err, tol, _ = check("csr_rbf_1m", 200_000, np.float32, sparse_algo="pattern")  # the real kernel passes
    assert err <= tol


@pytest.mark.parametrize("ablate", ["1", "2"])
def test_overlap_check_sees_an_ablated_expansion(ablate):
    """Kernel expansion ablations (PLSSVM_MI_EXP_ABLATE): 1 drops the stored remainder of the pairs that
    share two or more features, 2 keeps only the first Taylor term. Both are ~1e-6 of the overlap scale
    at this occupancy (below the fp32 bar), so the fp64 check (1e-12) must see them."""
    res = _ablated({"PLSSVM_MI_EXP_ABLATE": ablate}, "f64", "auto")
    assert res["sparse_algo"] == pm_algo("auto")
    assert res["err"] > 10 * res["tol"], res
