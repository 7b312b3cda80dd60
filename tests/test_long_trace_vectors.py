"""The long CG-trace fixtures (tests/golden/cg_traces_long/) pinned on the CPU: every case's inputs rebuild to the
recorded sha256, the fp64 oracle reproduces itself (1 vs 8 threads within 1e-9) and its extended-precision CG
(within 1e-6) over the compared window, and the oracle built here reproduces one case's committed curve (the full
regeneration is tests/golden/make_long_trace_vectors.py, ~1 minute)."""
import json
import os
import sys

import numpy as np
import pytest

import long_trace_cases as lc

sys.path.insert(0, os.path.join(lc.ROOT, "tests", "golden"))
import make_long_trace_vectors as mk  # noqa: E402

MANIFEST = json.load(open(os.path.join(lc.VECTORS, "manifest.json")))
WINDOW = 61


def test_manifest_covers_cases():
    assert sorted(MANIFEST) == sorted(lc.CASES)


@pytest.mark.parametrize("name", sorted(lc.CASES))
def test_inputs_rebuild_to_recorded_hash(name):
    s = lc.build(name)
    assert lc.input_hash(s) == MANIFEST[name]["input_sha256"]
    assert lc.input_hash(lc.load(name)) == MANIFEST[name]["input_sha256"]  # the fixture's copy (GPU tests)


@pytest.mark.parametrize("name", sorted(lc.CASES))
def test_oracle_reproducible_over_window(name):
    g = np.load(os.path.join(lc.VECTORS, name + ".npz"))
    f64 = lc.CASES[name][1] == np.float64
    t1, t8 = (g["trace"], g["trace_t8"]) if f64 else (g["trace64"], g["trace64_t8"])
    assert len(t1) == lc.IMAX + 1 and len(t8) == lc.IMAX + 1
    assert np.abs(t8[:WINDOW] / t1[:WINDOW] - 1).max() <= 1e-9, name
    if f64:
        assert np.abs(t1[:WINDOW] / g["trace_ld"][:WINDOW] - 1).max() <= 1e-6, name
    # a descent that stays far above the rounding floor over the window (no collapse in the first steps)
    assert t1[WINDOW - 1] / t1[0] > 1e-12, name


def test_oracle_reproduces_long_fixture(oracle):
    name = "rbf_f64_expansion"
    s = lc.build(name)
    r1 = mk.oracle_learn(s, np.float64, 1)
    g = np.load(os.path.join(lc.VECTORS, name + ".npz"))
    np.testing.assert_allclose(r1["trace"], g["trace"], rtol=1e-9)
    assert int(r1["iters"]) == int(g["iters"][0])
