"""The sparse CG-trace fixtures (tests/golden/cg_traces/) pinned on the CPU: every case's inputs rebuild to the
recorded sha256, and the oracle (built in this container) reproduces one case's committed trace and alphas
(the full regeneration is tests/golden/make_cg_trace_vectors.py, ~5 minutes)."""
import json
import os
import sys

import numpy as np
import pytest

import cg_trace_cases as cc

sys.path.insert(0, os.path.join(cc.ROOT, "tests", "golden"))
import make_cg_trace_vectors as mk  # noqa: E402

MANIFEST = json.load(open(os.path.join(cc.VECTORS, "manifest.json")))


def test_manifest_covers_cases():
    assert sorted(MANIFEST) == sorted(cc.CASES)


@pytest.mark.parametrize("name", sorted(cc.CASES))
def test_inputs_rebuild_to_recorded_hash(name):
    assert cc.input_hash(cc.build(name)) == MANIFEST[name]["input_sha256"]


def test_oracle_reproduces_trace_fixture(oracle):
    name = "rbf_f32_bf16_flags"
    s = cc.build(name)
    r1 = mk.oracle_learn(s, np.float32, 1)
    g = np.load(os.path.join(cc.VECTORS, name + ".npz"))
    np.testing.assert_allclose(r1["trace"], g["trace"], rtol=1e-6)
    np.testing.assert_allclose(r1["alpha"], g["alpha"], rtol=1e-6, atol=1e-6 * np.abs(g["alpha"]).max())
    assert int(r1["iters"]) == int(g["iters"][0])
