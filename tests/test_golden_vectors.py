"""The committed oracle golden vectors (tests/golden/oracle_vectors/) are pinned here on the CPU:

* every set's inputs rebuild from their seeded recipe / fixture file to the recorded sha256;
* the oracle (built in this container) reproduces the committed vectors — all combinations of the
  small sets, one combination of each larger set (the full regeneration is
  tests/golden/make_oracle_vectors.py, ~1.5 min);
* the FP22 set's quantisation (plssvm_sparse_fp22_amd.fp22) equals the oracle's FP22 codec.
The oracle itself is pinned by the reference fixtures in tests/test_oracle.py.
"""
import json
import os
import sys

import numpy as np
import pytest

import golden_sets as gs

sys.path.insert(0, os.path.join(gs.ROOT, "tests", "golden"))
import make_oracle_vectors as mk  # noqa: E402

MANIFEST = json.load(open(os.path.join(gs.VECTORS, "manifest.json")))
SMALL = {"config1_500x4", "5x4"}
# every combination of the small sets; one per larger set (few CG iterations: the CPU suite stays short)
CHECKED = sorted([k for k, v in MANIFEST.items() if v["set"] in SMALL] +
                 ["500x200__rbf__f64", "blobs_3000x64__polynomial__f64", "csr_2000x5000__polynomial__f32",
                  "fp22_2000x5000__polynomial__f64"])


def test_manifest_covers_survey_matrix():
    assert len(MANIFEST) == len(gs.SETS) * len(gs.KERNELS) * len(gs.DTYPES)
    for k in MANIFEST:
        assert os.path.exists(os.path.join(gs.VECTORS, k + ".npz"))


@pytest.mark.parametrize("name", gs.SETS)
def test_inputs_rebuild_to_recorded_hash(name):
    for tag, dtype in gs.DTYPES.items():
        meta = MANIFEST[gs.key(name, "rbf", tag)]
        assert gs.input_hash(gs.build(name, dtype)) == meta["input_sha256"]


@pytest.mark.parametrize("key", CHECKED)
def test_oracle_reproduces_golden(oracle, key):
    meta = MANIFEST[key]
    dtype = np.dtype(meta["dtype"]).type
    arrays, meta2 = mk.vectors(meta["set"], meta["kernel"], dtype)
    assert meta2 == meta
    g = np.load(os.path.join(gs.VECTORS, key + ".npz"))
    rt = 1e-13 if dtype == np.float64 else 1e-6
    for name, want in g.items():
        if name.endswith("_t8"):  # 8-thread run: a noise estimate, not reproducible (OpenMP atomics)
            continue
        np.testing.assert_allclose(arrays[name], want, rtol=rt, atol=rt * max(1e-300, float(np.abs(want).max())),
                                   err_msg=f"{key}: {name}")


def test_fp22_set_matches_oracle_codec(oracle):
    s = gs.build("fp22_2000x5000", np.float32)
    raw, _ = gs.datagen.sparse_csr(2000, 5000, 50, seed=9, dtype=np.float32)
    words = oracle.fp22_pack(raw[2])
    assert np.array_equal(words, s["fp22"])
    assert np.array_equal(oracle.fp22_unpack(words, raw[2].size), s["csr"][2])
