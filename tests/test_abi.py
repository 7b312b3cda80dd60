"""CPU tests of the C-ABI boundary: the library builds, loads and exports every declared entry point.
No compute call is made here (there is no GPU in the build container)."""
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "plssvm_mi355x.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"PLSSVM_MI_API\s+[\w\s\*]*?\b(plssvm_mi_\w+)\s*\(", txt)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    assert "plssvm_mi_kp" in syms and "plssvm_mi_solve_cg" in syms and "plssvm_mi_setup_csr" in syms
    assert len(syms) >= 20


def test_library_exports_every_declared_symbol():
    from plssvm_sparse_fp22_amd import _abi

    L = _abi.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
    assert set(declared_symbols()) == set(_abi.EXPORTS)


def test_no_gpu_fails_loudly():
    import plssvm_sparse_fp22_amd as pm

    if pm.device_count() > 0:
        pytest.skip("GPU present")
    import numpy as np

    p = pm.Parameter("rbf")
    p.data = np.ones((4, 3))
    with pytest.raises(pm.BackendError) as e:
        pm.CSVM(p)
    assert "no HIP devices" in str(e.value)


def test_missing_library_raises(monkeypatch, tmp_path):
    from plssvm_sparse_fp22_amd import _abi

    monkeypatch.setattr(_abi, "LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(_abi, "_lib", None)
    with pytest.raises(ImportError):
        _abi.lib()
