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


def test_info_struct_mirrors_the_header(tmp_path):
    """_abi.Info (ctypes) has the C header's plssvm_mi_info layout: every field at the same offset, same size
    (a C program compiled against include/plssvm_mi355x.h prints offsetof / sizeof)."""
    import ctypes
    import subprocess

    from plssvm_sparse_fp22_amd import _abi

    names = [f[0] for f in _abi.Info._fields_]
    src = tmp_path / "info.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "plssvm_mi355x.h"\nint main(void) {\n'
                   + "".join(f'    printf("{n} %zu\\n", offsetof(plssvm_mi_info, {n}));\n' for n in names)
                   + '    printf("sizeof %zu\\n", sizeof(plssvm_mi_info));\n    return 0;\n}\n')
    exe = tmp_path / "info"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    for n in names:
        assert int(got[n]) == getattr(_abi.Info, n).offset, n
    assert int(got["sizeof"]) == ctypes.sizeof(_abi.Info)
