"""Host data formats (no GPU): the PLSSVMB1 binary CSR / FP22 file and the LIBSVM reader."""
import numpy as np
import pytest

import plssvm_sparse_fp22_amd as pm
from plssvm_sparse_fp22_amd import datagen, io
from plssvm_sparse_fp22_amd.fp22 import pack, unpack
from conftest import fixture_path


@pytest.mark.parametrize("fmt", [io.BIN_F32, io.BIN_F64, io.BIN_FP22])
@pytest.mark.parametrize("labels", [True, False])
def test_binary_round_trip(tmp_path, fmt, labels):
    csr, y = datagen.sparse_csr(777, 301, 9, seed=4, dtype=np.float64)
    fn = tmp_path / "d.bin"
    io.write_binary(fn, csr, y if labels else None, fmt)
    (rowptr, col, val, n, d), y2, f2 = io.read_binary(fn)
    assert f2 == fmt and (n, d) == (777, 301)
    assert np.array_equal(rowptr, csr[0]) and np.array_equal(col, csr[1])
    if fmt == io.BIN_FP22:
        assert np.array_equal(val, pack(csr[2].astype(np.float32)))
    elif fmt == io.BIN_F32:
        assert np.array_equal(val, csr[2].astype(np.float32).astype(np.float64))
    else:
        assert np.array_equal(val, csr[2])
    assert (y2 is None) == (not labels) and (not labels or np.array_equal(y2, y))


def test_binary_parameter_detection(tmp_path):
    X, y = io.parse_libsvm(fixture_path("5x4.libsvm"), sparse=True)
    fn = tmp_path / "5x4.bin"
    io.write_binary(fn, X, y, io.BIN_FP22)
    p = pm.Parameter("linear", real_type=np.float32).parse_train_file(str(fn))
    assert p.val_fmt == pm._abi.VAL_FP22 and p.num_data_points == 5 and p.num_features == 4
    assert np.array_equal(unpack(p.csr[2], X[2].size), unpack(pack(X[2].astype(np.float32)), X[2].size))
    assert p.gamma == pytest.approx(0.25)


def test_binary_rejects_garbage(tmp_path):
    fn = tmp_path / "x.bin"
    fn.write_bytes(b"NOTPLSSVM" + b"\0" * 64)
    with pytest.raises(ValueError):
        io.read_binary(fn)
