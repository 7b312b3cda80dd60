"""LIBSVM data / model files (host side).

Restates the reference parser semantics (src/plssvm/parameter.cpp:40-176 and
src/plssvm/detail/file_reader.cpp:129-153):

* lines are left-trimmed; empty lines and lines starting with ``#`` are skipped;
* the label is the token before the first space when it has no ``:``; labels map through
  ``sign`` (x > 0 -> +1 else -1, include/plssvm/detail/operators.hpp:174-177);
* feature indices are taken **0-based as written** (parameter.cpp:75-83); the number of
  features is max(index)+1 over the file; missing entries are 0;
* ``gamma`` defaults to 1/num_features in the real type (parameter.cpp:150-152).

Unlike the reference, which always densifies, :func:`parse_libsvm` can return CSR
(int64 rowptr, int32 col, values) so large sparse sets never exist as dense host arrays.
"""
from __future__ import annotations

import numpy as np


def _lines(path):
    with open(path, "r") as f:
        for raw in f:
            s = raw.lstrip()
            if not s or s.startswith("#"):
                continue
            yield s.rstrip("\n")


def parse_libsvm(path, dtype=np.float64, sparse=False):
    """Returns (X, y) with X dense [n][d] (or (rowptr, col, val, n, d) when sparse) and y in {-1,+1}
    (None when the file carries no labels)."""
    dtype = np.dtype(dtype)
    labels, rows_c, rows_v = [], [], []
    has_label = None
    for line in _lines(path):
        pos = line.find(" ")
        colon = line.find(":")
        if pos == -1:
            pos = len(line)
        if colon == -1 or colon >= pos:
            labels.append(float(line[:pos]))
            rest = line[pos:]
            has_label = True if has_label is None else has_label
        else:
            rest = line
            has_label = False
        cols, vals = [], []
        for tok in rest.split():
            if ":" not in tok:
                break  # trailing comment or garbage after the last feature
            k, v = tok.split(":", 1)
            cols.append(int(k))
            vals.append(float(v))
        order = np.argsort(np.asarray(cols, dtype=np.int64), kind="stable")
        rows_c.append(np.asarray(cols, dtype=np.int64)[order])
        rows_v.append(np.asarray(vals, dtype=np.float64)[order])
    n = len(rows_c)
    if n == 0:
        raise ValueError("Can't parse file: no data points are given!")
    d = max((int(c.max()) + 1 for c in rows_c if c.size), default=0)
    if d == 0:
        raise ValueError("Can't parse file: no data points are given!")
    y = None
    if has_label:
        y = np.where(np.asarray(labels) > 0, 1.0, -1.0).astype(dtype)
    if sparse:
        rowptr = np.zeros(n + 1, dtype=np.int64)
        rowptr[1:] = np.cumsum([c.size for c in rows_c])
        col = np.concatenate(rows_c).astype(np.int32) if rowptr[-1] else np.zeros(0, np.int32)
        val = np.concatenate(rows_v).astype(dtype) if rowptr[-1] else np.zeros(0, dtype)
        return (rowptr, col, val, n, d), y
    X = np.zeros((n, d), dtype=dtype)
    for i, (c, v) in enumerate(zip(rows_c, rows_v)):
        X[i, c] = v.astype(dtype)
    return X, y


def parse_model(path, dtype=np.float64):
    """LIBSVM model file as written by csvm::write_model (src/plssvm/csvm.cpp:60-204)."""
    dtype = np.dtype(dtype)
    header, svs = {}, []
    with open(path) as f:
        lines = [ln.strip() for ln in f if ln.strip() and not ln.lstrip().startswith("#")]
    k = 0
    while lines[k] != "SV":
        key, _, val = lines[k].partition(" ")
        header[key] = val
        k += 1
    alphas, rows = [], []
    for ln in lines[k + 1:]:
        toks = ln.split()
        alphas.append(float(toks[0]))
        rows.append({int(t.split(":")[0]): float(t.split(":")[1]) for t in toks[1:]})
    d = max(max(r) for r in rows if r) + 1
    SV = np.zeros((len(rows), d), dtype=dtype)
    for i, r in enumerate(rows):
        for c, v in r.items():
            SV[i, c] = v
    out = dict(kernel=header["kernel_type"], rho=float(header["rho"]), alpha=np.asarray(alphas, dtype=dtype), SV=SV,
               nr_sv=[int(t) for t in header["nr_sv"].split()])
    if "degree" in header:
        out["degree"] = int(header["degree"])
    if "gamma" in header:
        out["gamma"] = float(header["gamma"])
    if "coef0" in header:
        out["coef0"] = float(header["coef0"])
    return out


# ---- binary CSR / FP22 data file (build-defined; SURVEY.md §8(f)1: input path without densification) ----
# little endian:
#   0  char[8]  "PLSSVMB1"
#   8  uint32   version (1)          12 uint32 flags (bit 0: labels present)
#   16 int64    n                    24 int64  d
#   32 int64    nnz                  40 int32  value format (0 float32, 1 float64, 2 packed FP22)  44 int32 0
#   48 int64    rowptr[n + 1]; int32 col[nnz]; pad to 8 bytes; values (float32[nnz] | float64[nnz] |
#      uint32[11 * ceil(nnz / 16)]); pad to 8 bytes; float64 labels[n] (flag bit 0)
# Readers memory-map the arrays (a 2M x 100k @ 0.05 % set loads without parsing text).
BIN_MAGIC = b"PLSSVMB1"
BIN_F32, BIN_F64, BIN_FP22 = 0, 1, 2


def _pad8(nbytes):
    return (-nbytes) % 8


def write_binary(path, csr, labels=None, fmt=None):
    """Write (rowptr, col, val, n, d) [+ labels]. fmt: BIN_F32 | BIN_F64 | BIN_FP22 (val then holds
    real values, packed here) — default from val's dtype."""
    from .fp22 import pack

    rowptr, col, val, n, d = csr
    rowptr = np.ascontiguousarray(rowptr, dtype="<i8")
    col = np.ascontiguousarray(col, dtype="<i4")
    nnz = int(rowptr[-1])
    if fmt is None:
        fmt = BIN_F64 if np.asarray(val).dtype == np.float64 else BIN_F32
    if fmt == BIN_FP22:
        vbytes = np.ascontiguousarray(pack(np.asarray(val, dtype=np.float32)), dtype="<u4").tobytes()
    else:
        vbytes = np.ascontiguousarray(val, dtype="<f8" if fmt == BIN_F64 else "<f4").tobytes()
    hdr = np.zeros(48, dtype=np.uint8)
    hdr[:8] = np.frombuffer(BIN_MAGIC, dtype=np.uint8)
    hdr[8:16] = np.frombuffer(np.array([1, 1 if labels is not None else 0], dtype="<u4").tobytes(), dtype=np.uint8)
    hdr[16:40] = np.frombuffer(np.array([n, d, nnz], dtype="<i8").tobytes(), dtype=np.uint8)
    hdr[40:48] = np.frombuffer(np.array([fmt, 0], dtype="<i4").tobytes(), dtype=np.uint8)
    with open(path, "wb") as f:
        f.write(hdr.tobytes())
        f.write(rowptr.tobytes())
        cb = col.tobytes()
        f.write(cb + b"\0" * _pad8(len(cb)))
        f.write(vbytes + b"\0" * _pad8(len(vbytes)))
        if labels is not None:
            f.write(np.ascontiguousarray(labels, dtype="<f8").tobytes())


def read_binary(path, dtype=np.float64, mmap=True):
    """Returns ((rowptr, col, val, n, d), labels or None, fmt); FP22 values stay packed (uint32 words,
    use Parameter.val_fmt = VAL_FP22), real values are converted to dtype."""
    raw = np.memmap(path, dtype=np.uint8, mode="r") if mmap else np.fromfile(path, dtype=np.uint8)
    if raw.size < 48 or bytes(raw[:8]) != BIN_MAGIC:
        raise ValueError(f"{path}: not a PLSSVMB1 binary data file")
    version, flags = np.frombuffer(bytes(raw[8:16]), dtype="<u4")
    if version != 1:
        raise ValueError(f"{path}: unsupported binary version {version}")
    n, d, nnz = (int(v) for v in np.frombuffer(bytes(raw[16:40]), dtype="<i8"))
    fmt = int(np.frombuffer(bytes(raw[40:44]), dtype="<i4")[0])
    off = 48
    rowptr = raw[off:off + 8 * (n + 1)].view("<i8")
    off += 8 * (n + 1)
    col = raw[off:off + 4 * nnz].view("<i4")
    off += 4 * nnz + _pad8(4 * nnz)
    if fmt == BIN_FP22:
        nb = 4 * (11 * ((nnz + 15) // 16))
        val = raw[off:off + nb].view("<u4")
    else:
        nb = (8 if fmt == BIN_F64 else 4) * nnz
        val = raw[off:off + nb].view("<f8" if fmt == BIN_F64 else "<f4").astype(dtype)
    off += nb + _pad8(nb)
    labels = None
    if flags & 1:
        labels = raw[off:off + 8 * n].view("<f8").astype(dtype)
    if rowptr[0] != 0 or rowptr[-1] != nnz:
        raise ValueError(f"{path}: corrupt row pointers")
    return (rowptr, col, val, n, d), labels, fmt
