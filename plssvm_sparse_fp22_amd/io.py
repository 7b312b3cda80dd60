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
    try:
        f = open(path, "r")
    except FileNotFoundError:
        raise FileNotFoundError(f"Couldn't find file: '{path}'!") from None
    with f:
        for raw in f:
            s = raw.lstrip()
            if not s or s.startswith("#"):
                continue
            yield s.rstrip("\n")


def _convert_token(tok, dtype):
    """A whole token as a real of dtype (InvalidFileFormat with the reference's message otherwise)."""
    try:
        return float(tok)
    except ValueError:
        raise InvalidFileFormat(f"Can't convert '{tok.strip()}' to a value of type {_type_name(dtype)}!") from None


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
            labels.append(_convert_token(line[:pos], dtype))
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
            if not k.strip().isdigit():
                raise InvalidFileFormat(f"Can't convert '{k.strip()}' to a value of type unsigned long!")
            cols.append(int(k))
            vals.append(_convert_token(v, dtype))
        order = np.argsort(np.asarray(cols, dtype=np.int64), kind="stable")
        rows_c.append(np.asarray(cols, dtype=np.int64)[order])
        rows_v.append(np.asarray(vals, dtype=np.float64)[order])
    n = len(rows_c)
    if n == 0:
        raise InvalidFileFormat("Can't parse file: no data points are given!")
    d = max((int(c.max()) + 1 for c in rows_c if c.size), default=0)
    if d == 0:
        raise InvalidFileFormat("Can't parse file: no data points are given!")
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


class InvalidFileFormat(ValueError):
    """plssvm::invalid_file_format_exception (include/plssvm/exceptions/exceptions.hpp)."""


def _type_name(dtype):
    return "float" if np.dtype(dtype) == np.float32 else "double"


def _convert(text, kind):
    """detail::convert_to (include/plssvm/detail/string_conversion.hpp:39-64): leading whitespace is
    skipped and the longest valid prefix converted (std::from_chars / fast_float semantics)."""
    import re

    t = text.lstrip()
    pat = r"[+-]?(\d+\.?\d*([eE][+-]?\d+)?|\.\d+([eE][+-]?\d+)?|inf|infinity|nan)" if kind not in (
        "unsigned int", "unsigned long long") else r"\d+"
    mt = re.match(pat, t, re.IGNORECASE)
    if mt is None or (kind in ("float", "double") and t.startswith("+")):
        raise InvalidFileFormat(f"Can't convert '{t}' to a value of type {kind}!")
    return float(mt.group(0)) if kind in ("float", "double") else int(mt.group(0))


def parse_model(path, dtype=np.float64):
    """LIBSVM model file (parameter<T>::parse_model_file, src/plssvm/parameter.cpp:366-520), as written
    by csvm::write_model (src/plssvm/csvm.cpp:60-204). Same header rules and error messages:
    lines left-trimmed, '#' comments skipped, header lines lower-cased, the entries svm_type c_svc,
    kernel_type, gamma, degree, coef0, nr_class 2, total_sv > 0, rho, label 1 -1 (either order),
    nr_sv a b with a + b == total_sv, then SV and total_sv lines 'alpha idx:val ...'."""
    dtype = np.dtype(dtype)
    tn = _type_name(dtype)
    try:
        with open(path) as f:
            raw = f.read().split("\n")
    except FileNotFoundError:
        raise FileNotFoundError(f"Couldn't find file: '{path}'!") from None
    lines = [ln.lstrip() for ln in raw]
    lines = [ln for ln in lines if ln and not ln.startswith("#")]
    header = {}
    num_sv, labels, rho, nr_sv = 0, (0.0, 0.0), None, None
    h = 0
    while h < len(lines):
        line = lines[h].strip().lower()
        sp = line.find(" ")
        value = line[sp + 1:].lstrip() if sp >= 0 else ""
        if line.startswith("svm_type"):
            if value != "c_svc":
                raise InvalidFileFormat(f"Can only use c_svc as svm_type, but '{value}' was given!")
        elif line.startswith("kernel_type"):
            tok = value.split()[0] if value.split() else ""
            k = {"linear": "linear", "0": "linear", "polynomial": "polynomial", "1": "polynomial", "rbf": "rbf",
                 "2": "rbf"}.get(tok)
            if k is None:
                raise InvalidFileFormat(f"Unrecognized kernel type '{value}'!")
            header["kernel_type"] = k
        elif line.startswith("gamma"):
            header["gamma"] = _convert(value, tn)
        elif line.startswith("degree"):
            header["degree"] = _convert(value, "int")
        elif line.startswith("coef0"):
            header["coef0"] = _convert(value, tn)
        elif line.startswith("nr_class"):
            nc = _convert(value, "unsigned int")
            if nc != 2:
                raise InvalidFileFormat(f"Can only use 2 classes, but {nc} were given!")
        elif line.startswith("total_sv"):
            num_sv = _convert(value, "unsigned long long")
            if num_sv == 0:
                raise InvalidFileFormat(f"The number of support vectors must be greater than 0, but is {num_sv}!")
        elif line.startswith("rho"):
            rho = _convert(value, tn)
        elif line.startswith("label"):
            sp1 = value.find(" ")
            first = value if sp1 < 0 else value[:sp1]
            rest = "" if sp1 < 0 else value[sp1 + 1:]
            sp2 = rest.find(" ")
            second = rest if sp2 < 0 else rest[:sp2]
            tail = "" if sp2 < 0 else rest[sp2 + 1:].lstrip()
            labels = (_convert(first, tn), _convert(second, tn))
            if tail or labels[0] not in (1.0, -1.0) or labels[1] not in (1.0, -1.0):
                raise InvalidFileFormat(f"Only the labels 1 and -1 are allowed, but '{line}' were given!")
        elif line.startswith("nr_sv"):
            sp1 = value.find(" ")
            first = value if sp1 < 0 else value[:sp1]
            rest = "" if sp1 < 0 else value[sp1 + 1:]
            sp2 = rest.find(" ")
            second = rest if sp2 < 0 else rest[:sp2]
            tail = "" if sp2 < 0 else rest[sp2 + 1:].lstrip()
            a, b = _convert(first, "unsigned long long"), _convert(second, "unsigned long long")
            if tail:
                raise InvalidFileFormat(f"Only two numbers are allowed, but more were given '{line}'!")
            if a + b != num_sv:
                raise InvalidFileFormat("The number of positive and negative support vectors doesn't add up to the "
                                        f"total number: {a} + {b} != {num_sv}!")
            nr_sv = [a, b]
        elif line == "sv":
            break
        else:
            raise InvalidFileFormat(f"Unrecognized header entry '{lines[h].rstrip()}'! Maybe SV is missing?")
        h += 1
    if num_sv == 0:
        raise InvalidFileFormat("Missing total number of support vectors!")
    if labels[0] == 0 or labels[1] == 0:
        raise InvalidFileFormat("Missing labels!")
    if nr_sv is None:
        raise InvalidFileFormat("Missing number of support vectors per class!")
    if rho is None:
        raise InvalidFileFormat("Missing rho value!")
    if h + 1 >= len(lines):
        raise InvalidFileFormat("Can't parse file: no support vectors are given or SV is missing!")
    sv_lines = lines[h + 1:h + 1 + num_sv]
    if len(sv_lines) < num_sv:
        raise InvalidFileFormat(f"total_sv is {num_sv}, but only {len(sv_lines)} support vectors are given!")
    alphas, rows = [], []
    for ln in sv_lines:
        toks = ln.split()
        alphas.append(_convert(toks[0], tn))
        r = {}
        for t in toks[1:]:
            if ":" not in t:
                break
            k, v = t.split(":", 1)
            r[int(k)] = _convert(v, tn)
        rows.append(r)
    d = max((max(r) for r in rows if r), default=-1) + 1
    if d == 0:
        raise InvalidFileFormat("Can't parse file: no data points are given!")
    SV = np.zeros((len(rows), d), dtype=dtype)
    for i, r in enumerate(rows):
        for c, v in r.items():
            SV[i, c] = v
    out = dict(kernel=header.get("kernel_type", "linear"), rho=float(rho), alpha=np.asarray(alphas, dtype=dtype),
               SV=SV, nr_sv=nr_sv, labels=labels)
    for key in ("degree", "gamma", "coef0"):
        if key in header:
            out[key] = header[key]
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
