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
