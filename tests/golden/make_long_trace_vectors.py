#!/usr/bin/env python3
"""Generates tests/golden/cg_traces_long/ with the C oracle (the reference OpenMP path restated, oracle/; test
infrastructure only) for the long CG-trace cases of tests/long_trace_cases.py.

Per case (<case>.npz): the oracle's learn() in the case's real type on 1 thread (trace, alpha, bias, iters) and on
8 threads (trace_t8: the reference's own run-to-run spread — its OpenMP atomics reorder the sums), the same CG in
extended precision on the explicit Q~ (trace_ld); for fp32 cases also the fp64 oracle on the same fp32-representable
inputs, 1 and 8 threads (trace64, trace64_t8, alpha64). manifest.json: parameters, input sha256, and the measured
reproducibility — rep_1e9 = the number of leading iterations over which the fp64 oracle's 1- and 8-thread traces
agree to 1e-9 relative, and for fp32 cases f32_oracle_dev = max over the first 60 iterations of the fp32 oracle's
relative distance from the fp64 one.

usage (build container, ~1 minute): python tests/golden/make_long_trace_vectors.py [case ...]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import long_trace_cases as lc  # noqa: E402
from oracle import pyoracle  # noqa: E402


def oracle_learn(s, dtype, nthreads):
    if "X" in s:
        data = pyoracle.Data(X=np.asarray(s["X"], dtype), dtype=dtype)
    else:
        rowptr, col, val, n, d = s["csr"]
        data = pyoracle.Data(rowptr=rowptr, col=col, val=np.asarray(val, dtype), n=n, d=d, dtype=dtype)
    dt = np.dtype(dtype).type
    return pyoracle.learn(s["kernel"], data, s["y"].astype(dtype), cost=s["cost"], eps=s["eps"], imax=lc.IMAX,
                          degree=3, gamma=dt(s["gamma"]), coef0=dt(s["coef0"]), nthreads=nthreads)


def reproducible(t1, t8, tol=1e-9):
    n = min(len(t1), len(t8))
    bad = np.nonzero(np.abs(t8[:n] / t1[:n] - 1) > tol)[0]
    return int(bad[0]) if bad.size else n


def vectors(name):
    s = lc.build(name)
    dtype = s["dtype"]
    r1 = oracle_learn(s, dtype, 1)
    r8 = oracle_learn(s, dtype, 8)
    arrays = dict(trace=r1["trace"], alpha=r1["alpha"], bias=np.array([r1["bias"]], np.float64),
                  iters=np.array([r1["iters"]], np.int64), trace_t8=r8["trace"], trace_ld=lc.trace_extended(s), **lc.input_arrays(s))
    meta = dict(kernel=s["kernel"], dtype=np.dtype(dtype).name, n=lc.N, cost=s["cost"], eps=s["eps"], imax=lc.IMAX,
                gamma=float(s["gamma"]), coef0=float(s["coef0"]), input_sha256=lc.input_hash(s),
                iters=int(r1["iters"]), delta_ratio_last=float(r1["trace"][-1] / r1["trace"][0]))
    if dtype == np.float32:
        a = oracle_learn(s, np.float64, 1)
        b = oracle_learn(s, np.float64, 8)
        arrays.update(trace64=a["trace"], trace64_t8=b["trace"], alpha64=a["alpha"],
                      bias64=np.array([a["bias"]], np.float64))
        meta["rep_1e9"] = reproducible(a["trace"], b["trace"])
        meta["rep_1e6"] = reproducible(a["trace"], b["trace"], 1e-6)
        n = min(61, len(r1["trace"]), len(a["trace"]))
        meta["f32_oracle_dev"] = float(np.abs(r1["trace"][:n] / a["trace"][:n] - 1).max())
        # the curve the fp32 GPU runs are compared with: the fp64 oracle's (delta_ratio_last is the fp32 oracle's own)
        meta["delta_ratio_last64"] = float(a["trace"][-1] / a["trace"][0])
        meta["delta_ratio_60_64"] = float(a["trace"][min(60, len(a["trace"]) - 1)] / a["trace"][0])
    else:
        meta["rep_1e9"] = reproducible(r1["trace"], r8["trace"])
        meta["ld_dev"] = float(np.abs(r1["trace"] / arrays["trace_ld"][:len(r1["trace"])] - 1).max())
    return arrays, meta


def main():
    pyoracle.build()
    os.makedirs(lc.VECTORS, exist_ok=True)
    mpath = os.path.join(lc.VECTORS, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    for name in (sys.argv[1:] or sorted(lc.CASES)):
        arrays, meta = vectors(name)
        np.savez_compressed(os.path.join(lc.VECTORS, name + ".npz"), **arrays)
        manifest[name] = meta
        print(name, meta, flush=True)
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
