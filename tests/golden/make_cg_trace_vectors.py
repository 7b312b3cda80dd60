#!/usr/bin/env python3
"""Generates tests/golden/cg_traces/ with the C oracle (the reference OpenMP path restated, oracle/;
test infrastructure only) for the sparse CG-trace cases of tests/cg_trace_cases.py.

Per case (<case>.npz, plain arrays): the oracle's learn() on 1 thread (trace, alpha, iters) and on 8
threads (trace_t8, alpha_t8: the reference's own run-to-run spread, its OpenMP atomics reorder the sums),
the same CG in extended precision on the explicit Q~ (trace_ld), and for fp32 cases the fp64 oracle on the
same fp32-representable inputs (trace64, alpha64); manifest.json holds the parameters and an input sha256.

usage (build container, ~2 minutes): python tests/golden/make_cg_trace_vectors.py [case ...]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import cg_trace_cases as cc  # noqa: E402
from oracle import pyoracle  # noqa: E402


def oracle_learn(s, dtype, nthreads):
    rowptr, col, val, n, d = s["csr"]
    data = pyoracle.Data(rowptr=rowptr, col=col, val=val.astype(dtype), n=n, d=d, dtype=dtype)
    dt = np.dtype(dtype).type
    return pyoracle.learn(s["kernel"], data, s["y"].astype(dtype), cost=s["cost"], eps=s["eps"], imax=cc.IMAX, degree=3,
                          gamma=dt(s["gamma"]), coef0=dt(s["coef0"]), nthreads=nthreads)


def vectors(name):
    s = cc.build(name)
    dtype = s["dtype"]
    r1 = oracle_learn(s, dtype, 1)
    r8 = oracle_learn(s, dtype, 8)
    arrays = dict(trace=r1["trace"], alpha=r1["alpha"], bias=np.array([r1["bias"]], np.float64),
                  iters=np.array([r1["iters"]], np.int64), trace_t8=r8["trace"], alpha_t8=r8["alpha"],
                  trace_ld=cc.trace_extended(s))
    if dtype == np.float32:
        r64 = oracle_learn(s, np.float64, 1)
        arrays.update(trace64=r64["trace"], alpha64=r64["alpha"], bias64=np.array([r64["bias"]], np.float64))
    meta = dict(kernel=s["kernel"], dtype=np.dtype(dtype).name, n=cc.N, d=cc.D, cost=s["cost"], eps=s["eps"],
                imax=cc.IMAX, gamma=float(s["gamma"]), coef0=float(s["coef0"]), fp22=s["fp22"] is not None,
                input_sha256=cc.input_hash(s), iters=int(r1["iters"]))
    return arrays, meta


def main():
    pyoracle.build()
    os.makedirs(cc.VECTORS, exist_ok=True)
    mpath = os.path.join(cc.VECTORS, "manifest.json")
    manifest = json.load(open(mpath)) if os.path.exists(mpath) else {}
    for name in (sys.argv[1:] or sorted(cc.CASES)):
        arrays, meta = vectors(name)
        np.savez_compressed(os.path.join(cc.VECTORS, name + ".npz"), **arrays)
        manifest[name] = meta
        print(name, "iters", meta["iters"], flush=True)
    with open(mpath, "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
