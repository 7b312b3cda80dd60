#!/usr/bin/env python3
"""bench.py — CG iterations/s of the MI355X PLSSVM hot path (BASELINE.json metric).

One "step" = one CG iteration of openmp::csvm::solver_CG semantics (one implicit Q~·p over the
whole problem + the device-resident vector updates + the per-iteration RCCL all-reduce when
N > 1). Default workload = BASELINE.json configs[1]: dense RBF, 100k points x 256 features,
fp64, generate_data.py-style blobs (seeded, synthetic). N > 1 splits the same problem's
lower-triangle tiles over the ranks (strong scaling) with one all-reduce of the m-vector per K·p.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N > 1 under torch.distributed.run
(one process per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the environment).
Rank 0 prints exactly one JSON line on stdout; diagnostics go to stderr.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import plssvm_sparse_fp22_amd as pm  # noqa: E402  (loads libplssvm_mi355x.so before torch)
from plssvm_sparse_fp22_amd import datagen  # noqa: E402

PEAKS = {  # MI355X_MICROARCH.md: dense fp64 78.6 TF (vector = matrix), fp32 157.3 TF, HBM 8 TB/s
    "f64": 78.6e12,
    "f32": 157.3e12,
    "hbm": 8.0e12,
}

CONFIGS = {
    # name: (kernel, n, d, dtype, layout, description)
    "dense_rbf_100k": ("rbf", 100_000, 256, np.float64, "dense", "Dense RBF, 100k points x 256 features, fp64"),
    "dense_linear_500": ("linear", 500, 4, np.float64, "dense", "generate_data.py 500x4 dense, linear, fp64"),
    "dense_linear_500k": ("linear", 500_000, 1024, np.float32, "dense", "Dense linear, 500k x 1024, fp32 (MFMA)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="dense_rbf_100k", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=0, help="override number of points")
    ap.add_argument("--kp-reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo")
        uid = [pm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        uid = uid[0]
    else:
        uid = None

    kernel, n, d, dtype, layout, desc = CONFIGS[args.config]
    if args.n:
        n = args.n
    t0 = time.time()
    X, y = datagen.blobs(n, d, seed=2, dtype=dtype)
    log(f"[rank {rank}] data {n}x{d} {np.dtype(dtype).name} generated in {time.time() - t0:.1f}s")

    p = pm.Parameter(kernel, gamma=1.0 / d, real_type=dtype)
    p.data, p.labels = X, y
    svm = pm.CSVM(p, device=local_rank, rank=rank, world_size=world, uid=uid)
    t0 = time.time()
    svm.setup_data_on_device()
    q = svm.generate_q()
    b = (y[:-1] - y[-1]).astype(dtype)
    delta0 = svm.cg_begin(b, q, eps=1e-3)
    log(f"[rank {rank}] setup+q+r0 {time.time() - t0:.2f}s delta0={delta0:.6e}")

    def barrier():
        if dist is not None:
            dist.barrier()

    if args.warmup:
        svm.cg_step(args.warmup, force=True)
    barrier()
    t_start = time.perf_counter()
    svm.cg_step(args.steps, force=True)  # ends with hipStreamSynchronize
    elapsed = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    iters_per_s = args.steps / elapsed

    # ---- roofline of the dominant kernel (hipEvents on the engine stream) ----
    info = svm.info()
    ms_kp, ms_dom = svm.time_kp(args.kp_reps)
    m = n - 1
    pairs = m * (m + 1) / 2 * (info["tiles_local"] / max(1, info["tiles_total"]))
    if info["kp_mode"] == pm._abi.KP_FACTORED:
        alg = 2.0 * (m // world + 1) * d * np.dtype(dtype).itemsize  # gemv_n pass: XT rows of this rank
        bound, unit, peak = "hbm", "GB/s", PEAKS["hbm"]
        achieved = alg / (ms_dom * 1e-3)
        roof = dict(bound=bound, achieved=achieved / 1e9, peak=peak / 1e9, unit=unit, frac=achieved / peak,
                    traffic=None)
    else:
        alg = 2.0 * d * pairs  # the Gram-block FLOP of the lower triangle (norm-trick form)
        pk = PEAKS["f64" if dtype == np.float64 else "f32"]
        achieved = alg / (ms_dom * 1e-3)
        roof = dict(bound="mfma", achieved=achieved / 1e12, peak=pk / 1e12, unit="TFLOP/s", frac=achieved / pk,
                    traffic=None, alg_flop_per_launch=alg, alg_flop_per_kp_survey=3.0 * d * m * (m + 1) / 2,
                    kernel="kp_tile_kernel", launch_ms=ms_dom)

    # ---- CPU baseline: the oracle (port of the reference OpenMP kernel), rank 0, N = 1 only ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(kernel, X, dtype, d, m, args.cpu_seconds)

    if rank == 0:
        out = {
            "metric": "CG iters/sec + implicit K·p HBM GB/s vs roofline, N×d stated, 1/2/4/8 GPU",
            "value": iters_per_s,
            "unit": "CG iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64" if dtype == np.float64 else "f32",
            "data": "synthetic (seeded generate_data.py-style blobs)",
            "config": {"workload": desc, "N": n, "d": d, "kernel": kernel, "layout": layout,
                       "parallelism": f"row-block triangle tiles x{world}, RCCL all-reduce"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "kp_ms": ms_kp,
        }
        print(json.dumps(out), flush=True)
    svm.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(kernel, X, dtype, d, m, budget_s):
    """Time the oracle's OpenMP K·p (reference Release flags) on a leading-rows sample; scale by (m/m')^2."""
    from oracle import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    gamma = np.dtype(dtype).type(1.0 / d)

    def run(n_s):
        data = pyoracle.Data(X[:n_s], dtype=dtype)
        q = pyoracle.generate_q(kernel, data, gamma=gamma, fast=True)
        pvec = np.ones(n_s - 1, dtype=dtype)
        t = time.perf_counter()
        pyoracle.kp(kernel, data, q, dtype(1.0), dtype(1.0), 1.0, pvec, gamma=gamma, nthreads=threads, fast=True)
        return time.perf_counter() - t

    n_s = min(X.shape[0], 3000)
    t = run(n_s)
    target = budget_s * 0.8
    if t < target and n_s < X.shape[0]:
        n_s = int(min(X.shape[0], 40_000, n_s * math.sqrt(target / max(t, 1e-3))))
        t = run(n_s)
    ms = n_s - 1
    t_full = t * (m * (m + 1)) / (ms * (ms + 1))
    return {"value": 1.0 / t_full, "unit": "CG iterations/s", "cores": threads, "kind": "port",
            "sample": f"one K·p on the first {n_s} of {m + 1} points ({t:.2f}s), scaled by pair count to N={m + 1}",
            "pair_feature_per_s": ms * (ms + 1) / 2 * d / t}


if __name__ == "__main__":
    main()
