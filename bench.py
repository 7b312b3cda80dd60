#!/usr/bin/env python3
"""bench.py — CG iterations/s of the MI355X PLSSVM hot path (BASELINE.json metric).

One "step" = one CG iteration with openmp::csvm::solver_CG semantics: one implicit Q~·p over the
whole problem + the device-resident vector updates + (N > 1) the per-iteration RCCL all-reduce.
Default workload = BASELINE.json configs[1]: dense RBF, 100k points x 256 features, fp64,
generate_data.py-style blobs (seeded, synthetic). N > 1 splits the same problem over the ranks
(strong scaling). Other configs (--config) are the sparse / fp32 rows of BASELINE.json.

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

import plssvm_sparse_fp22_amd as pm  # noqa: E402
from plssvm_sparse_fp22_amd import datagen  # noqa: E402

pm._abi.lib()  # load libplssvm_mi355x.so (and its RCCL, /opt/rocm/lib) before torch brings its own librccl

PEAKS = {"f64": 78.6e12, "f32": 157.3e12, "hbm": 8.0e12}  # MI355X_MICROARCH.md (dense MFMA, HBM3E)
METRIC = "CG iters/sec + implicit K·p HBM GB/s vs roofline, N×d stated, 1/2/4/8 GPU"

CONFIGS = {
    # name: kernel, N, d, dtype, layout, nnz/row, description
    "dense_rbf_100k": ("rbf", 100_000, 256, np.float64, "dense", 0,
                       "Dense RBF, 100k points x 256 features, fp64 (BASELINE configs[1])"),
    "dense_linear_500": ("linear", 500, 4, np.float64, "dense", 0,
                         "generate_data.py 500x4 dense, linear, fp64 (configs[0])"),
    "dense_linear_500k": ("linear", 500_000, 1024, np.float32, "dense", 0,
                          "Dense linear, 500k x 1024, fp32, MFMA pairwise (configs[3])"),
    "csr_linear_1m": ("linear", 1_000_000, 50_000, np.float32, "csr", 50,
                      "CSR-sparse linear, 1M x 50k @ 0.1% nnz, fp32, factored (configs[2])"),
    "csr_rbf_1m": ("rbf", 1_000_000, 50_000, np.float32, "csr", 50,
                   "CSR-sparse RBF, 1M x 50k @ 0.1% nnz, fp32 (configs[2] with RBF: the 70% HBM target)"),
    "fp22_rbf_2m": ("rbf", 2_000_000, 100_000, np.float32, "fp22", 50,
                    "COO/CSR RBF with FP22-packed features, 2M x 100k @ 0.05% nnz (configs[4])"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_problem(cfg, n_override, d_override, rank):
    kernel, n, d, dtype, layout, k, desc = cfg
    if n_override:
        if layout != "dense" and not d_override:  # keep the column occupancy c_f = n k / d fixed
            d = max(k, int(round(d * n_override / n)))
        n = n_override
    if d_override:
        d = d_override
    t0 = time.time()
    p = pm.Parameter(kernel, gamma=1.0 / d, real_type=dtype)
    if layout == "dense":
        X, y = datagen.blobs(n, d, seed=2, dtype=dtype)
        p.data, p.labels = X, y
        extra = dict(X=X)
    else:
        csr, y = datagen.sparse_csr(n, d, k, seed=3 if layout == "csr" else 5, dtype=dtype)
        if layout == "fp22":
            from plssvm_sparse_fp22_amd.fp22 import pack

            p.csr = (csr[0], csr[1], pack(csr[2]), n, d)
            p.val_fmt = pm._abi.VAL_FP22
        else:
            p.csr = csr
        p.labels = y
        extra = dict(csr=csr)
    log(f"[rank {rank}] {layout} data {n}x{d} {np.dtype(dtype).name} generated in {time.time() - t0:.1f}s")
    return p, n, d, y, extra


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="dense_rbf_100k", choices=sorted(CONFIGS))
    ap.add_argument("--points", type=int, default=0, help="override number of points (N)")
    ap.add_argument("--features", type=int, default=0, help="override number of features (d)")
    ap.add_argument("--kernel", choices=["linear", "polynomial", "rbf"], default=None,
                    help="override the configuration's kernel function (ablations)")
    ap.add_argument("--dtype", choices=["f32", "f64"], default=None,
                    help="override the configuration's real type (parity/throughput studies, not the headline line)")
    ap.add_argument("--kp-reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--sim-rank", default=None, metavar="R/W",
                    help="one GPU computes rank R's share of a W-GPU job (no collective): measures one rank of a "
                         "multi-GPU configuration that does not fit one GPU (e.g. configs[4])")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    dist = None
    uid = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        box = [pm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]

    cfg = CONFIGS[args.config]
    if args.kernel:
        cfg = (args.kernel,) + tuple(cfg[1:])
    if args.dtype:
        cfg = cfg[:3] + ({"f32": np.float32, "f64": np.float64}[args.dtype],) + tuple(cfg[4:])
    kernel, _, _, dtype, layout, _, desc = cfg
    p, n, d, y, extra = make_problem(cfg, args.points, args.features, rank)
    sim = None
    if args.sim_rank:
        if world > 1:
            raise SystemExit("--sim-rank is a single-process option")
        sim = tuple(int(v) for v in args.sim_rank.split("/"))
    ndev = pm.device_count()
    device = local_rank % ndev if ndev > 0 else local_rank  # more ranks than GPUs: share (rehearsal only)
    svm = pm.CSVM(p, device=device, rank=rank, world_size=world, uid=uid, sim_rank=sim)
    share = sim[1] if sim else world  # the work split divides the implicit matrix by this
    t0 = time.time()
    svm.setup_data_on_device()
    t_setup = time.time() - t0
    q = svm.generate_q()
    b = (y[:-1] - y[-1]).astype(dtype)
    delta0 = svm.cg_begin(b, q, eps=1e-3)
    log(f"[rank {rank}] setup {t_setup:.2f}s, q + r0 {time.time() - t0 - t_setup:.2f}s, delta0={delta0:.6e}")

    def barrier():
        if dist is not None:
            dist.barrier()

    if args.warmup:
        svm.cg_step(args.warmup, force=True)
    barrier()
    t_start = time.perf_counter()
    svm.cg_step(args.steps, force=True)  # ends with hipStreamSynchronize on the engine stream
    elapsed = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    iters_per_s = args.steps / elapsed

    info = svm.info()
    ms_kp, ms_dom = svm.time_kp(args.kp_reps)
    roof = roofline(cfg, info, n, d, share, ms_dom, extra)
    tkey = args.config + (f"_sim{sim[0]}of{sim[1]}" if sim else "")
    roof["traffic"], roof["traffic_source"] = pmc_traffic(tkey, n, d, world, roof["kernel"])
    if roof["bound"] == "mfma":
        roof["mfma_util"], roof["mfma_util_source"] = pmc_mfma(tkey, n, d, world, kernel)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(kernel, dtype, d, n - 1, args.cpu_seconds, extra)

    if rank == 0:
        out = {
            "metric": METRIC,
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
            "data": "synthetic (seeded generate_data.py-style blobs / sparse CSR)",
            "config": {"workload": desc, "N": n, "d": d, "kernel": kernel, "layout": layout,
                       "kp_mode": {1: "pairwise", 2: "factored"}[info["kp_mode"]],
                       "parallelism": f"x{world} GPUs: work split of the implicit matrix, RCCL all-reduce per K·p",
                       "setup_s": round(t_setup, 3)},
            "roofline": roof,
            "cpu_baseline": cpu,
            "kp_ms": ms_kp,
        }
        if sim:
            out["config"]["simulated_rank"] = f"{sim[0]}/{sim[1]}"
            out["config"]["parallelism"] = (f"one MI355X computing rank {sim[0]}'s share of a {sim[1]}-GPU job "
                                            "(no collective); value = CG iterations/s of that share")
        print(json.dumps(out), flush=True)
    svm.close()
    if dist is not None:
        dist.destroy_process_group()


def roofline(cfg, info, n, d, world, ms_dom, extra):
    kernel, _, _, dtype, layout, _, _ = cfg
    m = n - 1
    s = ms_dom * 1e-3
    if layout == "dense" and info["kp_mode"] == pm._abi.KP_PAIRWISE:
        pairs = m * (m + 1) / 2 * info["tiles_local"] / max(1, info["tiles_total"])
        alg = 2.0 * d * pairs  # Gram-block FLOP of this rank's lower-triangle tiles (GEMM form)
        pk = PEAKS["f64" if dtype == np.float64 else "f32"]
        return dict(bound="mfma", achieved=alg / s / 1e12, peak=pk / 1e12, unit="TFLOP/s", frac=alg / s / pk,
                    traffic=None, kernel="kp_tile_kernel", launch_ms=ms_dom, alg_flop_per_launch=alg,
                    alg_flop_per_kp_survey=(3.0 if kernel == "rbf" else 2.0) * d * m * (m + 1) / 2)
    es = np.dtype(dtype).itemsize
    if info["kp_mode"] == pm._abi.KP_FACTORED:
        if layout == "dense":
            alg = 2.0 * m * d * es / world
            kname = "gemv_t_kernel+gemv_n_kernel"
        else:
            nnz = info["nnz"]
            alg = (2 * (nnz * (4 + es) + (m + 1) * 8) + 4 * m * es + 2 * d * es) / world
            kname = "sell_spmv_kernel*2+panel_reduce_kernel*2"  # CSC pass + CSR pass
            moved = info["spmv_bytes"]  # what the two SELL passes actually stream (16-bit panel indices)
            return dict(bound="hbm", achieved=alg / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                        frac=alg / s / PEAKS["hbm"], traffic=None, kernel=kname, launch_ms=ms_dom, alg_bytes=alg,
                        stream_bytes_per_launch=moved, stream_GBps=moved / s / 1e9)
        return dict(bound="hbm", achieved=alg / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                    frac=alg / s / PEAKS["hbm"], traffic=None, kernel=kname, launch_ms=ms_dom, alg_bytes=alg)
    # sparse Gram pattern (poly / rbf): SURVEY §8(d) 3-RBF / 5 figure, this rank's share of the pairs
    col = extra["csr"][1]
    c = np.bincount(col, minlength=d).astype(np.float64)
    vb = 2.75 if layout == "fp22" else es
    co = float((c * (c + 1) / 2).sum())
    alg = (co * (4 + vb) + col.size * (4 + vb) + 3 * m * es) / world
    stream = info["pair_slots"] * (2 + es)  # stored slots (rows padded to 8 per cell)
    return dict(bound="hbm", achieved=alg / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s", frac=alg / s / PEAKS["hbm"],
                traffic=None, kernel="gram_kp_kernel", launch_ms=ms_dom, alg_bytes=alg,
                stream_bytes_per_launch=stream, stream_GBps=stream / s / 1e9, pairs=info["pairs"],
                pair_slots=info["pair_slots"])


def pmc_traffic(config, n, d, world, kernel):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC pass of this exact
    workload (profiles/*_<config>_traffic.json, written by tools/pmc_traffic.py), else None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_traffic.json")), reverse=True):
        t = json.load(open(path))
        if t["N"] == n and t["d"] == d and t["n_gpus"] == world and kernel == t["kernel"]:
            return t["hbm_read_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def pmc_mfma(config, n, d, world, kernel):
    """MFMA utilisation of the dense tile kernel from the newest committed PMC pass of this exact
    workload (profiles/*_<config>_mfma.json, written from tools/pmc_dense.sh), else None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_mfma.json")), reverse=True):
        t = json.load(open(path))
        if t["N"] == n and t["d"] == d and t["n_gpus"] == world and t["kernel"] == kernel:
            return t["mfma_util"], os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(kernel, dtype, d, m, budget_s, extra):
    """The oracle's OpenMP K·p (reference Release flags) on a leading-rows sample, scaled to N."""
    from oracle import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    gamma = np.dtype(dtype).type(1.0 / d)

    def sample(n_s):
        if "X" in extra:
            return pyoracle.Data(extra["X"][:n_s], dtype=dtype)
        rowptr, col, val, n, dd = extra["csr"]
        e = rowptr[n_s]
        return pyoracle.Data(rowptr=rowptr[: n_s + 1], col=col[:e], val=val[:e], n=n_s, d=dd, dtype=dtype)

    def run(n_s):
        data = sample(n_s)
        q = pyoracle.generate_q(kernel, data, gamma=gamma, fast=True)
        pvec = np.ones(n_s - 1, dtype=dtype)
        t = time.perf_counter()
        pyoracle.kp(kernel, data, q, dtype(1.0), dtype(1.0), 1.0, pvec, gamma=gamma, nthreads=threads, fast=True)
        return time.perf_counter() - t

    n_all = m + 1
    n_s = min(n_all, 3000)
    t = run(n_s)
    target = budget_s * 0.8
    if t < target and n_s < n_all:
        n_s = int(min(n_all, 60_000, n_s * math.sqrt(target / max(t, 1e-3))))
        t = run(n_s)
    ms = n_s - 1
    t_full = t * (m * (m + 1)) / (ms * (ms + 1))  # the reference kernel visits every lower-triangle pair
    return {"value": 1.0 / t_full, "unit": "CG iterations/s", "cores": threads, "kind": "port",
            "sample": f"one K·p of the oracle (reference OpenMP kernel restated, -O3 -ffast-math) on the first "
                      f"{n_s} of {n_all} points ({t:.2f}s), scaled by the lower-triangle pair count to N={n_all}",
            "pair_per_s": ms * (ms + 1) / 2 / t}


if __name__ == "__main__":
    main()
