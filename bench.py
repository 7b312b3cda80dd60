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

CONFIG_DTYPE = {k: ("f64" if v[3] == np.float64 else "f32") for k, v in CONFIGS.items()}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_problem(cfg, n_override, d_override, rank, cache=None):
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
        key = (n, d, k, layout, np.dtype(dtype).name)
        if cache is not None and key in cache:
            csr, y = cache[key]
        else:
            csr, y = datagen.sparse_csr(n, d, k, seed=3 if layout == "csr" else 5, dtype=dtype)
            if cache is not None:
                cache.clear()  # one sparse matrix at a time (config 5 is 1e8 entries)
                cache[key] = (csr, y)
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


def collective_desc(world, sim, exchange):
    if sim:
        return (f"one MI355X computing rank {sim[0]}'s share of a {sim[1]}-GPU job (no collective); "
                "value = CG iterations/s of that share")
    if world == 1:
        return "single GPU, no collective"
    via = "host-staged exchange over gloo" if exchange else "RCCL over xGMI"
    return f"{world} GPUs, one process each: work split of the implicit matrix, one all-reduce of m per K·p ({via})"


def run_config(name, args, rank, world, dist, uid, steps, warmup, want_cpu, cpu_seconds, kp_reps, sim=None,
               kernel=None, dtype=None, points=0, features=0, data_cache=None, solve=False, solve_cap_s=20.0):
    """Measure one BASELINE configuration: setup, q, r0, `warmup` + `steps` CG iterations (timed with
    a barrier and stream synchronisation on both sides, max over ranks), the dominant kernel's
    average launch time (hipEvents on the engine stream), roofline, committed PMC traffic and the
    oracle's CPU baseline. Returns the record (bench-line keys) without the metric header."""
    cfg = CONFIGS[name]
    if kernel:
        cfg = (kernel,) + tuple(cfg[1:])
    if dtype:
        cfg = cfg[:3] + ({"f32": np.float32, "f64": np.float64}[dtype],) + tuple(cfg[4:])
    kern, _, _, dt, layout, _, desc = cfg
    p, n, d, y, extra = make_problem(cfg, points, features, rank, data_cache)
    ndev = pm.device_count()
    device = int(os.environ.get("LOCAL_RANK", str(rank))) % ndev if ndev > 0 else 0
    svm = pm.CSVM(p, device=device, rank=rank, world_size=world, uid=uid, sim_rank=sim,
                  sparse_algo=getattr(args, "sparse_algo", "auto") if layout != "dense" else "auto",
                  cg_variant=getattr(args, "cg_variant", None))
    share = sim[1] if sim else world  # the work split divides the implicit matrix by this
    t0 = time.time()
    svm.setup_data_on_device()
    t_setup = time.time() - t0
    q = svm.generate_q()
    b = (y[:-1] - y[-1]).astype(dt)
    delta0 = svm.cg_begin(b, q, eps=1e-3)
    log(f"[rank {rank}] {name}: setup {t_setup:.2f}s, q + r0 {time.time() - t0 - t_setup:.2f}s, delta0={delta0:.6e}")

    def barrier():
        if dist is not None:
            dist.barrier()

    if warmup:
        svm.cg_step(warmup, force=True)
    barrier()
    t_start = time.perf_counter()
    svm.cg_step(steps, force=True)  # ends with hipStreamSynchronize on the engine stream
    elapsed = time.perf_counter() - t_start
    barrier()
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    info = svm.info()
    ms_kp, ms_dom = svm.time_kp(kp_reps)
    learn = None
    if solve:
        # time to solution (csvm.cpp:226-266 reports setup and CG separately): the reference's learn() —
        # q, then CG from x0 = 1 at the default eps = 1e-3 with imax = num_features — on the resident data
        t_q0 = time.perf_counter()
        q = svm.generate_q()
        t_q = time.perf_counter() - t_q0
        # stepwise (the same device CG as solve_cg, 50-iteration graph blocks) so the bench stays bounded: a
        # solve that has not converged after solve_cap_s is reported with the iterations it reached
        t_cg0 = time.perf_counter()
        delta0 = svm.cg_begin(b, q, eps=1e-3)
        it, conv, batch = 0, False, 4
        while not conv and it < d and time.perf_counter() - t_cg0 < solve_cap_s:
            # solve_cg's polling: batches of 4, 8, 16, ... up to the first reset, then 50-iteration blocks
            nstep = min(batch, 50 - it % 50, d - it) if it < 50 else min(50 - it % 50, d - it)
            it, conv = svm.cg_step(nstep)
            batch *= 2
        t_cg = time.perf_counter() - t_cg0
        _, tr, _ = svm.cg_result(min(it + 1, 4096))
        learn = {"eps": 1e-3, "imax": d, "setup_s": round(t_setup, 3), "q_s": round(t_q, 4), "cg_iters": it,
                 "cg_s": round(t_cg, 4), "learn_s": round(t_setup + t_q + t_cg, 3), "converged": bool(conv),
                 "final_rel_residual": float(tr[-1] / delta0) if len(tr) else None,
                 "cap_s": solve_cap_s}
        log(f"[rank {rank}] {name}: learn at eps 1e-3: setup {t_setup:.2f}s + q {t_q:.3f}s + CG {it} iterations "
            f"{t_cg:.3f}s (converged: {conv})")
    svm.close()
    roof = roofline(cfg, info, n, d, share, ms_dom, extra, ms_kp)
    dts = "f64" if dt == np.float64 else "f32"
    tkey = name + (f"_sim{sim[0]}of{sim[1]}" if sim else "")
    hs = roof.get("h_storage")
    tag = None if hs is None else ("bf16" if hs.startswith("bfloat16") else "real") + \
        ("_pairs" if "slot pair" in roof.get("stream_layout", "") else "_flags" if "flags" in roof.get("stream_layout", "") else "")
    roof["traffic"], roof["traffic_source"] = pmc_traffic(tkey, n, d, world, roof["kernel"], dts, kern,
                                                          cfg is CONFIGS[name], tag)
    if roof["traffic"] and roof["bound"] == "hbm":
        roof["traffic_GBps"] = roof["traffic"] / (ms_dom * 1e-3) / 1e9
        roof["traffic_frac"] = roof["traffic_GBps"] * 1e9 / PEAKS["hbm"]
    if roof["bound"] == "mfma":
        roof["mfma_util"], roof["mfma_util_source"] = pmc_mfma(tkey, n, d, world, kern, dts)
    cpu = cpu_fact = None
    if want_cpu and rank == 0 and world == 1 and not sim:
        cpu = cpu_baseline(kern, dt, d, n - 1, cpu_seconds, extra)
        if layout != "dense" and kern == "linear":
            cpu_fact = cpu_baseline_factored(dt, extra, cpu_seconds * 0.5)
    rec = {
        "value": steps / elapsed, "unit": "CG iterations/s", "ms_per_step": elapsed / steps * 1e3, "steps": steps,
        "warmup": warmup, "dtype": dts,
        "config": {"workload": desc, "N": n, "d": d, "kernel": kern, "layout": layout,
                   "kp_mode": {1: "pairwise", 2: "factored"}[info["kp_mode"]],
                   "parallelism": collective_desc(world, sim, args.host_exchange), "setup_s": round(t_setup, 3)},
        "roofline": roof, "cpu_baseline": cpu, "kp_ms": ms_kp,
    }
    if cpu_fact is not None:
        rec["cpu_baseline_factored"] = cpu_fact
    if learn is not None:
        rec["learn"] = learn
    if info["is_sparse"]:
        rec["config"]["nnz"] = info["nnz"]
    if sim:
        rec["config"]["simulated_rank"] = f"{sim[0]}/{sim[1]}"
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="dense_rbf_100k", choices=sorted(CONFIGS))
    ap.add_argument("--points", type=int, default=0, help="override number of points (N)")
    ap.add_argument("--features", type=int, default=0, help="override number of features (d)")
    ap.add_argument("--kernel", choices=["linear", "polynomial", "rbf"], default=None,
                    help="override the configuration's kernel function (ablations)")
    ap.add_argument("--dtype", choices=["f32", "f64"], default=None,
                    help="override the configuration's real type (parity/throughput studies, not the headline line)")
    ap.add_argument("--kp-reps", type=int, default=3)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the sparse BASELINE rows measured beside the default headline (configs[2], 3-RBF)")
    ap.add_argument("--no-solve", action="store_true",
                    help="skip the default line's learn() timing (profiling runs: a converged solve's early-exit "
                         "launches would enter the kernel averages)")
    ap.add_argument("--host-exchange", action="store_true",
                    help="N > 1: exchange through the host over gloo (plssvm_mi_comm_init_host) instead of RCCL")
    ap.add_argument("--sim-rank", default=None, metavar="R/W",
                    help="one GPU computes rank R's share of a W-GPU job (no collective): measures one rank of a "
                         "multi-GPU configuration that does not fit one GPU (e.g. configs[4])")
    ap.add_argument("--cg-variant", default=None, choices=["reference", "one_reduction", "auto"],
                    help="CG recurrence (default: the library's auto: one-reduction in a sharded group of several ranks)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--sparse-algo", default="auto", choices=["auto", "pattern", "expansion", "dense", "onthefly"],
                    help="sparse poly/rbf K·p algorithm (PLSSVM_MI_OPT_SPARSE_ALGO; ablations / time-to-solution studies)")
    ap.add_argument("--solve", action="store_true",
                    help="also time the whole learn() at eps = 1e-3 (setup, q, CG to convergence): 'learn' record")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    uid = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("gloo")
        if not args.host_exchange:
            box = [pm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(box, src=0)
            uid = box[0]
    sim = None
    if args.sim_rank:
        if world > 1:
            raise SystemExit("--sim-rank is a single-process option")
        sim = tuple(int(v) for v in args.sim_rank.split("/"))
    if args.host_exchange and world > 1:
        _orig = pm.CSVM

        def _csvm(p, **kw):  # host-staged group (test transport / no-RCCL groups)
            kw.pop("uid", None)
            return _orig(p, exchange=pm.torch_exchange(dist), **kw)

        pm.CSVM = _csvm

    cache = {}
    default_cfg = args.config == "dense_rbf_100k" and not (args.kernel or args.dtype or args.points or args.features
                                                          or sim)
    default_run = default_cfg and world == 1
    rec = run_config(args.config, args, rank, world, dist, uid, args.steps, args.warmup, not args.no_cpu,
                     args.cpu_seconds, args.kp_reps, sim=sim, kernel=args.kernel, dtype=args.dtype,
                     points=args.points, features=args.features, data_cache=cache,
                     solve=(args.solve or default_run) and not args.no_solve and world == 1)
    extra = None
    if default_cfg and not args.no_extra:
        # the other BASELINE rows measured under the same clock. One GPU: configs[2] with RBF (the >= 70 % HBM
        # row), configs[2] itself (sparse linear, same seeded matrix), configs[4] (2M x 100k FP22 RBF, on one
        # GPU: the kernel expansion's memory is O(nnz + multi-feature pairs)) and configs[3] (dense linear
        # 500k x 1024 fp32 on the MFMA tiles, ~1.8 s per K·p). N > 1: the two 8-GPU rows of BASELINE
        # (configs[3], configs[4]) with the same max-over-ranks timing as the headline, so a 1/2/4/8 scaling
        # run yields their curves too.
        extra = {}
        if world == 1:
            rows = (("csr_rbf_1m", 50, 2), ("csr_linear_1m", 200, 2), ("fp22_rbf_2m", 30, 2), ("dense_linear_500k", 2, 1))
        else:
            rows = (("fp22_rbf_2m", 30, 2), ("dense_linear_500k", 3, 1))
        for name, steps, warm in rows:
            # an extra row that raises (every rank raises the same error: the engine's group protocol) is recorded
            # and the remaining rows skipped; the headline line is printed either way
            try:
                extra[name] = run_config(name, args, rank, world, dist, uid, steps, warm, not args.no_cpu,
                                         args.cpu_seconds * 0.6, args.kp_reps if steps >= 10 else 1, data_cache=cache,
                                         solve=world == 1)
            except Exception as e:  # noqa: BLE001
                log(f"[rank {rank}] extra {name} failed: {e!r}")
                extra[name] = {"error": repr(e)[:400]}
                break
    if rank == 0:
        out = {
            "metric": METRIC,
            "value": rec["value"],
            "unit": rec["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": rec["ms_per_step"],
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": rec["dtype"],
            "data": "synthetic (seeded generate_data.py-style blobs / sparse CSR)",
            "config": rec["config"],
            "roofline": rec["roofline"],
            "cpu_baseline": rec["cpu_baseline"],
            "kp_ms": rec["kp_ms"],
        }
        for k in ("cpu_baseline_factored", "learn"):
            if k in rec:
                out[k] = rec[k]
        if extra:
            out["extra"] = extra
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def kp_whole(streams, m, es, world, ms_kp):
    """The whole K·p against HBM: the bytes every kernel of one K·p must stream — the dominant
    stream(s) + the SELL passes' streams + the O(m) vectors (p read, the result written, e read: 3 m sizeof(real)
    per rank share) — over the whole K·p's time (time_kp: kp_device back to back, finalize included)."""
    b = streams + 3.0 * m * es / world
    return dict(kp_bytes=b, kp_ms=ms_kp, kp_GBps=b / (ms_kp * 1e-3) / 1e9, kp_frac=b / (ms_kp * 1e-3) / PEAKS["hbm"],
                kp_bytes_def="dominant stream + SELL pass streams (spmv_bytes) + 3 m sizeof(real) of vectors")


def roofline(cfg, info, n, d, world, ms_dom, extra, ms_kp=None):
    kernel, _, _, dtype, layout, _, _ = cfg
    m = n - 1
    s = ms_dom * 1e-3
    densified = info.get("sparse_algo") == pm._abi.SPARSE_DENSE  # sparse data on the dense MFMA tiles
    if (layout == "dense" or densified) and info["kp_mode"] == pm._abi.KP_PAIRWISE:
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
            r = dict(bound="hbm", achieved=alg / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                     frac=alg / s / PEAKS["hbm"], traffic=None, kernel=kname, launch_ms=ms_dom, alg_bytes=alg,
                     stream_bytes_per_launch=moved, stream_GBps=moved / s / 1e9,
                     stream_frac=moved / s / PEAKS["hbm"])  # on the bytes the passes move
            if ms_kp:
                r.update(kp_whole(moved, m, es, world, ms_kp))
            return r
        return dict(bound="hbm", achieved=alg / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                    frac=alg / s / PEAKS["hbm"], traffic=None, kernel=kname, launch_ms=ms_dom, alg_bytes=alg)
    # sparse Gram pattern (poly / rbf): SURVEY §8(d) 3-RBF / 5 figure, this rank's share of the pairs
    col = extra["csr"][1]
    c = np.bincount(col, minlength=d).astype(np.float64)
    vb = 2.75 if layout == "fp22" else es
    co = float((c * (c + 1) / 2).sum())
    survey = (co * (4 + vb) + col.size * (4 + vb) + 3 * m * es) / world
    if info.get("sparse_algo") == pm._abi.SPARSE_EXPANSION:
        # kernel expansion: the dominant kernel is the remainder stream of the pairs sharing
        # two or more features (uint16 j + H per slot, uint16 row per 4-slot chunk), read once per K·p;
        # the column-moment and Horner passes are the two SELL SpMV passes of the linear path
        hb = info["exp_hbytes"] or es
        # the stored row index: 2 B per 4-slot chunk in the indexed layout (exp_layout 1); none with row-start
        # flags (2: the dummies of empty cells are in pair_slots) or runs (3)
        rem = info["pair_slots"] * (2 + hb) + (info["exp_chunks"] * 2 if info["exp_layout"] == 1 else 0)
        whole = kp_whole(rem + info["spmv_bytes"], m, es, world, ms_kp) if ms_kp else {}
        return dict(**whole, bound="hbm", achieved=rem / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                    frac=rem / s / PEAKS["hbm"], traffic=None, kernel="exp_hcell_kernel", launch_ms=ms_dom,
                    alg_bytes=rem, alg_bytes_def="remainder stream: slots x (2 + bytes per stored H) + chunks x 2 (run layout: chunks = 0, slots = entries + dummies)",
                    h_storage="bfloat16 (precision bound, DESIGN §5.1.2)" if hb == 2 else f"real ({hb} B)",
                    stream_layout={1: "4-slot chunks + row index", 2: "4-slot chunks, row-start flags",
                                   3: "runs", 4: "4-slot chunks, row-start flags per slot pair (2-slot cells)"}.get(
                                       info["exp_layout"], "?"),
                    exp_terms=info["exp_terms"], multi_pairs=info["pairs"], pair_slots=info["pair_slots"],
                    spmv_bytes=info["spmv_bytes"], survey_alg_bytes=survey,
                    survey_effective_GBps=survey / s / 1e9, survey_effective_frac=survey / s / PEAKS["hbm"])
    # the kernel's algorithmic bytes: the stored pair stream it must read once per K·p (uint16 j + s_ij
    # per slot, rows padded to 8 per cell); SURVEY's column-join figure counts every co-occurrence
    # with multiplicity at 8 B, more than this algorithm needs, so it is reported as an effective rate
    stream = info["pair_slots"] * (2 + es)
    return dict(bound="hbm", achieved=stream / s / 1e9, peak=PEAKS["hbm"] / 1e9, unit="GB/s",
                frac=stream / s / PEAKS["hbm"], traffic=None, kernel="gram_kp_kernel", launch_ms=ms_dom,
                alg_bytes=stream, alg_bytes_def="stored pair stream: pair_slots x (2 + sizeof(real))",
                survey_alg_bytes=survey, survey_effective_GBps=survey / s / 1e9,
                survey_effective_frac=survey / s / PEAKS["hbm"], pairs=info["pairs"], pair_slots=info["pair_slots"])


def _pmc_match(t, n, d, world, dtype, kfun, default_cfg):
    """A committed PMC summary applies only to the exact workload: N, d, world, real type and kernel
    function (files written before these fields existed hold the configuration's defaults)."""
    if t["N"] != n or t["d"] != d or t["n_gpus"] != world:
        return False
    if "dtype" in t or "kernel_function" in t:
        return t.get("dtype") == dtype and t.get("kernel_function") == kfun
    return default_cfg


def pmc_traffic(config, n, d, world, kernel, dtype, kfun, default_cfg, tag=None):
    """HBM bytes per launch of the dominant kernel from the newest committed PMC pass of this exact
    workload (profiles/*_<config>_traffic.json, written by tools/pmc_traffic.py), else None. tag: the
    expansion's remainder layout ('bf16' / 'real'; files written before the tag existed measured 'real')."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_traffic.json")), reverse=True):
        t = json.load(open(path))
        if tag is not None and (t.get("layout_tag") or "real") != tag:
            continue
        if kernel == t["kernel"] and _pmc_match(t, n, d, world, dtype, kfun, default_cfg):
            return t["hbm_read_bytes_per_launch"], os.path.relpath(path, ROOT)
    return None, None


def pmc_mfma(config, n, d, world, kfun, dtype):
    """MFMA utilisation of the dense tile kernel from the newest committed PMC pass of this exact
    workload (profiles/*_<config>_mfma.json, written from tools/pmc_dense.sh), else None."""
    import glob

    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_mfma.json")), reverse=True):
        t = json.load(open(path))
        if t["N"] == n and t["d"] == d and t["n_gpus"] == world and t["kernel"] == kfun and \
                t.get("dtype", CONFIG_DTYPE.get(config)) == dtype:
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
    if "X" in extra:
        what = "the oracle (reference OpenMP kernel restated, -O3 -ffast-math)"
    else:
        # the reference itself densifies sparse input (parameter.cpp:66-87) and evaluates every pair over
        # all d features; its 32-bit indices cannot address configs 3 / 5 at all. The oracle's
        # CSR twin visits the same pairs but merges the two CSR rows per pair (O(nnz/row), not O(d))
        what = ("the oracle's CSR twin of the reference OpenMP kernel (every lower-triangle pair, CSR rows merged per "
                "pair instead of the reference's densified O(d) rows; -O3 -ffast-math)")
    return {"value": 1.0 / t_full, "unit": "CG iterations/s", "cores": threads, "kind": "port",
            "sample": f"one K·p of {what} on the first {n_s} of {n_all} points ({t:.2f}s), scaled by the "
                      f"lower-triangle pair count to N={n_all}",
            "pair_per_s": ms * (ms + 1) / 2 / t}


def cpu_baseline_factored(dtype, extra, budget_s):
    """The O(nnz) factored CPU K·p of sparse linear data at full size: w = X_m^T p,
    then X_m w + the rank-1 terms, OpenMP on all host threads (oracle/oracle_tmpl.h orc_kp_csr_factored)."""
    from oracle import pyoracle

    threads = int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))
    rowptr, col, val, n, d = extra["csr"]
    data = pyoracle.Data(rowptr=rowptr, col=col, val=val, n=n, d=d, dtype=dtype)
    m = n - 1
    q = np.ones(m, dtype=dtype)
    pvec = np.ones(m, dtype=dtype)
    ret = np.zeros(m, dtype=dtype)
    pyoracle.kp_csr_factored(data, q, dtype(1.0), 1.0, 1.0, pvec, ret, nthreads=threads)  # warm-up (page-in)
    reps, t0 = 0, time.perf_counter()
    while True:
        pyoracle.kp_csr_factored(data, q, dtype(1.0), 1.0, 1.0, pvec, ret, nthreads=threads)
        reps += 1
        t = time.perf_counter() - t0
        if t >= budget_s or reps >= 200:
            break
    return {"value": reps / t, "unit": "CG iterations/s (K·p only)", "cores": threads, "kind": "port",
            "sample": f"{reps} full-size K·p of the O(nnz) factored form X_m(X_m^T p) + rank-1 terms on the CSR data "
                      f"({t:.2f}s, OpenMP, -O3 -ffast-math): the honest CPU cost of the sparse linear product, "
                      f"which the reference (densifying, pairwise) does not implement"}


if __name__ == "__main__":
    main()
