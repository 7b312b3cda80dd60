#!/usr/bin/env python3
"""Predicted strong scaling of a W-GPU job from its measured rank shares (tools/sim_shares.sh).

Every rank's share of one CG iteration is measured on one MI355X (bench.py --sim-rank r/W: exactly that
rank's kernels, no collective); the job's iteration = the slowest share + the iteration's collectives,
which one GPU cannot measure. They are modelled per collective as  t = alpha + bytes / beta  (ring
algorithms over xGMI; bytes = what one GPU sends: all-gather (G-1)/G x total, all-reduce 2 (G-1)/G x
total) for a range of RCCL latencies alpha and bus bandwidths beta — an assumption, stated as such.

Collectives per CG iteration (engine.hip / sparse.hip / expand.hip) and what hides them:
  dense pairwise (replicated CG):   all-reduce of raw (m reals), exposed
  sparse expansion (sharded CG):    all-gather of w (m reals, or m bfloat16 + the ranks' S partials with
                                    bfloat16 windows; carries the pending direction partials),
                                    overlapping the rank's column-moment pass (expansion_kp_raw: the pass
                                    needs only the rank's own w) -> exposed max(0, t - t_moments);
                                    all-reduce of the column moments (d x KM reals) on the collective
                                    stream under the remainder stream -> exposed max(0, t - t_stream);
                                    2 all-gathers of 2 x 512 dot partials per rank, exposed
  sparse factored linear (sharded): all-reduce of w (d reals), 2 partial all-gathers, exposed
t_stream is the share's exp_hcell_kernel launch (roofline.launch_ms of the share record), t_moments the
column-moment pass of one share (optional argument, microseconds, from the share's kernel stats; 0 = no
credit).

With --cg1 (shares measured with bench.py --cg-variant one_reduction, the default of a sharded group since round 6)
the iteration's inner products travel in ONE all-gather of 4 x 512 partials per rank instead of two of 2 x 512.

usage: tools/predict_scaling.py [--cg1] <shares.jsonl> <one-GPU ms per iteration> [KM] [t_moments_us]
"""
import json
import sys

MODELS = [("fast", 8e-6, 200e9), ("mid", 12e-6, 150e9), ("slow", 20e-6, 100e9)]


CG1 = False


def collectives(rec, G, km):
    """(kind, bytes of the collective's whole buffer, name of the share's work that hides it or None)"""
    cfg = rec["config"]
    m, d = cfg["N"] - 1, cfg["d"]
    s = 8 if rec["dtype"] == "f64" else 4
    tiny = 2 * 512 * s * G  # gathered partials (bytes of the gathered buffer)
    if cfg["layout"] == "dense" and cfg["kp_mode"] == "pairwise":
        return [("allreduce", m * s, None)]
    if cfg["kp_mode"] == "factored":
        return [("allreduce", d * s, None)] + ([("allgather", 2 * tiny, None)] if CG1 else [("allgather", tiny, None)] * 2)
    # bfloat16 windows: the group gathers w as bfloat16 plus the ranks' S partials
    ws = 2 if "bfloat16" in str(rec["roofline"].get("h_storage", "")) else s
    extra = tiny if ws == 2 else 0
    dots = [("allgather", 2 * tiny, None)] if CG1 else [("allgather", tiny, None)] * 2
    return [("allgather", m * ws + tiny + extra, "moments"), ("allreduce", d * km * s, "stream")] + dots


def t_coll(kind, total, G, alpha, beta):
    f = (G - 1) / G * (2 if kind == "allreduce" else 1)
    return alpha + f * total / beta


def main():
    global CG1
    argv = sys.argv[1:]
    if argv and argv[0] == "--cg1":
        CG1, argv = True, argv[1:]
    rows = [json.loads(l) for l in open(argv[0]) if l.startswith("{")]
    one = float(argv[1])
    km = int(argv[2]) if len(argv) > 2 else 2
    t_mom = float(argv[3]) * 1e-6 if len(argv) > 3 else 0.0
    G = len(rows)
    ms = [r["ms_per_step"] for r in rows]
    out = {"config": rows[0]["config"]["workload"], "W": G, "ms_per_step_by_rank": ms, "max_share_ms": max(ms),
           "one_gpu_ms": one, "cg": "one-reduction" if CG1 else "reference", "predictions": {}}
    for name, alpha, beta in MODELS:
        c = 0.0
        for r in rows:  # the slowest rank's share + its exposed collective time
            hide = {"moments": t_mom, "stream": r["roofline"].get("launch_ms", 0.0) * 1e-3
                    if r["roofline"].get("kernel") == "exp_hcell_kernel" else 0.0, None: 0.0}
            exp = sum(max(0.0, t_coll(k, b, G, alpha, beta) - hide[h]) for k, b, h in collectives(r, G, km))
            c = max(c, r["ms_per_step"] + exp * 1e3)
        t = c
        c = t - max(ms)
        out["predictions"][name] = {"alpha_us": alpha * 1e6, "beta_GBps": beta / 1e9, "collectives_ms": round(c, 4),
                                    "iteration_ms": round(t, 4), "speedup": round(one / t, 2)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
