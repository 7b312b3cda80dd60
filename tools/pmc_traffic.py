#!/usr/bin/env python3
"""Summarise a tools/profile_config.sh run into profiles/ (runs here, after gpurun merged the outputs).

Writes profiles/<round>_<config>_kernel_stats.csv (rocprofv3 --stats summary, copied),
profiles/<round>_<config>_bench.json (the bench line of the traced run) and
profiles/<round>_<config>_traffic.json: HBM read bytes per launch of the dominant kernel from the
FETCH_SIZE pass, corrected as MI355X_MICROARCH.md's HBM section prescribes (FETCH_SIZE is in KiB and
on gfx950 counts half the bytes of wide coalesced streaming reads: x 1024 x 2).
bench.py reads the traffic file back into roofline.traffic for the same config and N x d.

usage: tools/pmc_traffic.py <tag> <config> <round-prefix, e.g. r01>
"""
import csv
import glob
import gzip
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def layout_tag(roof):
    """'bf16' / 'real' for the kernel expansion's remainder stream (roofline.h_storage), else None"""
    hs = roof.get("h_storage")
    if hs is None:
        return None
    lay = roof.get("stream_layout", "")
    return ("bf16" if hs.startswith("bfloat16") else "real") + ("_pairs" if "slot pair" in lay else "_flags" if "flags" in lay else "")


def find(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


def main():
    tag, config, rnd = sys.argv[1:4]
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    bench = json.loads(open(os.path.join(src, "bench_trace.json")).read().strip().splitlines()[-1])
    # the dominant launch may be several kernels; "name*k" = k dispatches of that kernel per launch
    parts = [k.split("*") for k in bench["roofline"]["kernel"].split("+")]
    kernels = [p[0] for p in parts]
    mult = {p[0]: int(p[1]) if len(p) > 1 else 1 for p in parts}
    stats = find(os.path.join(src, "trace", "**", "*kernel_stats.csv"))
    prof = os.path.join(ROOT, "profiles")
    shutil.copy(stats, os.path.join(prof, f"{rnd}_{config}_kernel_stats.csv"))
    with open(os.path.join(prof, f"{rnd}_{config}_bench.json"), "w") as f:
        json.dump(bench, f, indent=1)
    avg = {}
    for row in csv.DictReader(open(stats)):
        for k in kernels:
            if k in row["Name"] and k not in avg:
                avg[k] = float(row["AverageNs"])
    avg_ns = sum(avg[k] * mult[k] for k in avg) if len(avg) == len(kernels) else None
    vals = {k: [] for k in kernels}
    pmc = find(os.path.join(src, "pmc", "**", "*counter_collection.csv*"))
    with (gzip.open(pmc, "rt") if pmc.endswith(".gz") else open(pmc)) as f:
        for row in csv.DictReader(f):
            for k in kernels:
                if row["Counter_Name"] == "FETCH_SIZE" and k in row["Kernel_Name"]:
                    vals[k].append(float(row["Counter_Value"]))
    if not all(vals.values()):
        raise SystemExit(f"no FETCH_SIZE rows for {kernels}")
    fetch_kib = sum(statistics.mean(v) * mult[k] for k, v in vals.items())
    out = {
        "config": config, "N": bench["config"]["N"], "d": bench["config"]["d"], "n_gpus": bench["n_gpus"],
        "dtype": bench["dtype"], "kernel_function": bench["config"]["kernel"],
        "kernel": bench["roofline"]["kernel"], "dispatches": min(len(v) for v in vals.values()), "fetch_size_kib_mean": fetch_kib,
        "hbm_read_bytes_per_launch": fetch_kib * 1024 * 2,
        "correction": "FETCH_SIZE KiB x 1024 x 2 (gfx950 counts half of wide streaming reads)",
        "rocprof_avg_ms": None if avg_ns is None else avg_ns * 1e-6,
        "bench_launch_ms": bench["roofline"].get("launch_ms"),
        # the stream layout the counters saw (bench.py matches it: a bfloat16 remainder moves other bytes)
        "layout_tag": layout_tag(bench["roofline"]),
    }
    with open(os.path.join(prof, f"{rnd}_{config}_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
