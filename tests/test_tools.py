"""CPU tests of the measurement tools whose outputs DESIGN.md quotes: the scaling predictor's collective model
(tools/predict_scaling.py) and the traffic summary's layout tags (tools/pmc_traffic.py, matched by bench.py)."""
import json
import os
import subprocess
import sys

from conftest import ROOT

TOOLS = os.path.join(ROOT, "tools")


def share(ms, layout="fp22", kp_mode="pairwise", launch_ms=0.1, h="bfloat16 (precision bound, DESIGN §5.1.2)"):
    return {"ms_per_step": ms, "dtype": "f32", "config": {"workload": "w", "N": 2_000_000, "d": 100_000,
                                                          "layout": layout, "kp_mode": kp_mode},
            "roofline": {"kernel": "exp_hcell_kernel", "launch_ms": launch_ms, "h_storage": h}}


def run_predict(tmp_path, rows, one_ms, *extra, flags=()):
    f = tmp_path / "shares.jsonl"
    f.write_text("".join(json.dumps(r) + "\n" for r in rows))
    out = subprocess.run([sys.executable, os.path.join(TOOLS, "predict_scaling.py"), *flags, str(f), str(one_ms), *extra],
                         check=True, capture_output=True, text=True).stdout
    return json.loads(out)


def test_predict_scaling_collective_model(tmp_path):
    """iteration = slowest share + exposed collectives; the sparse expansion gathers w as bfloat16 (2 B per row)
    plus the ranks' S partials, all-reduces d x KM moments (hidden under the remainder stream) and gathers two
    sets of 2 x 512 dot partials; ring costs alpha + (G-1)/G x bytes / beta (x 2 for an all-reduce)"""
    rows = [share(0.22 + 0.001 * r) for r in range(8)]
    out = run_predict(tmp_path, rows, 1.3, "2", "0")
    assert out["W"] == 8 and abs(out["max_share_ms"] - 0.227) < 1e-12
    G, m, alpha, beta = 8, 2_000_000 - 1, 8e-6, 200e9
    tiny = 2 * 512 * 4 * G
    ag_w = alpha + (G - 1) / G * (m * 2 + 2 * tiny) / beta
    ar_mom = max(0.0, alpha + 2 * (G - 1) / G * (100_000 * 2 * 4) / beta - 0.1e-3)  # hidden under the stream
    ag_tiny = alpha + (G - 1) / G * tiny / beta
    want = 0.227e-3 + ag_w + ar_mom + 2 * ag_tiny
    got = out["predictions"]["fast"]["iteration_ms"] * 1e-3
    assert abs(got - want) < 1e-7, (got, want)
    assert out["predictions"]["fast"]["speedup"] == round(1.3e-3 / want, 2)
    # slower interconnect assumptions can only predict less
    sp = [out["predictions"][k]["speedup"] for k in ("fast", "mid", "slow")]
    assert sp[0] >= sp[1] >= sp[2]


def test_predict_scaling_one_reduction_cg(tmp_path):
    """--cg1 (the one-reduction CG of a sharded group): the iteration's dot partials travel in one all-gather of
    4 x 512 partials per rank instead of two of 2 x 512 — one latency fewer"""
    rows = [share(0.22 + 0.001 * r) for r in range(8)]
    ref = run_predict(tmp_path, rows, 1.3, "2", "0")
    one = run_predict(tmp_path, rows, 1.3, "2", "0", flags=("--cg1",))
    G, alpha, beta = 8, 8e-6, 200e9
    tiny = 2 * 512 * 4 * G
    saved = 2 * (alpha + (G - 1) / G * tiny / beta) - (alpha + (G - 1) / G * 2 * tiny / beta)
    got = (ref["predictions"]["fast"]["iteration_ms"] - one["predictions"]["fast"]["iteration_ms"]) * 1e-3
    assert one["cg"] == "one-reduction" and ref["cg"] == "reference"
    assert abs(got - saved) < 1e-7, (got, saved)


def test_predict_scaling_dense_allreduce(tmp_path):
    """dense pairwise: one exposed all-reduce of m reals per K·p"""
    rows = [share(5.0, layout="dense", h=None) for _ in range(8)]
    for r in rows:
        r["dtype"] = "f64"
        r["config"].update(N=100_000, d=256)
    out = run_predict(tmp_path, rows, 39.0)
    G, m = 8, 99_999
    want = 5.0e-3 + 8e-6 + 2 * (G - 1) / G * m * 8 / 200e9
    assert abs(out["predictions"]["fast"]["iteration_ms"] * 1e-3 - want) < 1e-7


def test_traffic_layout_tags_match_bench():
    """tools/pmc_traffic.py and bench.py name the remainder layouts the same way, so a FETCH pass measured on
    one stream layout is never applied to another"""
    sys.path.insert(0, TOOLS)
    try:
        import pmc_traffic
    finally:
        sys.path.remove(TOOLS)
    assert pmc_traffic.layout_tag({"h_storage": "bfloat16 (x)", "stream_layout": "4-slot chunks, row-start flags"}) == "bf16_flags"
    assert pmc_traffic.layout_tag({"h_storage": "bfloat16 (x)", "stream_layout": "4-slot chunks + row index"}) == "bf16"
    assert pmc_traffic.layout_tag({"h_storage": "real (4 B)", "stream_layout": "4-slot chunks + row index"}) == "real"
    assert pmc_traffic.layout_tag({}) is None
