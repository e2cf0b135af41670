"""The committed headline bench line against the bench.py contract and the
profile set it cites (CPU only: reads files under profiles/).

A bench line's roofline must be its own arithmetic (frac = achieved / peak,
value = individual·loci per step / step time), its traffic and VALU-issue
figures must come from a profile set of the same library build (sha256
prefix), and the rocprofv3 kernel trace of that set must agree with the
line's own HIP-event launch time.
"""
import csv
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADLINES = ["profiles/r06/bench/bench_cfg3_r06.json", "profiles/r06/bench/bench_cfg5_r06.json",
             "profiles/r06/bench/bench_cfg2_r06.json"]

REQUIRED = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"]


def _line(rel):
    path = os.path.join(ROOT, rel)
    if not os.path.exists(path):
        pytest.skip(f"{rel} not committed")
    with open(path) as f:
        return json.loads(f.read().strip().splitlines()[-1])


@pytest.mark.parametrize("rel", HEADLINES)
def test_headline_line_keeps_the_contract(rel):
    d = _line(rel)
    for k in REQUIRED:
        assert k in d, k
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert "workload" in d["config"]
    cfg = d["config"]
    # value = whole-job individual·loci per timed step over the step time
    assert d["value"] == pytest.approx(cfg["individuals"] * cfg["loci"] / (d["ms_per_step"] / 1e3), rel=1e-9)
    r = d["roofline"]
    for k in ["bound", "achieved", "peak", "unit", "frac", "traffic"]:
        assert k in r, k
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-12)
    assert r["unit"] == "GB/s" and r["peak"] == 8000.0
    # achieved = algorithmic bytes per launch / HIP-event launch time
    assert r["achieved"] == pytest.approx(r["alg_bytes_per_launch"] / (r["avg_launch_ms"] / 1e3) / 1e9, rel=1e-9)
    cb = d["cpu_baseline"]
    for k in ["value", "unit", "cores", "kind", "sample"]:
        assert k in cb, k
    assert cb["kind"] in ("port", "reference") and cb["cores"] >= 1 and cb["value"] > 0


@pytest.mark.parametrize("rel", HEADLINES)
def test_headline_counters_from_the_same_build(rel):
    d = _line(rel)
    sha = d["library"]["sha256_16"]
    r = d["roofline"]
    assert r["traffic_same_build"] and r["valu_issue_same_build"]
    assert r["traffic"] is not None and r["valu_issue_frac"] is not None
    with open(os.path.join(ROOT, r["traffic_source"])) as f:
        pmc = json.load(f)
    assert pmc["library"]["sha256_16"] == sha and pmc["launches_match"]
    assert r["traffic_over_alg"] == pytest.approx(pmc["traffic_over_alg"], rel=1e-12)
    with open(os.path.join(ROOT, r["valu_issue_source"])) as f:
        sq = json.load(f)
    assert sq["library"]["sha256_16"] == sha
    # the bound is the larger measured fraction, or latency when both are small
    frac = max(r["valu_issue_frac"], r["hbm_frac_measured"])
    want = "latency" if frac < 0.5 else ("valu-issue" if r["valu_issue_frac"] >= r["hbm_frac_measured"] else "hbm")
    assert r["bound"] == want


@pytest.mark.parametrize("rel", HEADLINES)
def test_headline_launch_time_agrees_with_kernel_trace(rel):
    d = _line(rel)
    r = d["roofline"]
    tag = d["config"]["workload"].split(":")[0]  # "cfg3", "cfg5", ...
    stats = os.path.join(os.path.dirname(os.path.join(ROOT, r["traffic_source"])), f"kernel_stats_{tag}.csv")
    with open(stats) as f:
        rows = [row for row in csv.DictReader(f) if "estep_values" in row["Name"]]
    calls = sum(int(row["Calls"]) for row in rows)
    avg_ms = sum(float(row["TotalDurationNs"]) for row in rows) / calls / 1e6
    assert avg_ms == pytest.approx(r["avg_launch_ms"], rel=0.05)
