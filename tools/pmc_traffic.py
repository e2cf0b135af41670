"""HBM traffic per launch of a kernel from two rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv KERNEL_REGEX OUT.json "command" [FETCH_BENCH.json [WRITE_BENCH.json]]

hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch — gfx950 tallies
128-B fabric reads at 64 B in FETCH_SIZE (MI355X_MICROARCH.md, HBM section);
both counters are in KiB.  With the bench line of the profiled run, the
algorithmic bytes of the same launches (8 B per retained link)
are added: the warmup steps are the first `warmup` steps of the same
deterministic chain, so they repeat the timed steps' R_E.  The two passes are
separate processes whose store budgets follow the free HBM each sees, so
their group counts can differ by a launch; with the WRITE pass's own bench
line each counter is divided by its own run's algorithmic bytes.
"""
import csv
import json
import re
import sys


def per_launch(path, counter, rx):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter or not re.search(rx, r["Kernel_Name"]):
            continue
        d = r["Dispatch_Id"]
        vals[d] = vals.get(d, 0.0) + float(r["Counter_Value"])
    return vals


fetch = per_launch(sys.argv[1], "FETCH_SIZE", sys.argv[3])
write = per_launch(sys.argv[2], "WRITE_SIZE", sys.argv[3])
fm = sum(fetch.values()) / max(1, len(fetch))
wm = sum(write.values()) / max(1, len(write))
out = {
    "kernel": sys.argv[3],
    "launches": len(fetch),
    "FETCH_SIZE_KiB_mean": fm,
    "WRITE_SIZE_KiB_mean": wm,
    "fetch_bytes_raw_per_launch": fm * 1024.0,
    "fetch_bytes_x2_per_launch": 2 * fm * 1024.0,
    "write_bytes_per_launch": wm * 1024.0,
    "correction": "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md HBM section: gfx950 FETCH_SIZE x2; "
                  "the x2 is specified for wide coalesced streams, so the raw FETCH is reported too)",
    "hbm_bytes_per_launch": (2 * fm + wm) * 1024.0,
    "hbm_bytes_raw_fetch_per_launch": (fm + wm) * 1024.0,
    "command": sys.argv[5] if len(sys.argv) > 5 else "",
}
def run_alg(path):
    """(algorithmic bytes, value-kernel launches) of every E-step of a profiled run"""
    b = json.loads(open(path).read().strip().splitlines()[-1])
    if "run_estep_log" in b:  # every E-step of the profiled process after M0, in order
        run = b["run_estep_log"]
        return sum(8.0 * r for r, _ in run), sum(v for _, v in run)
    steps, w = b["per_step"], b["warmup"]  # older lines: warmup + timed steps only
    run = steps[:w] + steps
    return sum(8.0 * s["r_e"] for s in run), sum(s["value_passes"] for s in run)


if len(sys.argv) > 6:
    try:  # the profiled build: bench.py reports traffic only for the library it loads itself
        out["library"] = json.loads(open(sys.argv[6]).read().strip().splitlines()[-1]).get("library")
    except (OSError, ValueError, IndexError):
        out["library"] = None
    alg, nl = run_alg(sys.argv[6])
    alg_w, nl_w = run_alg(sys.argv[7]) if len(sys.argv) > 7 else (alg, nl)
    out["alg_bytes_per_launch"] = alg / max(1, nl)
    out["alg_launches"] = nl
    out["alg_launches_write_run"] = nl_w
    out["launches_match"] = nl == len(fetch) and nl_w == len(write)
    # each pass over its own run's algorithmic bytes
    f_over = sum(2 * fetch[d] * 1024.0 for d in fetch) / alg if alg else None
    w_over = sum(write[d] * 1024.0 for d in write) / alg_w if alg_w else None
    out["fetch_x2_over_alg"] = f_over
    out["write_over_alg"] = w_over
    out["traffic_over_alg"] = f_over + w_over if f_over is not None and w_over is not None else None
    out["traffic_over_alg_raw_fetch"] = f_over / 2 + w_over if f_over is not None and w_over is not None else None
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
