"""HBM traffic per launch of a kernel from two rocprofv3 PMC passes.

usage: python tools/pmc_traffic.py FETCH.csv WRITE.csv KERNEL_REGEX OUT.json "command" [BENCH.json]

hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 per launch — gfx950 tallies
128-B fabric reads at 64 B in FETCH_SIZE (MI355X_MICROARCH.md, HBM section);
both counters are in KiB.  With the bench line of the profiled run, the
algorithmic bytes of the same launches (8 B per retained link)
are added: the warmup steps are the first `warmup` steps of the same
deterministic chain, so they repeat the timed steps' R_E.
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
if len(sys.argv) > 6:
    b = json.loads(open(sys.argv[6]).read().strip().splitlines()[-1])
    if "run_estep_log" in b:  # every E-step of the profiled process after M0, in order
        run = b["run_estep_log"]
        alg = sum(8.0 * r for r, _ in run)
        nl = sum(v for _, v in run)
    else:  # older lines: warmup + timed steps only (misses the steady leg)
        steps, w = b["per_step"], b["warmup"]
        run = steps[:w] + steps
        alg = sum(8.0 * s["r_e"] for s in run)
        nl = sum(s["value_passes"] for s in run)
    out["alg_bytes_per_launch"] = alg / max(1, nl)
    out["alg_launches"] = nl
    out["launches_match"] = nl == len(fetch) == len(write)
    # the same launches on both sides: all PMC bytes over all algorithmic bytes
    tot = sum(2 * fetch[d] * 1024.0 for d in fetch) + sum(write[d] * 1024.0 for d in write)
    out["traffic_over_alg"] = tot / alg if alg else None
    out["write_over_alg"] = sum(write.values()) * 1024.0 / alg if alg else None
json.dump(out, open(sys.argv[4], "w"), indent=1)
print(json.dumps(out))
