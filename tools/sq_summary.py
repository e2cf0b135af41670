"""SQ counter summary per kernel from the two SQ passes of
tools/profile_round.sh (sq_SQ_WAVES_*.csv, sq_SQ_INSTS_LDS_*.csv).

usage: python tools/sq_summary.py SQ_WAVES.csv SQ_INSTS_LDS.csv [KERNEL_REGEX [OUT.json [BENCH.json]]]

Wave-cycle shares (quad-cycles summed over waves): parked = SQ_WAIT_ANY
(s_waitcnt / barrier), issue-stalled = SQ_WAIT_INST_ANY, issuing =
SQ_ACTIVE_INST_ANY, each over SQ_WAVE_CYCLES; instruction counts summed over
the kernel's launches; LDS bank-conflict cycles over LDS-active cycles.

Issue roofline of the kernel (the limiter of estep_values):
valu_issue_frac = SQ_INSTS_VALU x 4 cycles / (SIMDs x 2.4 GHz x kernel time),
kernel time = the sum of the launches' durations in the same pass (PMC runs
serialize kernels).  4 cycles is the issue cost of one wave's wave64 VALU
instruction on gfx950 (FP64 ops take 4 cycles of a SIMD; 32-bit ops 2 with
several waves per SIMD, so `valu_issue_frac_2cyc` is the lower bound);
MI355X_MICROARCH.md: 256 CUs x 4 SIMDs, 2 400 MHz.  With OUT.json the
summary is written there, with the library identity of the profiled run's
bench line (BENCH.json) so bench.py can refuse counters of another build.
"""
import collections
import csv
import json
import re
import sys

SIMDS = 256 * 4
CLOCK_HZ = 2.4e9


def load(path, rx):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    span = collections.defaultdict(dict)  # kernel -> dispatch -> ns
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not re.search(rx, name):
            continue
        k = name.split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        span[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return acc, span


def summarize(waves_csv, lds_csv, rx="estep_values"):
    """Per kernel: wave-cycle shares, instruction counts, LDS conflict ratio and
    the VALU issue fraction over the kernel time of the SQ_WAVES pass."""
    a, sa = load(waves_csv, rx)
    b, _ = load(lds_csv, rx)
    out = {}
    for k in sorted(set(a) | set(b)):
        x, y = a.get(k, {}), b.get(k, {})
        wc = x.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        valu, salu = x.get("SQ_INSTS_VALU", 0.0), x.get("SQ_INSTS_SALU", 0.0)
        t_s = sum(sa.get(k, {}).values()) * 1e-9
        cap = SIMDS * CLOCK_HZ * t_s
        out[k] = {
            "launches": len(sa.get(k, {})),
            "kernel_seconds": t_s,
            "parked": x.get("SQ_WAIT_ANY", 0.0) / wc,
            "issue_stalled": x.get("SQ_WAIT_INST_ANY", 0.0) / wc,
            "issuing": x.get("SQ_ACTIVE_INST_ANY", 0.0) / wc,
            "valu_insts": valu,
            "salu_insts": salu,
            "lds_insts": y.get("SQ_INSTS_LDS", 0.0),
            "lds_bank_conflict_ratio": y.get("SQ_LDS_BANK_CONFLICT", 0.0) / (y.get("SQ_ACTIVE_INST_LDS", 0.0) or 1.0),
            "valu_issue_frac": 4.0 * valu / cap if cap > 0 else None,
            "valu_issue_frac_2cyc": 2.0 * valu / cap if cap > 0 else None,
        }
    return out


def main():
    rx = sys.argv[3] if len(sys.argv) > 3 else "estep_values"
    s = summarize(sys.argv[1], sys.argv[2], rx)
    print("| kernel | waves parked | issue-stalled | issuing | VALU : SALU instructions | LDS instructions | "
          "LDS bank-conflict / LDS active | VALU issue (4 cyc) |")
    print("|---|---|---|---|---|---|---|---|")
    for k, d in s.items():
        vf = d["valu_issue_frac"]
        print(f"| `{k}` | {100 * d['parked']:.0f} % | {100 * d['issue_stalled']:.0f} % | {100 * d['issuing']:.0f} % | "
              f"{d['valu_insts'] / 1e12:.2f} : {d['salu_insts'] / 1e12:.2f} ·10¹² | {d['lds_insts'] / 1e12:.2f} ·10¹² | "
              f"{100 * d['lds_bank_conflict_ratio']:.0f} % | " + (f"{100 * vf:.0f} % |" if vf is not None else "- |"))
    if len(sys.argv) > 4:
        doc = {"kernels": s, "source": [sys.argv[1], sys.argv[2]],
               "formula": "valu_issue_frac = SQ_INSTS_VALU * 4 / (1024 SIMDs * 2.4e9 Hz * kernel seconds of the pass)"}
        if len(sys.argv) > 5:
            try:
                b = json.loads(open(sys.argv[5]).read().strip().splitlines()[-1])
                doc["library"] = b.get("library")
            except (OSError, ValueError, IndexError):
                doc["library"] = None
        json.dump(doc, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
