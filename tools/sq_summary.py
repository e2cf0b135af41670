"""SQ counter summary per kernel from the two SQ passes of
tools/profile_round.sh (sq_SQ_WAVES_*.csv, sq_SQ_INSTS_LDS_*.csv).

usage: python tools/sq_summary.py SQ_WAVES.csv SQ_INSTS_LDS.csv [KERNEL_REGEX]

Wave-cycle shares (quad-cycles summed over waves): parked = SQ_WAIT_ANY
(s_waitcnt / barrier), issue-stalled = SQ_WAIT_INST_ANY, issuing =
SQ_ACTIVE_INST_ANY, each over SQ_WAVE_CYCLES; instruction counts summed over
the kernel's launches; LDS bank-conflict cycles over LDS-active cycles.
"""
import collections
import csv
import re
import sys


def load(path, rx):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if not re.search(rx, name):
            continue
        k = name.split("(")[0].replace("void ", "")
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


rx = sys.argv[3] if len(sys.argv) > 3 else "estep_values"
a = load(sys.argv[1], rx)
b = load(sys.argv[2], rx)
print("| kernel | waves parked | issue-stalled | issuing | VALU : SALU instructions | LDS instructions | "
      "LDS bank-conflict / LDS active |")
print("|---|---|---|---|---|---|---|")
for k in sorted(set(a) | set(b)):
    x, y = a.get(k, {}), b.get(k, {})
    wc = x.get("SQ_WAVE_CYCLES", 0.0) or 1.0
    parked = x.get("SQ_WAIT_ANY", 0.0) / wc
    stall = x.get("SQ_WAIT_INST_ANY", 0.0) / wc
    issue = x.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
    valu, salu = x.get("SQ_INSTS_VALU", 0.0), x.get("SQ_INSTS_SALU", 0.0)
    lds = y.get("SQ_INSTS_LDS", 0.0)
    conf = y.get("SQ_LDS_BANK_CONFLICT", 0.0) / (y.get("SQ_ACTIVE_INST_LDS", 0.0) or 1.0)
    print(f"| `{k}` | {100 * parked:.0f} % | {100 * stall:.0f} % | {100 * issue:.0f} % | "
          f"{valu / 1e12:.2f} : {salu / 1e12:.2f} ·10¹² | {lds / 1e12:.2f} ·10¹² | {100 * conf:.0f} % |")
