"""SQ counter summary per kernel from the SQ passes of tools/profile_round.sh
(sq_SQ_WAVES_*.csv, sq_SQ_INSTS_LDS_*.csv, and since round 6 sq_SQ_ACTIVE_INST_VALU_*.csv,
the "busy" pass, and sq_SQ_INSTS_VALU_INT32_*.csv, the instruction-mix pass).

usage: python tools/sq_summary.py SQ_WAVES.csv SQ_INSTS_LDS.csv [KERNEL_REGEX [OUT.json [BENCH.json [BUSY.csv [MIX.csv]]]]]

Wave-cycle shares (quad-cycles summed over waves): parked = SQ_WAIT_ANY
(s_waitcnt / barrier), issue-stalled = SQ_WAIT_INST_ANY, issuing =
SQ_ACTIVE_INST_ANY, each over SQ_WAVE_CYCLES; instruction counts summed over
the kernel's launches; LDS bank-conflict cycles over LDS-active cycles.

Issue roofline of the kernel (the limiter of estep_values),
MEASURED (round 6, profiles/r06/issue/): a SIMD issues one VALU instruction
per quad-cycle, or two from different waves when both can dual-issue
(SQ_ACTIVE_INST_VALU2 counts those quad-cycles; tools/diag/issue_bench.hip:
v_add_u32 / v_mov_b32 pair up, FP64 ops, v_cndmask_b32_e64, v_cmp_*_f64 and
64-bit shifts do not — 4 cycles each at any occupancy).  So
  valu_issue_frac = 4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2)
                    / (32 SIMDs per SE x SQ_BUSY_CYCLES)
where SQ_BUSY_CYCLES sums the cycles with active waves over the 32 shader
engines (8 XCDs x 4), at the clock the kernel actually ran (also reported).
The older nominal figures — 4 or 2 cycles per SQ_INSTS_VALU over 1 024 SIMDs
x 2.4 GHz x the kernel time — stay in the JSON as *_nominal.  With OUT.json the
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
SE = 32               # shader engines (8 XCDs x 4); SQ_BUSY_CYCLES is summed over them
SIMDS_PER_SE = SIMDS // SE
MIX_KEYS = ["SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
            "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_TRANS_F64"]


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


def summarize(waves_csv, lds_csv, rx="estep_values", busy_csv=None, mix_csv=None):
    """Per kernel: wave-cycle shares, instruction counts, LDS conflict ratio and
    the VALU issue fraction — measured from the busy pass when given, else the
    nominal 4-cycle figure over the kernel time of the SQ_WAVES pass."""
    a, sa = load(waves_csv, rx)
    b, _ = load(lds_csv, rx)
    c, sc = load(busy_csv, rx) if busy_csv else ({}, {})
    mx, _ = load(mix_csv, rx) if mix_csv else ({}, {})
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
            "valu_issue_frac_nominal": 4.0 * valu / cap if cap > 0 else None,
            "valu_issue_frac_2cyc_nominal": 2.0 * valu / cap if cap > 0 else None,
        }
        z = c.get(k)
        if z and z.get("SQ_BUSY_CYCLES"):
            v1, v2, busy = z.get("SQ_INSTS_VALU", 0.0), z.get("SQ_ACTIVE_INST_VALU2", 0.0), z["SQ_BUSY_CYCLES"]
            tb = sum(sc.get(k, {}).values()) * 1e-9
            out[k].update({
                "valu_issue_frac": 4.0 * (v1 - v2) / (SIMDS_PER_SE * busy),
                "valu_dual_issue_share": 2.0 * v2 / v1 if v1 else None,
                "valu_cycles_per_inst": 4.0 * (v1 - v2) / v1 if v1 else None,
                "clock_ghz": busy / SE / tb / 1e9 if tb > 0 else None,
                "busy_pass": {kk: z.get(kk) for kk in ("SQ_INSTS_VALU", "SQ_ACTIVE_INST_VALU2", "SQ_BUSY_CYCLES",
                                                       "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE")},
            })
        else:
            out[k]["valu_issue_frac"] = None
        m = mx.get(k)
        if m and m.get("SQ_INSTS_VALU"):
            out[k]["valu_mix"] = {kk.replace("SQ_INSTS_VALU_", ""): m.get(kk, 0.0) / m["SQ_INSTS_VALU"] for kk in MIX_KEYS}
    return out


def main():
    rx = sys.argv[3] if len(sys.argv) > 3 else "estep_values"
    busy = sys.argv[6] if len(sys.argv) > 6 else None
    mix = sys.argv[7] if len(sys.argv) > 7 else None
    s = summarize(sys.argv[1], sys.argv[2], rx, busy, mix)
    print("| kernel | waves parked | issue-stalled | issuing | VALU : SALU instructions | LDS instructions | "
          "LDS bank-conflict / LDS active | VALU issue, measured (dual-issue share) | nominal 4 cyc |")
    print("|---|---|---|---|---|---|---|---|---|")
    for k, d in s.items():
        vf, vn = d["valu_issue_frac"], d["valu_issue_frac_nominal"]
        print(f"| `{k}` | {100 * d['parked']:.0f} % | {100 * d['issue_stalled']:.0f} % | {100 * d['issuing']:.0f} % | "
              f"{d['valu_insts'] / 1e12:.2f} : {d['salu_insts'] / 1e12:.2f} ·10¹² | {d['lds_insts'] / 1e12:.2f} ·10¹² | "
              f"{100 * d['lds_bank_conflict_ratio']:.0f} % | "
              + (f"{100 * vf:.0f} % ({100 * d['valu_dual_issue_share']:.0f} %) |" if vf is not None else "- |")
              + (f" {100 * vn:.0f} % |" if vn is not None else " - |"))
    if len(sys.argv) > 4:
        doc = {"kernels": s, "source": [x for x in sys.argv[1:3] + sys.argv[6:8]],
               "formula": "valu_issue_frac = 4 * (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / (32 SIMDs per SE * "
                          "SQ_BUSY_CYCLES), measured issue (profiles/r06/issue/); *_nominal = SQ_INSTS_VALU * 4 (or 2) "
                          "/ (1024 SIMDs * 2.4e9 Hz * kernel seconds)"}
        if len(sys.argv) > 5:
            try:
                b = json.loads(open(sys.argv[5]).read().strip().splitlines()[-1])
                doc["library"] = b.get("library")
            except (OSError, ValueError, IndexError):
                doc["library"] = None
        json.dump(doc, open(sys.argv[4], "w"), indent=1)


if __name__ == "__main__":
    main()
