"""VALU issue calibration (round 6): what one wave64 VALU instruction costs a
gfx950 SIMD, from tools/diag/issue_bench.hip's kernels under rocprofv3, and the
same measure applied to the selection microbenchmark (coop_bench mode 5,
seg2_nth_slots at 4 waves per SIMD) and to the E-step passes of a short cfg 3
bench.

usage: python tools/issue_calib.py DIR [OUT.json]
  DIR holds ib_{BUSY,MIX}/ or ib_{BUSY,MIX}.csv (issue_bench 1024 under --pmc), issue_cpi.json
  (issue_bench stamps), cb_{BUSY,MIX}/ (coop_bench 32 2000 5 10) and
  b3_{BUSY,MIX}/ (bench.py --config 3 --steps 2 --warmup 0), as written by the
  round-6 GPU run (profiles/r06/issue/cmd.sh).

The busy pass counts SQ_INSTS_VALU, SQ_ACTIVE_INST_VALU2 (quad-cycles in which
a SIMD issued two VALU instructions) and SQ_BUSY_CYCLES (cycles with waves,
summed over the 32 shader engines).  A SIMD issues one VALU instruction per
quad-cycle, or two that dual-issue, so the SIMD cycles spent issuing VALU are
4 x (VALU - VALU2) and
  occupancy      = 4 (VALU - VALU2) / (32 SIMDs per SE x BUSY)
  cycles / inst  = 4 (VALU - VALU2) / VALU      (= 4 without dual issue)
For the issue_bench kernels at 4 and 8 waves per SIMD the occupancy is the
issue roof itself (their instruction streams have no other wait), which checks
the formula; for the real kernels it is how close they run to that roof.
"""
import collections
import csv
import glob
import json
import os
import sys

SE, SIMDS_PER_SE = 32, 32
OPS = ["v_add_u32", "v_cndmask_b32_e64", "v_add_f64", "v_mul_f64", "v_cmp_gt_f64_e64", "v_lshlrev_b64", "v_mov_b32",
       "v_fma_f32"]
WAVES = [1, 2, 4, 8]


def load(d, per_dispatch=False):
    """Counters of one pass: a rocprofv3 output directory, or the same name + .csv (committed copies)."""
    f = d + ".csv" if os.path.exists(d + ".csv") else glob.glob(os.path.join(d, "**", "*counter_collection.csv"),
                                                                  recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    span = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if per_dispatch:
            k = (k, int(r["Dispatch_Id"]))
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        span[k][r["Dispatch_Id"]] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
    return acc, span


def issue(v):
    v1, v2, b = v.get("SQ_INSTS_VALU", 0.0), v.get("SQ_ACTIVE_INST_VALU2", 0.0), v.get("SQ_BUSY_CYCLES", 0.0)
    return {"valu": v1, "dual_share": 2 * v2 / v1 if v1 else 0.0, "cycles_per_inst": 4 * (v1 - v2) / v1 if v1 else 0.0,
            "occupancy": 4 * (v1 - v2) / (SIMDS_PER_SE * b) if b else None}


def main():
    d = sys.argv[1]
    out = {"formula": "occupancy = 4 (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / (32 SIMDs per SE x SQ_BUSY_CYCLES); "
                      "cycles per instruction = 4 (VALU - VALU2) / VALU"}
    # issue_bench: dispatches in launch order, two per (op, W) (the first warms the clocks)
    acc, span = load(os.path.join(d, "ib_BUSY"), per_dispatch=True)
    keys = sorted(acc, key=lambda k: k[1])
    rows = []
    print("| instruction | waves / SIMD | cycles per instruction (issue) | dual-issue share | VALU issue occupancy |")
    print("|---|---|---|---|---|")
    for i, k in enumerate(keys[1::2]):
        op, w = OPS[i // len(WAVES)], WAVES[i % len(WAVES)]
        x = issue(acc[k])
        x.update(op=op, waves_per_simd=w)
        rows.append(x)
        print(f"| `{op}` | {w} | {x['cycles_per_inst']:.2f} | {100 * x['dual_share']:.0f} % | {100 * x['occupancy']:.0f} % |")
    out["issue_bench"] = rows
    try:
        out["issue_bench_stamps"] = json.load(open(os.path.join(d, "issue_cpi.json")))
    except (OSError, ValueError):
        pass
    for tag, name in (("cb", "coop_bench mode 5 (seg2_nth_slots, S = 10, 16 waves per CU)"),
                      ("b3", "bench.py --config 3 --steps 2 --warmup 0")):
        try:
            a, sa = load(os.path.join(d, f"{tag}_BUSY"))
            m, _ = load(os.path.join(d, f"{tag}_MIX"))
        except (IndexError, OSError):
            continue
        print(f"\n{name}:\n")
        print("| kernel | VALU instructions | cycles per instruction | dual-issue share | VALU issue occupancy | INT32 | INT64 | FP64 add/mul/fma | clock GHz |")
        print("|---|---|---|---|---|---|---|---|---|")
        res = {}
        for k in a:
            x = issue(a[k])
            t = sum(sa[k].values()) * 1e-9
            x["clock_ghz"] = a[k].get("SQ_BUSY_CYCLES", 0.0) / SE / t / 1e9 if t else None
            mm = m.get(k, {})
            tot = mm.get("SQ_INSTS_VALU") or 1.0
            x["mix"] = {c.replace("SQ_INSTS_VALU_", ""): mm.get(c, 0.0) / tot
                        for c in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_ADD_F64",
                                  "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")}
            res[k] = x
            f64 = x["mix"]["ADD_F64"] + x["mix"]["MUL_F64"] + x["mix"]["FMA_F64"]
            print(f"| `{k}` | {x['valu']:.3e} | {x['cycles_per_inst']:.2f} | {100 * x['dual_share']:.0f} % | "
                  f"{100 * x['occupancy']:.0f} % | {100 * x['mix']['INT32']:.0f} % | {100 * x['mix']['INT64']:.0f} % | "
                  f"{100 * f64:.1f} % | {x['clock_ghz']:.2f} |")
        out[tag] = res
    if len(sys.argv) > 2:
        json.dump(out, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
