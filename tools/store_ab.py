"""A/B of the E-step store budgets along the converged chain (E1, M1, E2, M2,
E3 from M0, twice per setting so the second pass runs on mapped stores): per
"TRACE_GIB:REC_GIB" (0:0 = automatic) each E-step's groups, device ms and
wall ms, and the M-steps' ms.  LL and R_E must not depend on the budgets.

    python tools/store_ab.py CFG 0:0 130:88 ...
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1])
confs = sys.argv[2:] or ["0:0"]
p = synth.config_panel(cfg)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
P, _ = m.find_patterns()
print(f"cfg {cfg}: M0 {P} patterns", flush=True)
m.model_save()
for c in confs:
    tg, rg = (float(x) for x in c.split(":"))
    m.set_store_budgets(int(tg * (1 << 30)), int(rg * (1 << 30)))
    for rep in range(2):
        m.em_rewind()
        line = []
        for k in range(1, 4):
            t0 = time.perf_counter()
            ll, H, re = m.resolve_all()
            wall = time.perf_counter() - t0
            s = m.estep_split_stats()
            line.append(f"E{k} wall {wall * 1e3:.0f} struct {s['structure_ms']:.0f} ({s['structure_passes']}) values "
                        f"{s['values_ms']:.0f} ({s['value_passes']}) ll={ll!r} re={re}")
            if k < 3:
                t0 = time.perf_counter()
                m.find_patterns()
                line.append(f"M{k} {1e3 * (time.perf_counter() - t0):.0f}")
        print(f"{c} rep {rep}: " + " | ".join(line), flush=True)
