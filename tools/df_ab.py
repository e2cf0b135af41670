"""A/B of the value-pass schedules along the converged chain (E1, M1, E2, M2,
E3 from M0): per configuration "mode:ring:vnw:vipc[:sv[:na[:eo[:snw:sipc]]]]" (mode classic | dataflow | fused,
0 = automatic; sv = structure pass version 1 or 2; na = A waves of the dataflow pass;
eo = 0: structure pass over the id-ordered pattern table, 1 (default): end-locus order;
snw / sipc: structure-pass waves per individual / individuals per CU) the chain restarts from M0 (hmc_em_rewind) and each E-step's
device ms of the passes is printed.  LL and R_E must not depend on the
schedule.

    python tools/df_ab.py CFG classic:0:0:0 dataflow:3:0:0 ...
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1])
confs = sys.argv[2:] or ["classic:0:0:0", "dataflow:3:0:0"]
p = synth.config_panel(cfg)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
t0 = time.perf_counter()
P, _ = m.find_patterns()
print(f"cfg {cfg}: M0 {P} patterns {time.perf_counter() - t0:.1f} s", flush=True)
m.model_save()
for c in confs:
    f = c.split(":")
    mode, ring, vnw, vipc = f[:4]
    m.set_structure_pass(int(f[4]) if len(f) > 4 else 1)
    m.set_dataflow_waves(int(f[5]) if len(f) > 5 else 0)
    m.set_end_order(int(f[6]) if len(f) > 6 else 1)
    m.set_estep_mode(1 if mode == "fused" else 0)  # fused: the single-pass kernel (no record store)
    m.set_value_pass("classic" if mode == "fused" else mode, int(ring))
    m.set_pass_shapes(int(f[7]) if len(f) > 7 else 0, int(f[8]) if len(f) > 8 else 0, int(vnw), int(vipc))
    m.em_rewind()
    line = []
    for k in range(1, 4):
        t0 = time.perf_counter()
        ll, H, re = m.resolve_all()
        wall = time.perf_counter() - t0
        s = m.estep_split_stats()
        df = m.last_value_pass_dataflow()
        line.append(f"E{k} {'df' if df else 'cl'} wall {wall * 1e3:.0f} struct {s['structure_ms']:.0f} values "
                    f"{s['values_ms']:.0f} ({s['value_passes']}) ll={ll!r} re={re}")
        if k < 3:
            m.find_patterns()
    print(f"{c}: " + " | ".join(line), flush=True)
