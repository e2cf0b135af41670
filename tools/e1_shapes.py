"""E1 (the first E-step, on the genotype-mined model M0) under different launch
shapes: M0 once, then per shape hmc_em_rewind + one E-step.  Results must not
change with the shape (LL printed); times are device ms of the passes.

    python tools/e1_shapes.py CFG "s1nw:s1ipc:vnw:vipc[:traceGB:recGB]" ...   (0 = automatic)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1])
shapes = sys.argv[2:] or ["0:0:0"]
p = synth.config_panel(cfg)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
t0 = time.perf_counter()
P, _ = m.find_patterns()
print(f"M0 {P} patterns {time.perf_counter() - t0:.1f} s", flush=True)
m.model_save()
for sh in shapes:
    f = [int(x) for x in sh.split(":")] + [0, 0]
    m.set_pass_shapes(f[0], f[1], f[2], f[3])
    m.set_store_budgets(f[4] * 10**9, f[5] * 10**9)
    m.em_rewind()
    t0 = time.perf_counter()
    ll, H, re = m.resolve_all()
    wall = time.perf_counter() - t0
    s = m.estep_split_stats()
    print(f"shape {sh}: E1 wall {wall * 1e3:.0f} ms structure {s['structure_ms']:.0f} ms ({s['structure_passes']}) "
          f"values {s['values_ms']:.0f} ms ({s['value_passes']}) ll={ll!r} R_E={re}", flush=True)
