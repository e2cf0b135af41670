import sys, os
sys.path.insert(0, os.getcwd())
import hmc_amd
from hmc_amd import synth
p = synth.founder_mosaic(10000, 1000, A=8, missing=0.0, seed=5)
g = hmc_amd.GenoData.from_panel(p)
for nw in [3, 4, 3, 4]:
    m = hmc_amd.HaploModel(); m.set_estep_shape(nw, 4); m.load(g); m.find_patterns()
    out = []
    for it in range(3):
        ll, H, re = m.resolve_all(); t = m.timings(); sp = m.estep_split_stats()
        out.append(f"E{it+1} {t['estep_forward_ms']:.1f}ms (s {sp['structure_ms']:.1f} v {sp['values_ms']:.1f}) ll={ll:.6f}")
        m.find_patterns()
    print(f"nw {nw}: " + " | ".join(out), flush=True)
    del m
