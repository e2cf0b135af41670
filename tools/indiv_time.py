"""Diagnostic build: distribution of per-individual E-step time (kcycles)."""
import sys, os
os.environ["HMC_AMD_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hmc_amd", "libhmc_amd_diag.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, hmc_amd
from hmc_amd import synth
m = hmc_amd.HaploModel()
m.set_estep_shape(int(os.environ.get('HMC_NW', '3')), 4)
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(int(sys.argv[1]) if len(sys.argv) > 1 else 2)))
m.find_patterns()
for it in range(3):
    m.resolve_all()
    t = m.frontier_max().astype(float)
    q = np.percentile(t, [0, 10, 50, 90, 99, 100])
    print(f"E{it+1} fwd {m.timings()['estep_forward_ms']:.1f} ms; per-individual kcycles: mean {t.mean():.0f} "
          f"pct0/10/50/90/99/100 {' '.join(f'{x:.0f}' for x in q)}; max/mean {t.max()/t.mean():.2f}")
    top = np.argsort(-t)[:5]
    print("   slowest individuals", top.tolist(), t[top].astype(int).tolist())
    m.find_patterns()
