"""Variance check: the same E-step (E_2 of cfg2) repeated."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd
from hmc_amd import synth
m = hmc_amd.HaploModel()
if len(sys.argv) > 1:
    nw, ipc = (int(x) for x in sys.argv[1].split(':'))
    m.set_estep_shape(nw, ipc)
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(2)))
m.find_patterns()
m.resolve_all()
m.find_patterns()
out = []
for r in range(8):
    ll, H, re = m.resolve_all()
    t = m.timings()
    out.append(f"{t['estep_forward_ms']:.1f}")
print(sys.argv[1:] or "default", "E2 x8 fwd ms:", " ".join(out), "| fmax", int(m.frontier_max().max()))
