"""One cfg2 E-step (E_1) on the GPU, for profiler runs."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd
from hmc_amd import synth
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(2)))
m.find_patterns()
ll, H, re = m.resolve_all()
print("E1", m.timings()["estep_forward_ms"], "ms", ll)
m.find_patterns()
ll, H, re = m.resolve_all()
print("E2", m.timings()["estep_forward_ms"], "ms", ll)
