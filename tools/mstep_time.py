"""M-step (find_patterns on samples) timing at cfg2."""
import sys, os
if "--diag" in sys.argv:
    os.environ["HMC_AMD_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hmc_amd", "libhmc_amd_diag.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd
from hmc_amd import synth
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(2)))
P, rm = m.find_patterns()
print("M0", m.timings()["mstep_ms"], "ms", P, rm)
for it in range(3):
    m.resolve_all()
    P, rm = m.find_patterns()
    print(f"M{it+1}", f"{m.timings()['mstep_ms']:.2f} ms", P, rm)
