import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, hmc_amd
from hmc_amd import synth
for cfg, miss in [(2, 0.0), (2, 0.02)]:
    p = synth.config_panel(cfg, missing=miss)
    m = hmc_amd.HaploModel(); m.load(hmc_amd.GenoData.from_panel(p)); m.find_patterns()
    for it in range(3):
        t = time.time(); ll, H, re = m.resolve_all(); dt = time.time() - t
        f = m.frontier_max()
        print(f"cfg{cfg} miss={miss} E{it+1}: t={dt*1e3:.1f}ms RE={re} fmax pct50/90/99/max = {np.percentile(f,50):.0f}/{np.percentile(f,90):.0f}/{np.percentile(f,99):.0f}/{f.max()} tim={m.timings()}", flush=True)
        m.find_patterns()
