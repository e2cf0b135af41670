"""E-step timing with repeats: E1, E2, E3 of cfg2, each run R times on the same
model (min / median of estep_forward ms).  usage: bench_e.py [W:I ...]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, hmc_amd
from hmc_amd import synth

R = int(os.environ.get("REPEATS", "5"))
p = synth.config_panel(2)
for shape in sys.argv[1:] or ["3:4"]:
    nw, ipc = (int(x) for x in shape.split(":"))
    m = hmc_amd.HaploModel()
    m.set_estep_shape(nw, ipc)
    m.load(hmc_amd.GenoData.from_panel(p))
    m.find_patterns()
    out, tot = [], 0.0
    for it in range(3):
        ts = []
        for r in range(R):
            m.resolve_all()
            ts.append(m.timings()["estep_forward_ms"])
        ts = np.array(ts)
        tot += np.median(ts)
        out.append(f"E{it+1} min {ts.min():.1f} med {np.median(ts):.1f}")
        m.find_patterns()
    print(f"shape {shape}: " + " | ".join(out) + f" | sum of medians {tot:.1f}", flush=True)
