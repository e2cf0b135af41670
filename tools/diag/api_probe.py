"""Wall time of each library call on a tiny panel (diagnostic): context
creation, load, M0, E1, M1, E2, close — twice in one process, so one-time
costs (code objects, first allocations) show apart from per-context ones."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

p = synth.founder_mosaic(10, 20, A=2, seed=1)
for rep in range(3):
    t = [time.perf_counter()]
    m = hmc_amd.HaploModel()
    t.append(time.perf_counter())
    m.load(hmc_amd.GenoData.from_panel(p))
    t.append(time.perf_counter())
    m.find_patterns()
    t.append(time.perf_counter())
    m.resolve_all()
    t.append(time.perf_counter())
    m.find_patterns()
    t.append(time.perf_counter())
    m.resolve_all()
    t.append(time.perf_counter())
    m.close()
    t.append(time.perf_counter())
    names = ["create", "load", "M0", "E1", "M1", "E2", "close"]
    print(f"rep {rep}: " + " ".join(f"{n} {1e3 * (t[i + 1] - t[i]):.1f}" for i, n in enumerate(names)) + " ms", flush=True)
