"""Wall time of each step of a small GPU parity test (diagnostic): the golden
cfg1 case (10 x 20) as tests/test_gpu_parity.py::test_against_golden_fixtures
runs it — two contexts, M0, E1, samples, a full run — three times in one
process, with the contexts' destruction timed apart (close vs garbage
collection), so a fixed per-test cost shows where it is spent."""
import gc
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

p = synth.founder_mosaic(10, 20, A=2, seed=1)
for rep in range(3):
    t = [("start", time.perf_counter())]

    def mark(name):
        t.append((name, time.perf_counter()))

    m = hmc_amd.HaploModel()
    m.sample_size = 10
    mark("create")
    m.load(hmc_amd.GenoData.from_panel(p))
    mark("load")
    m.find_patterns()
    mark("M0")
    pt = m.patterns(maxlen=20)
    mark("patterns")
    ll, H, _ = m.resolve_all()
    mark("E1")
    m.estep_results()
    m.samples(H)
    mark("samples")
    m2 = hmc_amd.HaploModel()
    m2.sample_size = 10
    m2.max_iteration = 20
    m2.load(hmc_amd.GenoData.from_panel(p))
    mark("create2")
    m2.run()
    mark(f"run({m2.iterations})")
    m.close()
    mark("close")
    del m2
    gc.collect()
    mark("gc")
    print(f"rep {rep}: " + " ".join(f"{t[i + 1][0]} {1e3 * (t[i + 1][1] - t[i][1]):.1f}" for i in range(len(t) - 1))
          + " ms", flush=True)
