"""Stage timing of one EM step at a BASELINE config (diagnostic): panel, load,
M0, E1, M1, with a line printed after each stage.  usage: cfg_stage_times.py CFG [N_FIRST] [ESTEP_MODE]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("WITH_TORCH"):
    import torch  # noqa: F401
    torch.cuda.set_device(0)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
mode = int(sys.argv[3]) if len(sys.argv) > 3 else 0
t0 = time.time()


def stamp(what):
    print(f"{time.time() - t0:8.2f} s  {what}", flush=True)


p = synth.config_panel(cfg)
if len(sys.argv) > 2 and int(sys.argv[2]) > 0:  # first n individuals only
    p = synth.Panel(p.alleles[: int(sys.argv[2])].copy(), p.types)
stamp(f"panel {p.N}x{p.L}")
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
m.set_estep_mode(mode)
stamp("load")
P, rm = m.find_patterns()
stamp(f"M0 {P} patterns")
ll, H, re = m.resolve_all()
stamp(f"E1 ll {ll:.3f} H {H} R_E {re} {m.estep_split_stats()}")
er = m.estep_results()
stamp("estep_results")
res = m.resolutions()
stamp("resolutions")
P, rm = m.find_patterns()
stamp(f"M1 {P} patterns")
pt = m.patterns()
stamp("patterns()")
