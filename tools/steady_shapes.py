"""Value-pass shapes on the steady E-step (E2 of a BASELINE config): M0, E1,
M1 with the automatic shapes, then per shape "vnw:vipc" the E-step on the M1
model twice (the model does not change, so neither may LL or R_E).

    python tools/steady_shapes.py CFG [s1nw:s1ipc:]vnw:vipc ...   (0 = automatic)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1])
m = hmc_amd.HaploModel()
m.set_value_layout(int(os.environ.get("LAYOUT", "2")))  # phase-B layout (hmc_set_value_layout)
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(cfg)))
m.find_patterns()
m.resolve_all()
m.find_patterns()
for sh in sys.argv[2:] or ["0:0"]:
    f = [int(x) for x in sh.split(":")]
    f = [0, 0] + f if len(f) == 2 else f
    m.set_pass_shapes(*f)
    for r in range(2):
        ll, H, re = m.resolve_all()
        s = m.estep_split_stats()
        print(f"shape {sh} run {r}: structure {s['structure_ms']:.1f} ms values {s['values_ms']:.1f} ms "
              f"({s['value_passes']} passes) ll={ll!r} re={re}", flush=True)
