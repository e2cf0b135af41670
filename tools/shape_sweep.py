"""E-step launch-shape sweep on a BASELINE config (env CFG, default 3): M0, E1,
M1 with the default shape, then E2 (the M1 model) repeated under each shape
"W:I" (waves per individual : individuals per CU's LDS) — structure and value
pass ms, and the LL / R_E, which must not depend on the shape.
usage: CFG=3 python tools/shape_sweep.py 3:4 2:8 ..."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

p = synth.config_panel(int(os.environ.get("CFG", "3")))
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
m.find_patterns()
m.resolve_all()
m.find_patterns()
ref = None
for shape in sys.argv[1:] or ["3:4"]:
    nw, ipc = (int(x) for x in shape.split(":"))
    m.set_estep_shape(nw, ipc)
    for r in range(2):
        ll, H, re = m.resolve_all()
        s = m.estep_split_stats()
        key = (ll, H, re)
        ref = ref or key
        assert key == ref, (shape, key, ref)
        print(f"shape {shape} run {r}: structure {s['structure_ms']:.1f} ms ({s['structure_passes']} passes) "
              f"values {s['values_ms']:.1f} ms ({s['value_passes']} passes; re-run {s['n_order_rerun']} individuals "
              f"{s['order_ms']:.1f} ms) ll={ll!r}", flush=True)
