import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, hmc_amd
from hmc_amd import synth
p = synth.config_panel(2)
# args: shapes as "W:I" (waves per individual : individuals per CU)
for shape in sys.argv[1:] or ["2:4"]:
    nw, ipc = (int(x) for x in shape.split(":"))
    wpc = shape
    m = hmc_amd.HaploModel(); m.set_estep_shape(nw, ipc); m.load(hmc_amd.GenoData.from_panel(p)); m.find_patterns()
    out = []
    for it in range(3):
        ll, H, re = m.resolve_all(); t = m.timings()
        out.append(f"E{it+1} {t['estep_forward_ms']:.1f}ms ll={ll!r}")
        m.find_patterns()
    print(f"shape {wpc}: " + " | ".join(out), flush=True)
