"""Per-individual value-pass time (kcycles) of the split E-step under several
launch shapes (waves per individual : individuals per CU), E1..E3 of cfg2:
how much co-residency on a CU slows one individual, and max/mean per shape.
usage: indiv_shapes.py [W:I ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

p = synth.config_panel(int(os.environ.get("CFG", "2")))
shapes = sys.argv[1:] or ["3:4", "3:2", "3:1"]
res = {}
for shape in shapes:
    nw, ipc = (int(x) for x in shape.split(":"))
    m = hmc_amd.HaploModel()
    m.set_estep_shape(nw, ipc)
    m.load(hmc_amd.GenoData.from_panel(p))
    m.find_patterns()
    for it in range(3):
        m.resolve_all()
        m.resolve_all()  # second run: ordered by the first run's cost
        c = m.estep_cost().astype(float)
        st = m.estep_split_stats()
        res[(shape, it)] = c
        print(f"{shape} E{it + 1}: values {st['values_ms']:.2f} ms structure {st['structure_ms']:.2f} ms; "
              f"kcycles mean {c.mean():.0f} max {c.max():.0f} max/mean {c.max() / c.mean():.2f} "
              f"p50/90/99 {' '.join(f'{x:.0f}' for x in np.percentile(c, [50, 90, 99]))}", flush=True)
        m.find_patterns()
base = shapes[0]
for shape in shapes[1:]:
    for it in range(3):
        r = res[(base, it)] / np.maximum(res[(shape, it)], 1)
        top = np.argsort(-res[(base, it)])[:20]
        print(f"E{it + 1}: time({base}) / time({shape}) per individual: median {np.median(r):.2f}, "
              f"20 slowest under {base}: {np.median(r[top]):.2f}")
