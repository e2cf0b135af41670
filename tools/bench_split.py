"""E-step timing of the split (structure + value pass) vs the fused kernel on
cfg2: E1..E3 of one EM chain, each E-step repeated R times; checks that both
modes give the same LL / R_E.  usage: bench_split.py [W:I ...]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

R = int(os.environ.get("REPEATS", "3"))
p = synth.config_panel(int(os.environ.get("CFG", "2")))
for shape in sys.argv[1:] or ["3:4"]:
    nw, ipc = (int(x) for x in shape.split(":"))
    m = hmc_amd.HaploModel()
    m.set_estep_shape(nw, ipc)
    m.load(hmc_amd.GenoData.from_panel(p))
    m.find_patterns()
    for it in range(3):
        out = []
        ref = None
        for mode in (0, 1):
            m.set_estep_mode(mode)
            ts, extra = [], []
            for r in range(R):
                ll, H, re = m.resolve_all()
                ts.append(m.timings()["estep_forward_ms"])
                if mode == 0:
                    st = m.estep_split_stats()
                    extra.append((st["structure_ms"], st["values_ms"], st["fallback_ms"], st["n_fallback"]))
                key = (ll, H, re, m.resolutions().tobytes())
                if ref is None:
                    ref = key
                assert key == ref, ("mode mismatch", mode, it)
            ts = np.array(ts)
            tag = "split" if mode == 0 else "fused"
            s = f"{tag} min {ts.min():.2f} med {np.median(ts):.2f} ms"
            if extra:
                e = np.array(extra)
                s += f" (structure {np.median(e[:, 0]):.2f} values {np.median(e[:, 1]):.2f} fallback {np.median(e[:, 2]):.2f} n_fb {int(e[0, 3])})"
            out.append(s)
        print(f"shape {shape} E{it + 1}: " + " | ".join(out), flush=True)
        m.set_estep_mode(0)
        m.find_patterns()
