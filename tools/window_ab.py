"""E1 on a config's M0 in classic groups and in windows (hmc_set_estep_windows),
one context: M0 once, then each setting twice (the second run is reported
warm).  Prints device ms per pass, windows and groups, and that every run
gives the same LL / H / R_E.  WINDOWS = "never:0,always:0,always:500,...".

    CFG=3 python tools/window_ab.py
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(os.environ.get("CFG", "3"))
sets = [(s.split(":")[0], int(s.split(":")[1])) for s in os.environ.get("WINDOWS", "never:0,always:0,always:1000,always:500").split(",")]
p = synth.config_panel(cfg)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
t0 = time.perf_counter()
P0, _ = m.find_patterns()
print(f"cfg {cfg}: M0 {P0} patterns, {time.perf_counter() - t0:.1f} s", flush=True)
ref = None
for mode, wl in sets:
    m.set_estep_windows(mode, wl)
    for rep in range(2):
        t0 = time.perf_counter()
        ll, H, re = m.resolve_all()
        wall = time.perf_counter() - t0
        s = m.estep_split_stats()
        w = m.estep_windows()
        print(f"{mode}:{wl} run {rep}: wall {wall * 1e3:.0f} ms; structure {s['structure_ms']:.0f} ms ({s['structure_passes']}), "
              f"values {s['values_ms']:.0f} ms ({s['value_passes']}; collection {w['collection_ms']:.0f}), "
              f"traceback {m.timings()['estep_traceback_ms']:.0f} ms; windows {w['windows']} of {w['window_loci']} loci, "
              f"{w['groups']} group(s); LL {ll!r} R_E {re}", flush=True)
        key = (float(ll).hex(), H, re)
        ref = ref or key
        assert key == ref, (key, ref)
print("all settings identical", flush=True)
m.close()
