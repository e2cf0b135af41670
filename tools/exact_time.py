"""Exact M-step (--exact-estimate) timing on a BASELINE config (env CFG,
default 2): M0, E1, then the exact M-step (rounds, candidates, trie-walk ms,
total ms) next to the sampling M-step on the same E1 samples, and E2 after it.
Env IPW: exact-walk items per wavefront (1 or 4)."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

def _beat():  # a line a minute: long exact M-steps print nothing else
    t0 = time.time()
    while True:
        time.sleep(60)
        print(f"  ... {time.time() - t0:.0f} s", flush=True)


threading.Thread(target=_beat, daemon=True).start()
p = synth.config_panel(int(os.environ.get("CFG", "2")))
m = hmc_amd.HaploModel()
m.set_exact_walk(int(os.environ.get("IPW", "1")))
m.load(hmc_amd.GenoData.from_panel(p))
P0, _ = m.find_patterns()
ll1, H, re = m.resolve_all()
P1s, rm = m.find_patterns()  # sampling M1 (reference default)
ts = m.timings()["mstep_ms"]
print(f"M0 {P0} patterns; E1 LL {ll1:.6f}; sampling M1: {P1s} patterns, {ts:.1f} ms", flush=True)
m.clear_samples()
m.find_patterns()
m.resolve_all()
m.exact_estimate = True
t0 = time.perf_counter()
P1, _ = m.find_patterns()
dt = time.perf_counter() - t0
st = m.exact_stats()
print(f"exact M1: {P1} patterns, {st['rounds']} rounds, {st['candidates']} candidates, walk {st['walk_ms']:.1f} ms, "
      f"device {m.timings()['mstep_ms']:.1f} ms, wall {dt * 1e3:.1f} ms; ratio to sampling {dt * 1e3 / ts:.1f}x; {st}",
      flush=True)
ll2, H, re = m.resolve_all()
print(f"E2 after exact M1: LL {ll2:.6f}, R_E {re}, {m.timings()['estep_forward_ms']:.1f} ms", flush=True)
