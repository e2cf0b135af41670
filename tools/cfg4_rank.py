"""Rank r's real E1 of the 8-GPU cfg 4 run, on one GPU: the global M0 mined
over all 50 000 individuals (the model every rank holds after the sharded
M0), then the E-step over rank r's balanced shard only (hmc_set_shard) —
exactly the E1 work of rank r in `bench.py --gpus 8 --config 4`.  Prints the
E-step's device ms (structure / values / trace collection), its windows, and
that a repeat is bit-identical.  SHAPES = "s_nw:s_ipc:v_nw:v_ipc,..." runs
the E-step once per pass-shape set (0 = automatic); WINDOW = loci per window
fixes the window length for every run (0 / unset: planned from the stores).

    python tools/cfg4_rank.py [RANK [WORLD [CFG]]]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402
from hmc_amd.model import balanced_shard  # noqa: E402

rank = int(sys.argv[1]) if len(sys.argv) > 1 else 0
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 4
shapes = [tuple(int(x) for x in s.split(":")) for s in os.environ.get("SHAPES", "0:0:0:0,0:0:0:0").split(",")]
t0 = time.perf_counter()
p = synth.config_panel(cfg)
print(f"cfg {cfg} panel {p.N} x {p.L} in {time.perf_counter() - t0:.1f} s", flush=True)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
t0 = time.perf_counter()
P0, rm0 = m.find_patterns()
print(f"global M0: {P0} patterns, R_M {rm0}, {time.perf_counter() - t0:.1f} s wall, {m.timings()['mstep_ms']:.0f} ms device; "
      f"{m.mine_stats()}", flush=True)
i0, i1 = balanced_shard(p.alleles, rank, world)
del p
m.set_shard(i0, i1)
print(f"rank {rank} of {world}: individuals [{i0}, {i1}) = {i1 - i0}", flush=True)
if os.environ.get("WINDOW"):  # fixed window length (loci), the same for every run of the sweep
    m.set_estep_windows("always", int(os.environ["WINDOW"]))
ref = None
for rep, sh in enumerate(shapes):
    m.set_pass_shapes(*sh)
    t0 = time.perf_counter()
    ll, H, re = m.resolve_all()
    wall = time.perf_counter() - t0
    s = m.estep_split_stats()
    t = m.timings()
    w = m.estep_windows()
    fr = m.estep_frontier()
    print(f"E1 run {rep} shapes {sh}: wall {wall:.2f} s; device: structure {s['structure_ms']:.0f} ms "
          f"({s['structure_passes']} passes), values {s['values_ms']:.0f} ms ({s['value_passes']}; trace collection "
          f"{w['collection_ms']:.0f} of it), traceback {t['estep_traceback_ms']:.0f} ms, fallback {s['fallback_ms']:.0f} ms "
          f"({s['n_fallback']}); windows {w['windows']} of {w['window_loci']} loci in {w['groups']} group(s), "
          f"{w['restarts']} restart(s), window scale {w['window_scale']:.3g}; "
          f"frontier {fr}; LL {ll!r} H {H} R_E {re}", flush=True)
    if ref is None:
        ref = (float(ll).hex(), H, re)
    else:
        print(f"identical to run 0: {(float(ll).hex(), H, re) == ref}", flush=True)
m.close()
