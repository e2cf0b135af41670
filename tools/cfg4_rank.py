"""Rank r's real E1 of the 8-GPU cfg 4 run, on one GPU: the global M0 mined
over all 50 000 individuals (the model every rank holds after the sharded
M0), then the E-step over rank r's balanced shard only (hmc_set_shard) —
exactly the E1 work of rank r in `bench.py --gpus 8 --config 4`.  Prints the
E-step's device ms (structure / values / recompute), its windows, and a
repeat's bit-identity.

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
ref = None
for rep in range(2):
    t0 = time.perf_counter()
    ll, H, re = m.resolve_all()
    wall = time.perf_counter() - t0
    s = m.estep_split_stats()
    t = m.timings()
    w = m.estep_windows()
    print(f"E1 run {rep}: wall {wall:.2f} s; device: structure {s['structure_ms']:.0f} ms ({s['structure_passes']} passes), "
          f"values {s['values_ms']:.0f} ms ({s['value_passes']}), traceback {t['estep_traceback_ms']:.0f} ms, "
          f"fallback {s['fallback_ms']:.0f} ms ({s['n_fallback']}); windows {w['windows']} of {w['window_loci']} loci in "
          f"{w['groups']} group(s), recompute {w['recompute_ms']:.0f} ms; LL {ll!r} H {H} R_E {re}", flush=True)
    if ref is None:
        ref = (float(ll).hex(), H, re)
    else:
        print(f"repeat identical: {(float(ll).hex(), H, re) == ref}", flush=True)
m.close()
