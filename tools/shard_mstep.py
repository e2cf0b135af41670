"""Per-rank EM step of a sharded run, projected on one GPU: rank 0 of W runs
alone with a stub collective that multiplies every all-reduced vector by W
(the other ranks' shards are statistically alike, so candidate sums, LL and
total weight come out near the W-rank values and the candidate tree is the
size the real run mines).  Rank 0 then does its real per-rank work: the
E-step over its balanced shard of individuals and every mining level's scan
over its own samples (its items only), with one all-reduce per level
(hmc_set_reduction "allreduce"; the ordered reduction adds W add chains and
W broadcasts per level, not modelled here).  Times are rank 0's device times
of each step of the converged chain from M0.  Not a measurement of an
N-GPU run: a projection of one rank's share of it.
usage: python tools/shard_mstep.py CFG "1,2,4,8"
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 3
worlds = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,2,4,8").split(",")]
p = synth.config_panel(cfg)
g = hmc_amd.GenoData.from_panel(p)
DBL_MAX = sys.float_info.max

for W in worlds:
    def stub(arr, W=W):
        arr *= W
    m = hmc_amd.HaploModel(rank=0, world=W, host_allreduce=stub) if W > 1 else hmc_amd.HaploModel()
    m.set_reduction("allreduce")
    m.load(g)
    t0 = time.perf_counter()
    P0, _ = m.find_patterns()
    t_m0 = time.perf_counter() - t0
    m.model_save()
    print(f"W={W} rank 0 individuals [{m.i0},{m.i1}): M0 {P0} patterns, {t_m0 * 1e3:.0f} ms wall, "
          f"{m.timings()['mstep_ms']:.0f} ms device", flush=True)
    for rep in range(2):  # the second chain runs warm (stores allocated)
        m.em_rewind()
        old, it, tot = -DBL_MAX, 0, 0.0
        while True:
            it += 1
            t0 = time.perf_counter()
            log, old, go = m.em_iteration(it, old, always_mstep=False)
            wall = time.perf_counter() - t0
            tot += wall
            t = m.timings()
            s = m.estep_split_stats()
            print(f"  chain {rep} iteration {it}: E {t['estep_forward_ms'] + t['estep_traceback_ms']:.0f} ms "
                  f"(structure {s['structure_ms']:.0f}, values {s['values_ms']:.0f}), "
                  f"M {t['mstep_ms'] if go else 0:.0f} ms ({log['n_patterns']} patterns), wall {wall * 1e3:.0f} ms"
                  + ("" if go else "  [stop]"), flush=True)
            hp = m.host_phases()
            print("    host ms: " + ", ".join(f"{k} {v:.0f}" for k, v in hp.items())
                  + f"; E-step wall minus device passes {hp['estep'] - t['estep_forward_ms'] - t['estep_traceback_ms']:.0f}",
                  flush=True)
            if not go or it >= 10:
                break
        print(f"  chain {rep}: {it} iterations, {tot / it * 1e3:.0f} ms per iteration "
              f"-> {p.alleles.shape[0] * p.alleles.shape[2] / (tot / it):.3g} individual-loci/s if every rank "
              f"matched rank 0", flush=True)
    m.close()
