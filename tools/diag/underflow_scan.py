"""Find small i.i.d. panels whose E-step underflows for some individuals
(forward likelihood 0 before the last locus) while every individual keeps a
positive genotype probability (diagnostic: picks the test panel for the
exact M-step's pruned re-run)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402

for L in range(900, 2600, 100):
    for seed in range(4):
        rng = np.random.default_rng(seed)
        a = (rng.integers(0, 2, (6, 2, L)) + ord("1")).astype(np.int32)
        m = hmc_amd.HaploModel()
        m.sample_size = 4
        m.load(hmc_amd.GenoData(a, "S" * L))
        m.find_patterns()
        ll, H, re = m.resolve_all()
        er = m.estep_results()
        nf = m.estep_split_stats()["n_fallback"]
        print(f"L {L} seed {seed}: n_fallback {nf} min total {er['total'].min():.3e} ll {ll}", flush=True)
        m.close()
