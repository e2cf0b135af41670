"""Find small panels whose E-step underflows for some individuals (a forward
likelihood reaches 0 before the last locus, so the structure pass re-runs
them in prune mode) while every individual keeps a positive genotype
probability, so the EM goes on to an M-step (diagnostic: picks the test panel
for the exact M-step's pruned re-run).  Two families: i.i.d. biallelic
panels, and founder mosaics with a few i.i.d. individuals appended."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402


def probe(tag, a, S=4):
    L = a.shape[2]
    m = hmc_amd.HaploModel()
    m.sample_size = S
    m.load(hmc_amd.GenoData(a, "S" * L))
    m.find_patterns()
    ll, H, re = m.resolve_all()
    er = m.estep_results()
    nf = m.estep_split_stats()["n_fallback"]
    print(f"{tag}: n_fallback {nf} min total {er['total'].min():.3e} ll {ll}", flush=True)
    m.close()


for L in range(920, 1100, 15):  # (900: no underflow; 1100 and longer: every individual's total is 0)
    for seed in range(4):
        rng = np.random.default_rng(seed)
        probe(f"iid L {L} seed {seed}", (rng.integers(0, 2, (6, 2, L)) + ord("1")).astype(np.int32))
for L in (1000, 1200):
    for k in (1, 2):
        p = synth.founder_mosaic(20, L, A=2, seed=7)
        rng = np.random.default_rng(L + k)
        extra = (rng.integers(0, 2, (k, 2, L)) + ord("1")).astype(np.int32)
        base = np.asarray(p.alleles).astype(np.int32)
        if base.max() < ord("1"):  # allele indices -> symbols
            base = base + ord("1")
        probe(f"mosaic20+{k} L {L}", np.concatenate([base, extra], axis=0))
