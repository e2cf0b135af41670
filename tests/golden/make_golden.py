"""Regenerate the regression fixtures in tests/golden/ from the CPU
restatement (oracle/).  These pin the restatement against its own history; they
are NOT reference outputs (the reference is unbuildable here — DESIGN.md §Oracle).

    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle  # noqa: E402
from hmc_amd import synth  # noqa: E402

CASES = {
    "cfg1": dict(N=10, L=20, A=2, missing=0.0, seed=1, S=10),
    "miss_a3": dict(N=30, L=30, A=3, missing=0.05, seed=11, S=10),
    "snp_miss": dict(N=40, L=40, A=2, missing=0.02, seed=12, S=10),
    "s3": dict(N=25, L=25, A=2, missing=0.0, seed=13, S=3),
}


def compute(c):
    p = synth.founder_mosaic(c["N"], c["L"], A=c["A"], missing=c["missing"], seed=c["seed"])
    o = oracle.Oracle(p.alleles, p.types, sample_size=c["S"])
    o.find_patterns()
    pt = o.patterns(maxlen=min(30, c["L"]))
    ll = o.resolve_all()
    nc, gp = o.estep_summary()
    al, w, tw = o.samples()
    o2 = oracle.Oracle(p.alleles, p.types, sample_size=c["S"], max_iter=20)
    r = o2.run()
    return dict(alleles=p.alleles, m0_start=pt["start"], m0_len=pt["len"], m0_freq=pt["freq"],
                m0_prefix=pt["prefix"], m0_tp=pt["tp"], m0_succ=pt["succ"], m0_alleles=pt["alleles"],
                e1_ll=np.array([ll]), e1_ncand=nc, e1_total=gp, e1_samples=al, e1_w=w, e1_tw=np.array([tw]),
                em_iterations=np.array([r["iterations"]]), em_ll=r["ll"], em_resolutions=r["resolutions"])


if __name__ == "__main__":
    for name, c in CASES.items():
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **compute(c))
        print("wrote", name)
