"""The exact M-step restatement against an independent one (CPU only).

oracle/hmc_oracle.cpp keeps two walks of HaploBuilder::estimateFrequency
(HaploBuilder.cpp:334-450): `xwalk`, which sums in the device walk's order
(gathers in add order, 64 strided partials, 2^-44 fixed-point totals) so the
GPU tables can be checked bit for bit, and `rwalk`, which follows the
reference's own grouping in double — list 0's terms, then list 1's, then
list 2's, predecessors in creation order (the stand-in for std::map's pointer
order), one running sum per child, frequencies added in visiting order.  The
two must give the same table (patterns, order, successors) and frequencies
within 1e-9 relative, including a panel whose patterns sit at the min_freq
threshold (1.25e-3) — so the bit-exact checker does not hide an error that
only the reference's arithmetic would expose.
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from hmc_amd import synth  # noqa: E402

PANELS = {
    "cfg1": (dict(N=10, L=20, A=2, seed=1), 1.5),
    "n60": (dict(N=60, L=40, A=2, seed=2), 1.5),
    "a8": (dict(N=60, L=50, A=8, missing=0.01, seed=6), 1.5),
    "a3miss5": (dict(N=80, L=60, A=3, missing=0.05, seed=5), 1.5),
    # many founders, frequent switches, min_freq_abs 0.2: the smallest
    # frequencies at the threshold 0.2 / 2N = 1.25e-3
    "rare": (dict(N=80, L=50, A=2, K=40, rho=0.05, seed=12), 0.2),
}


@pytest.mark.parametrize("name", sorted(PANELS))
def test_exact_device_order_equals_reference_order(name):
    import oracle
    kw, mfa = PANELS[name]
    p = synth.founder_mosaic(**kw)
    out = []
    for mode in ("device", "reference"):
        o = oracle.Oracle(p.alleles, p.types, sample_size=10, min_freq_abs=mfa)
        o.set_exact_order(mode)
        o.find_patterns()
        o.resolve_all()
        o.estimate_patterns()
        out.append(o.patterns())
    a, b = out
    for k in ("start", "len", "alleles", "succ"):
        assert np.array_equal(a[k], b[k]), k
    for k in ("freq", "prefix", "tp"):
        rel = np.abs(a[k] - b[k]) / np.maximum(np.abs(b[k]), 1e-300)
        assert rel.max() <= 1e-9, (k, rel.max())
