"""Full-size (BASELINE configs[1]: 1000 x 500) digest of the CPU restatement's
EM run, so GPU tests can check full-size parity without re-running the ~90 s
oracle.  Records per-iteration scalars (LL as float.hex, patterns, R_E, R_M)
and SHA-256 digests of the M0 pattern table and of the accepted resolutions.

    python tests/golden/make_cfg2_digest.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def digest_patterns(pt):
    h = hashlib.sha256()
    for k in ("start", "len", "freq", "prefix", "tp", "succ"):
        h.update(np.ascontiguousarray(pt[k]).tobytes())
    return h.hexdigest()


def digest_array(a):
    return hashlib.sha256(np.ascontiguousarray(a, np.int32).tobytes()).hexdigest()


if __name__ == "__main__":
    import oracle
    from hmc_amd import synth

    p = synth.config_panel(2)
    o = oracle.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    m0 = digest_patterns(o.patterns(maxlen=1))
    o2 = oracle.Oracle(p.alleles, p.types, sample_size=10, max_iter=50)
    r = o2.run()
    out = dict(config=2, N=p.N, L=p.L, m0_patterns_sha256=m0, iterations=int(r["iterations"]),
               ll_hex=[float(x).hex() for x in r["ll"]], n_patterns=[int(x) for x in r["n_patterns"]],
               R_E=[int(x) for x in r["R_E"]], R_M=[int(x) for x in r["R_M"]],
               resolutions_sha256=digest_array(r["resolutions"]),
               oracle_seconds=dict(m0=r["t_m0"], e=[float(x) for x in r["t_e"]], m=[float(x) for x in r["t_m"]]))
    with open(os.path.join(HERE, "cfg2_digest.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
