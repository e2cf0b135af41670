"""Full-size digests of the CPU restatement (oracle/) for BASELINE configs 3 and 5
(and 2), generated once in the build container so that `-m gpu` tests can check
the GPU at full size without re-running hours of CPU work on the GPU box.

The chain is the one bench.py times: M0 on the genotypes, then E1, M1, E2, M2,
E3 (HaploModel.cpp:117-155 without the convergence test).  Recorded:
  per M-step: pattern count, R_M and the SHA-256 of the table in id order
              (start, len, freq, prefix, tp, successors — as in make_cfg2_digest.py);
  per E-step: LL (float.hex), R_E, samples H, total weight (hex), SHA-256 of the
              per-individual totals (f64), candidate counts (i32) and selected
              pairs ([N][2][L] i32), plus the totals of every (N/200)-th individual.
The oracle runs multi-threaded (oracle.set_threads: start loci / individuals in
parallel, every result assembled in the reference's order; the cfg2 digest is
reproduced bit for bit that way).

    python tests/golden/make_full_digest.py 5 [threads]
    python tests/golden/make_full_digest.py 3 [threads]
"""
import hashlib
import json
import os
import sys
import time

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


def sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a, dt).tobytes()).hexdigest()


def subset(N):
    return list(range(0, N, max(1, N // 200)))


def estep_record(ll, H, re, tw, totals, ncand, res):
    sub = subset(len(totals))
    return dict(ll_hex=float(ll).hex(), R_E=int(re), H=int(H), total_weight_hex=float(tw).hex(),
                totals_sha256=sha(totals, np.float64), ncand_sha256=sha(ncand, np.int32),
                resolutions_sha256=sha(res, np.int32),
                subset=sub, subset_totals_hex=[float(totals[i]).hex() for i in sub])


def main():
    import oracle
    from hmc_amd import synth

    cfg = int(sys.argv[1])
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    oracle.set_threads(threads)
    p = synth.config_panel(cfg)
    c = synth.CONFIGS[cfg]
    out = dict(config=cfg, N=p.N, L=p.L, A=c["A"], seed=cfg, sample_size=10, min_freq_abs=1.5,
               pattern_len=[1, 30], threads=threads, m=[], e=[], seconds={})
    o = oracle.Oracle(p.alleles, p.types, sample_size=10)
    path = os.path.join(HERE, f"cfg{cfg}_chain_digest.json")

    def log(msg):
        print(f"[cfg{cfg} {time.strftime('%H:%M:%S')}] {msg}", flush=True)

    def mstep(k):
        o.reset_counters()
        t = time.time()
        P = o.find_patterns()
        out["seconds"][f"m{k}"] = time.time() - t
        _, rm = o.counters()
        pt = o.patterns(maxlen=1)
        out["m"].append(dict(P=int(P), R_M=int(rm), table_sha256=digest_patterns(pt)))
        log(f"M{k}: {P} patterns, R_M {rm}, {out['seconds'][f'm{k}']:.0f} s")
        del pt

    def estep(k):
        o.reset_counters()
        t = time.time()
        ll = o.resolve_all()
        out["seconds"][f"e{k}"] = time.time() - t
        re, _ = o.counters()
        nc, gp = o.estep_summary()
        H = oracle.lib().ora_sample_count(o.h)
        tw = oracle.lib().ora_total_weight(o.h)
        res = o.resolutions()
        out["e"].append(estep_record(ll, H, re, tw, gp, nc, res))
        log(f"E{k}: LL {ll}, R_E {re}, {out['seconds'][f'e{k}']:.0f} s")

    mstep(0)
    for k in (1, 2, 3):
        estep(k)
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        if k < 3:
            mstep(k)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    log("done")


if __name__ == "__main__":
    main()
