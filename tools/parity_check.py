"""Quick GPU-vs-oracle parity probe (development aid; the real gate is tests/)."""
import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import numpy as np
import hmc_amd
from hmc_amd import synth
import oracle

def last_symbols(pt):
    return np.array([pt["alleles"][i, pt["len"][i] - 1] for i in range(len(pt["len"]))], np.int32)

def check(N, L, A=2, miss=0.0, seed=1, S=10):
    p = synth.founder_mosaic(N, L, A=A, seed=seed, missing=miss)
    o = oracle.Oracle(p.alleles, p.types, sample_size=S)
    t = time.time(); o.find_patterns(); to_m = time.time() - t
    opt = o.patterns()
    m = hmc_amd.HaploModel()
    m.sample_size = S
    m.load(hmc_amd.GenoData.from_panel(p))
    # 1) E-step on the oracle's pattern table
    m.set_patterns(opt["start"], opt["len"], opt["freq"], opt["tp"], opt["succ"], last_symbols(opt))
    t = time.time(); ll_g, H_g, re_g = m.resolve_all(); tg = time.time() - t
    t = time.time(); ll_o = o.resolve_all(); to_e = time.time() - t
    re_o, _ = o.counters()
    nc_o, gp_o = o.estep_summary()
    er = m.estep_results()
    al_o, w_o, tw_o = o.samples()
    al_g, w_g, tw_g = m.samples(H_g)
    res_ok = np.array_equal(m.resolutions(), o.resolutions())
    print(f"[E] N={N} L={L} A={A} miss={miss}: ll {ll_g!r} vs {ll_o!r} eq={ll_g == ll_o}; H {H_g} vs {len(w_o)}; "
          f"RE {re_g} vs {re_o}; ncand eq={np.array_equal(er['ncand'], nc_o)} total eq={np.array_equal(er['total'], gp_o)} "
          f"samples eq={al_g.shape == al_o.shape and np.array_equal(al_g, al_o)} w eq={np.array_equal(w_g, w_o)} "
          f"tw eq={tw_g == tw_o} res eq={res_ok}; t_gpu={tg:.3f}s t_ora={to_e:.3f}s")
    # 2) M-step on genotypes (M0), fresh context
    m2 = hmc_amd.HaploModel()
    m2.sample_size = S
    m2.load(hmc_amd.GenoData.from_panel(p))
    t = time.time(); P, rm = m2.find_patterns(); tg = time.time() - t
    gpt = m2.patterns()
    same = P == len(opt["start"])
    msg = f"[M0] P {P} vs {len(opt['start'])}"
    if same:
        for k in ["start", "len", "freq", "prefix", "tp", "succ", "alleles"]:
            eq = np.array_equal(gpt[k], opt[k])
            msg += f" {k}={eq}"
    print(msg + f" t_gpu={tg:.3f}s t_ora={to_m:.3f}s")
    # 3) M1 on samples: GPU E-step (own model) then mine
    ll2, H2, re2 = m2.resolve_all()
    o.reset_counters()
    t = time.time(); P1, rm1 = m2.find_patterns(); tg = time.time() - t
    t = time.time(); o.find_patterns(); to_m1 = time.time() - t
    _, rm_o = o.counters()
    opt1 = o.patterns(); gpt1 = m2.patterns()
    msg = f"[M1] ll2 eq={ll2 == ll_o} P {P1} vs {len(opt1['start'])} RM {rm1} vs {rm_o}"
    if P1 == len(opt1["start"]):
        for k in ["start", "len", "freq", "prefix", "tp", "succ", "alleles"]:
            msg += f" {k}={np.array_equal(gpt1[k], opt1[k])}"
    print(msg + f" t_gpu={tg:.3f}s t_ora={to_m1:.3f}s", flush=True)

if __name__ == "__main__":
    check(10, 20)
    check(60, 40)
    check(100, 100, A=4)
    check(100, 100, miss=0.02)
    check(300, 200)
