"""GPU parity of the windowed E-step (ctx_window.cpp, hmc_set_estep_windows):
the loci cut into windows, each window's last frontier saved as the next one's
checkpoint, the records of one window at a time, the traces of two windows
with the older one's live entries collected into survivor nodes.  Forced on
small panels with tiny windows (down to one locus), it must equal the CPU
restatement bit for bit — the same bar as the classic passes (tolerance 0 for
every integer and double)."""
import os
import types

import numpy as np
import pytest

import hmc_amd
from hmc_amd import synth

from test_gpu_parity import PANELS, assert_estep_equal, gpu_model, last_symbols, panel

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,wl", [(n, w) for n in sorted(PANELS) for w in (1, 7)] + [("n300", 64), ("a4", 33)])
def test_windowed_estep_on_reference_model(oracle_mod, name, wl):
    """E-step on the restatement's M0 table in windows of `wl` loci ==
    HaploModel::resolveAll: LL, R_E, totals, candidates, priors, posteriors,
    samples, weights, resolutions."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p)
    m.set_estep_windows("always", wl)
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    w = m.estep_windows()
    assert w["windows"] == -(-(p.L) // wl), w
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.parametrize("name,wl", [("cfg1", 3), ("n60", 5), ("miss2", 11), ("a3miss5", 2), ("a8", 4)])
def test_windowed_full_em(oracle_mod, name, wl):
    """HaploModel::run with every E-step in windows: iteration count,
    per-iteration LL / R_E / R_M / pattern counts, HaploComp and the accepted
    pair of every individual."""
    p = panel(name)
    m = gpu_model(p, max_iteration=30)
    m.set_estep_windows("always", wl)
    res = m.run()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=30)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert [x["r_e"] for x in m.log] == r["R_E"].tolist()
    for k in range(r["iterations"] - 1):
        assert m.log[k]["r_m"] == r["R_M"][k + 1]
    assert np.array_equal(res, r["resolutions"])
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])


@pytest.mark.parametrize("S,wl", [(1, 3), (3, 1), (17, 4), (40, 6)])
def test_windowed_sample_sizes(oracle_mod, S, wl):
    """Windows with lists of one link, of an odd width, past 16 (one link per
    lane) and past 32 (a list over two lanes' slots)."""
    p = panel("a3miss5")
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    m = gpu_model(p, S)
    m.set_estep_windows("always", wl)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.parametrize("model,order", [("MC", 2), ("MA", 1)])
def test_windowed_head_len_models(oracle_mod, model, order):
    """Models whose head patterns span several loci (MC order 2: head_len 3):
    the first window starts at the head pairs, the traceback ends in them."""
    p = panel("n60")
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=6)
    o.set_model(model, order)
    r = o.run()
    m = gpu_model(p, max_iteration=6, model=model, mc_order=order)
    m.set_estep_windows("always", 4)
    res = m.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])


def test_windowed_underflow_hands_over(oracle_mod):
    """Individuals whose forward likelihoods underflow leave the windows and
    are re-run by the classic passes with extend()'s forward test
    (HaploBuilder.cpp:237): same LL (-inf) and resolutions as the reference."""
    rng = np.random.default_rng(5)
    a = (rng.integers(0, 2, (6, 2, 2500)) + ord("1")).astype(np.int32)
    o = oracle_mod.Oracle(a, "S" * 2500, sample_size=4, max_iter=3)
    r = o.run()
    m = hmc_amd.HaploModel()
    m.set_estep_windows("always", 300)
    m.sample_size = 4
    m.max_iteration = 3
    res = m.run(hmc_amd.GenoData(a, "S" * 2500))
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])
    assert m.estep_split_stats()["n_fallback"] > 0


def test_windowed_equals_classic_cfg2():
    """cfg 2 (1 000 x 500): E1 on the genotype-mined M0 and E2 in automatic
    windows of the store budgets and in windows of 50 loci equal the classic
    passes bit for bit (LL, R_E, samples, weights)."""
    p = synth.config_panel(2)
    runs = []
    for mode, wl in (("never", 0), ("always", 50), ("always", 0)):
        m = gpu_model(p)
        m.set_estep_windows(mode, wl)
        m.find_patterns()
        out = []
        for _ in range(2):
            ll, H, re = m.resolve_all()
            al, w, tw = m.samples(H)
            out.append((float(ll).hex(), H, re, al.tobytes(), w.tobytes(), float(tw).hex()))
            if mode == "always":
                assert m.estep_windows()["windows"] >= 1
            m.find_patterns()
        runs.append(out)
        m.close()
    assert runs[0] == runs[1] == runs[2]


def _homozygous_lead_panel(N=200, lead=80, L=160, seed=11):
    """A founder mosaic behind `lead` loci where everyone is homozygous: the
    window probe (the first >= 64 loci) sees one-state frontiers, so the plan
    under-sizes the trace ring for the later windows."""
    q = synth.founder_mosaic(N, L, A=2, seed=seed)
    a = np.concatenate([np.full((N, 2, lead), ord("1"), np.int32), q.alleles], axis=2)
    return synth.Panel(alleles=a, types="S" * (lead + L))


def test_windowed_fixed_length_trace_overflow_shrinks_group(oracle_mod):
    """The round-5 hang (gpurun_out/r5f: window_ab.py CFG=3 on `always:1000`)
    pinned: a FIXED window length whose two windows of traces exceed the trace
    store.  Before ecc6276 the plan ignored win_scale for a fixed length, so
    every ESTEP_RESTART re-made the same plan and the E-step never ended; now
    the plan takes smaller groups until the traces fit (ctx_window.cpp plan
    loop, `fits`), bounded by win_scale >= 1e-3.  Here a 2 MB trace budget
    and a probe that sees only homozygous loci force several restarts; the
    E-step must end in >= 2 groups, bit-exact against the restatement, and
    the next E-step (a new model, the shrunken scale kept) equal the classic
    passes'."""
    p = _homozygous_lead_panel()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p)
    m.set_estep_windows("always", 8)
    m.set_store_budgets(trace_bytes=2 << 20, record_bytes=64 << 20)
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    w = m.estep_windows()
    print(f"windows {w}", flush=True)
    assert w["restarts"] >= 1 and w["window_scale"] < 1.0, w
    assert w["groups"] >= 2 and w["window_loci"] == 8, w
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)
    # E2 on the GPU's own M1, windows at the scale learnt above vs the classic passes
    c = gpu_model(p)
    c.set_estep_windows("never")
    c.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    c.resolve_all()
    out = []
    for x in (m, c):
        x.find_patterns()
        ll, H2, re2 = x.resolve_all()
        al, wt, tw = x.samples(H2)
        out.append((float(ll).hex(), H2, re2, al.tobytes(), wt.tobytes(), float(tw).hex()))
    assert out[0] == out[1]
    assert m.estep_windows()["groups"] >= 2


def _heartbeat(path, stop):
    """A line every 30 s under gpurun_out/ while a multi-minute test runs, so
    that a runner watching its output directory sees progress."""
    import threading
    import time

    def beat():
        t0 = time.time()
        while not stop.wait(30.0):
            try:
                os.makedirs(os.path.dirname(path), exist_ok=True)
                with open(path, "a") as f:
                    f.write(f"cfg 4 rank-0 test alive {time.time() - t0:.0f} s\n")
            except OSError:
                pass

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    return th


@pytest.mark.slow
@pytest.mark.timeout(900)
def test_cfg4_rank0_real_shard_windowed_e1():
    """Rank 0's real E1 of the 8-GPU cfg 4 run on one GPU (~3 min): the global
    M0 over all 50 000 individuals (what every rank holds after the sharded
    M0), then the E-step over rank 0's balanced shard (hmc_set_shard).  It
    runs in automatic windows (one group); the samples phase the genotypes,
    weights sum to 1, priors are sorted; a second E1 repeats LL, H, R_E,
    samples and weights bit for bit."""
    import threading

    from hmc_amd.model import balanced_shard
    from test_gpu_parity import _estep_properties

    stop = threading.Event()
    _heartbeat(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                            "heartbeat_cfg4_test"), stop)
    try:
        p = synth.config_panel(4)
        m = gpu_model(p)
        m.find_patterns()
        i0, i1 = balanced_shard(p.alleles, 0, 8)
        m.set_shard(i0, i1)
        sub = types.SimpleNamespace(N=i1 - i0, alleles=p.alleles[i0:i1])
        del p
        out = []
        for rep in range(2):
            ll, H, re = m.resolve_all()
            w = m.estep_windows()
            assert w["windows"] >= 2 and w["groups"] == 1, w
            if rep == 0:
                _estep_properties(m, sub, ll, H)
            al, wt, tw = m.samples(H)
            out.append((float(ll).hex(), H, re, hash(al.tobytes()), wt.tobytes(), float(tw).hex()))
            del al
        assert out[0] == out[1]
        m.close()
    finally:
        stop.set()
