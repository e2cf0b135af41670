"""GPU parity: the gfx950 path (libhmc_amd.so, called through its C-ABI) against
the CPU restatement on the same seeded panels.  Bar: bit-exact for every
integer, allele and index output and for every double (likelihoods, weights,
frequencies, transition probabilities) — the kernels keep the reference's
operation order (tolerance 0 everywhere on one GPU)."""
import hashlib
import json
import os
import socket
import subprocess
import sys

import time

import numpy as np
import pytest

import hmc_amd
from hmc_amd import synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

PANELS = {
    "cfg1": dict(N=10, L=20, A=2, missing=0.0, seed=1),
    "n60": dict(N=60, L=40, A=2, missing=0.0, seed=2),
    "a4": dict(N=100, L=100, A=4, missing=0.0, seed=3),
    "miss2": dict(N=100, L=100, A=2, missing=0.02, seed=4),
    "a3miss5": dict(N=80, L=60, A=3, missing=0.05, seed=5),
    "a8": dict(N=60, L=50, A=8, missing=0.01, seed=6),
    "n300": dict(N=300, L=200, A=2, missing=0.0, seed=7),
}


def panel(name):
    c = PANELS[name]
    return synth.founder_mosaic(c["N"], c["L"], A=c["A"], missing=c["missing"], seed=c["seed"])


def gpu_model(p, S=10, **kw):
    m = hmc_amd.HaploModel()
    m.sample_size = S
    for k, v in kw.items():
        setattr(m, k, v)
    m.load(hmc_amd.GenoData.from_panel(p))
    return m


def last_symbols(pt):
    return np.array([pt["alleles"][i, pt["len"][i] - 1] for i in range(len(pt["len"]))], np.int32)


def assert_tables_equal(g, o):
    assert len(g["start"]) == len(o["start"])
    for k in ("start", "len", "freq", "prefix", "tp", "succ", "alleles"):
        assert np.array_equal(g[k], o[k]), k


def assert_estep_equal(m, o, ll_g, ll_o, H, re_g):
    re_o, _ = o.counters()
    assert ll_g == ll_o
    assert re_g == re_o
    nc, gp = o.estep_summary()
    er = m.estep_results()
    assert np.array_equal(er["ncand"], nc)
    assert np.array_equal(er["total"], gp)
    al_o, w_o, tw_o = o.samples()
    al_g, w_g, tw_g = m.samples(H)
    assert np.array_equal(al_g, al_o) and np.array_equal(w_g, w_o) and tw_g == tw_o
    for i in range(o.N):
        for c in range(nc[i]):
            _, pr, po = o.candidate(i, c)
            assert er["prior"][i, c] == pr and er["posterior"][i, c] == po
    assert np.array_equal(m.resolutions(), o.resolutions())


@pytest.mark.parametrize("name", sorted(PANELS))
@pytest.mark.parametrize("S", [10])
def test_estep_on_reference_model(oracle_mod, name, S):
    """E-step kernels fed the restatement's M0 table == HaploModel::resolveAll
    (structure pass + value pass)."""
    _estep_on_reference_model(oracle_mod, name, S, 0)


@pytest.mark.variants
def test_variant_fused_estep(oracle_mod):
    """The fused single-pass E-step kernel (hmc_set_estep_mode(1), variants
    library) == HaploModel::resolveAll."""
    _estep_on_reference_model(oracle_mod, "a3miss5", 10, 1)


def _estep_on_reference_model(oracle_mod, name, S, mode):
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p, S)
    m.set_estep_mode(mode)
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    ll_o = o.resolve_all()
    assert_estep_equal(m, o, ll_g, ll_o, H, re_g)


# the shapes the automatic rule selects (structure 1 x 4/8/12, 4 x 2, 16 x 1;
# values 1 x 20, 2 x 8, 3 x 8, 8 x 2, 16 / c x c) on two panels, and stress
# shapes the rule never picks on the stress panel (3 alleles, 5 % missing)
_AUTO_SHAPES = [(1, 12, 1, 20), (4, 2, 8, 2), (1, 8, 2, 8), (1, 4, 3, 8), (16, 1, 16, 1), (16, 1, 8, 2)]
_STRESS_SHAPES = [(4, 3, 4, 4), (4, 1, 2, 8), (4, 2, 16, 1), (1, 8, 8, 2), (4, 2, 5, 3), (8, 2, 8, 2),
                  (1, 16, 1, 20), (1, 20, 2, 8), (4, 2, 4, 5)]


@pytest.mark.parametrize("name,shape", [(n, s) for n in ("a3miss5", "n300") for s in _AUTO_SHAPES]
                         + [("a3miss5", s) for s in _STRESS_SHAPES])
def test_estep_pass_shapes(oracle_mod, name, shape):
    """Launch shapes of the split E-step's passes (hmc_set_pass_shapes:
    structure waves per individual 1, 4, 8 or 16, individuals per CU — the
    3, 4 and 5 waves-per-SIMD builds of the structure pass —, value-pass
    shape up to 16 waves per individual) change nothing: the E-step on the M0 model equals
    HaploModel::resolveAll bit for bit."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    m = gpu_model(p)
    m.set_pass_shapes(*shape)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


# combinations cut from the matrix in round 4 (n60 and a8 panels with shapes
# callers can still pick through hmc_set_pass_shapes)
_SLOW_COMBOS = [("n60", (1, 12, 1, 20)), ("n60", (4, 2, 16, 1)), ("a8", (1, 12, 1, 20)), ("a8", (4, 2, 16, 1)),
                ("a8", (16, 1, 8, 2)), ("n60", (4, 3, 4, 4))]


@pytest.mark.slow
@pytest.mark.parametrize("name,shape", _SLOW_COMBOS)
def test_estep_pass_shapes_more_panels(oracle_mod, name, shape):
    """The same check on the panels the round-4 matrix dropped (60 loci i.i.d.,
    8 alleles per locus)."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    m = gpu_model(p)
    m.set_pass_shapes(*shape)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.parametrize("name,S", [("cfg1", 10), ("a3miss5", 3), ("a8", 10), ("n300", 3)])
def test_value_only_mode_with_order_reruns(oracle_mod, name, S):
    """hmc_set_value_mode(0): value-only k-best lists (seg_rank_select), the
    libstdc++ permutations only for individuals with ties — same E-step, bit
    for bit, as HaploModel::resolveAll."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p, S)
    m.set_value_mode("fast")
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    ll_o = o.resolve_all()
    assert_estep_equal(m, o, ll_g, ll_o, H, re_g)
    st = m.estep_split_stats()
    assert 0 <= st["n_order_rerun"] <= p.N


@pytest.mark.parametrize("name,S,shape", [("a3miss5", S, sh) for S, sh in
                                          [(10, None), (1, None), (2, None), (3, None), (5, None), (16, None),
                                           (10, (0, 0, 8, 2)), (10, (0, 0, 2, 8)), (7, (0, 0, 4, 4))]]
                         + [(n, 10, None) for n in ("n60", "a8", "n300")])
def test_value_pair_layout(oracle_mod, name, S, shape):
    """hmc_set_value_layout(2): phase B of the value pass with two links per
    lane (seg2_nth_slots: S lanes and 64 / S lists per wavefront) for every
    group and launch shape — same E-step, bit for bit, as
    HaploModel::resolveAll."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    m = gpu_model(p, S)
    m.set_value_layout(2)
    if shape:
        m.set_pass_shapes(*shape)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.parametrize("name,S,shape", [("a3miss5", 10, None), ("a3miss5", 3, None), ("a3miss5", 10, (0, 0, 8, 2)),
                                          ("n300", 10, None), ("a8", 3, None)])
def test_value_one_link_layout(oracle_mod, name, S, shape):
    """hmc_set_value_layout(0): the round-2 phase-B layout (2S lanes, one link
    per lane; still the automatic one for S > 16) — same E-step, bit for bit,
    as HaploModel::resolveAll."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    m = gpu_model(p, S)
    m.set_value_layout(0)
    if shape:
        m.set_pass_shapes(*shape)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.variants
@pytest.mark.parametrize("name,S,shape,ring,na", [("a3miss5", 10, (0, 0, 8, 2), 3, 3), ("a8", 24, None, 4, 0)])
def test_dataflow_value_pass(oracle_mod, name, S, shape, ring, na):
    """hmc_set_value_pass(dataflow): A wavefronts build the lists locus by
    locus as soon as a state's predecessors are final, the others run the
    chains of adds of any open locus (estep_df.hip) — the E-step on the M0
    model equals HaploModel::resolveAll bit for bit, for sample sizes with two
    links per lane (S <= 16) and one (17..32), ring of 3 or 4 frontiers, 2 to
    16 waves per individual, 1 to 7 A waves (na; 0 = by the shape)."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    m = gpu_model(p, S)
    m.set_value_pass("dataflow", ring)
    m.set_dataflow_waves(na)
    if shape:
        m.set_pass_shapes(*shape)
    m.find_patterns()
    ll_g, H, re_g = m.resolve_all()
    assert m.last_value_pass_dataflow()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.variants
@pytest.mark.parametrize("name,shape,S", [("a3miss5", (4, 2, 0, 0), 10)])
def test_structure_pass_v2(oracle_mod, name, shape, S):
    """hmc_set_structure_pass(2): creation order from each key's first
    contribution and add order from each state's member segment (three block
    scans per locus) — the E-step on the M0 model equals
    HaploModel::resolveAll bit for bit, with both value-pass schedules."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    o.reset_counters()
    ll_o = o.resolve_all()
    for vpass in ("classic", "dataflow"):
        m = gpu_model(p, S)
        m.set_structure_pass(2)
        m.set_value_pass(vpass)
        if shape:
            m.set_pass_shapes(*shape)
        m.find_patterns()
        ll_g, H, re_g = m.resolve_all()
        assert_estep_equal(m, o, ll_g, ll_o, H, re_g)
        m.close()


@pytest.mark.parametrize("name,S", [("a3miss5", 10), ("n300", 10), ("a8", 3), ("cfg1", 10), ("a4", 40)])
def test_structure_end_order(oracle_mod, name, S):
    """hmc_set_end_order: the structure pass over the pattern table sorted by
    (end locus, id) (gmodel.hip) and over the id-ordered table give the same
    E-step as HaploModel::resolveAll on the M0 model (the full-EM tests run
    with it on: the default)."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    o.reset_counters()
    ll1 = o.resolve_all()
    for on in (True, False):
        m = gpu_model(p, S)
        m.set_end_order(on)
        m.find_patterns()
        ll_g, H, re_g = m.resolve_all()
        assert_estep_equal(m, o, ll_g, ll1, H, re_g)
        m.close()


@pytest.mark.variants
@pytest.mark.parametrize("name", ["n60"])
def test_structure_pass_v2_exact_em(oracle_mod, name):
    """The exact M-step's records (forward links in extendAll order, pair
    orientations) from the v2 structure pass: the whole exact EM as with v1."""
    p = panel(name)
    r = None
    logs = []
    for v in (1, 2):
        m = gpu_model(p, max_iteration=6)
        m.exact_estimate = True
        m.set_structure_pass(v)
        res = m.run()
        logs.append(([x["ll"] for x in m.log], res))
        m.close()
    assert logs[0][0] == logs[1][0]
    assert np.array_equal(logs[0][1], logs[1][1])


@pytest.mark.variants
@pytest.mark.parametrize("name", ["n60"])
def test_dataflow_full_em(oracle_mod, name):
    """The whole EM with the dataflow value pass: iteration count, LL, R_E and
    accepted pairs equal the restatement's."""
    p = panel(name)
    m = gpu_model(p, max_iteration=10)
    m.set_value_pass("dataflow")
    res = m.run()
    r = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10).run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])


@pytest.mark.parametrize("S", [1, 2, 5, 16, 17, 24, 32, 33, 40, 64])
def test_estep_sample_sizes(oracle_mod, S):
    p = panel("miss2")
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p, S)
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


def _check_frequency(p, model, start, alleles, samples=None):
    """PatternManager::checkFrequency (PatternManager.cpp:146-193), restated
    in Python floats (sequential IEEE adds in item order)."""
    num, sym, fr = model.allele_table()
    out = []
    for st, al in zip(start, alleles):
        total = 0.0
        if samples is None:
            for i in range(p.N):
                g = p.alleles[i]
                ok, f = True, 1.0
                for j, a in enumerate(al):  # Genotype::isMatch + getMatchingFrequency (:267-291)
                    k = st + j
                    b0, b1 = int(g[0, k]), int(g[1, k])
                    if not (b0 < 0 or b1 < 0 or b0 == a or b1 == a):
                        ok = False
                        break
                    af = 0.0
                    for q in range(num[k]):
                        if sym[k, q] == a:
                            af = fr[k, q]
                    x = 0.0
                    x += af if b0 < 0 else (1.0 if b0 == a else 0.0)
                    x += af if b1 < 0 else (1.0 if b1 == a else 0.0)
                    f *= 0.5 * x
                if ok:
                    total += f
            out.append(total / p.N)
        else:
            sal, w, tw = samples
            for h in range(len(w)):
                if all(sal[h, st + j] == a for j, a in enumerate(al)):
                    total += w[h]
            out.append(total / tw)
    return np.array(out)


@pytest.mark.parametrize("name", ["cfg1", "a3miss5", "a8"])
def test_mine_level_seam(oracle_mod, name):
    """hmc_mine_level (checkFrequency for caller-given candidates, the per-level
    seam of searchPattern): equals the mined tables' frequencies bit for bit,
    M0 from the genotypes and M1 from the samples, and a Python restatement of
    checkFrequency on random (mostly infrequent) candidates."""
    p = panel(name)
    m = gpu_model(p)
    rng = np.random.default_rng(5)
    num, sym, _ = m.allele_table()
    for it in range(2):
        m.find_patterns()
        pt = m.patterns()
        for lv in np.unique(pt["len"]):
            sel = pt["len"] == lv
            f, sc = m.mine_level(pt["start"][sel], pt["alleles"][sel, :lv])
            assert np.array_equal(f, pt["freq"][sel]), (it, lv)
        lv = 4
        st = rng.integers(0, p.L - lv, 40)
        al = np.array([[sym[s + j, rng.integers(0, num[s + j])] for j in range(lv)] for s in st], np.int32)
        f, sc = m.mine_level(st, al)
        samples = None if it == 0 else m.samples(H)
        assert np.array_equal(f, _check_frequency(p, m, st, al, samples)), it
        assert sc == 40 * (p.N if it == 0 else H)
        _, H, _ = m.resolve_all()


@pytest.mark.parametrize("name", sorted(PANELS))
def test_mine_genotypes_and_samples(oracle_mod, name):
    """M0 (genotype branch) and M1 (sample branch) pattern tables, bit-exact."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    _, rm0_o = o.counters()
    m = gpu_model(p)
    P0, rm0 = m.find_patterns()
    assert P0 == len(o.patterns()["start"]) and rm0 == rm0_o
    assert_tables_equal(m.patterns(), o.patterns())
    ll_g, H, _ = m.resolve_all()
    ll_o = o.resolve_all()
    assert ll_g == ll_o
    o.reset_counters()
    P1, rm1 = m.find_patterns()
    o.find_patterns()
    _, rm1_o = o.counters()
    assert rm1 == rm1_o
    assert_tables_equal(m.patterns(), o.patterns())


def test_long_patterns_near_monomorphic(oracle_mod):
    """Patterns far longer than 256 loci (max_pattern_len 0 = L on a
    near-monomorphic panel): M0 and M1 tables, successors included, and the
    E-step between them equal the restatement's."""
    rng = np.random.default_rng(17)
    N, L = 20, 300
    a = np.full((N, 2, L), ord("1"), np.int32)
    for k in (40, 150, 260):  # three polymorphic loci
        a[:, :, k] = np.where(rng.random((N, 2)) < 0.3, ord("2"), ord("1"))
    p = synth.Panel(alleles=a, types="S" * L)
    o = oracle_mod.Oracle(a, p.types, sample_size=4, max_len=0)
    o.find_patterns()
    m = gpu_model(p, S=4, max_pattern_len=0)
    P0, _ = m.find_patterns()
    g = m.patterns()
    assert g["len"].max() > 256
    assert_tables_equal(g, o.patterns())
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)
    m.find_patterns()
    o.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())


@pytest.mark.parametrize("name", ["cfg1", "n60", "a4", "miss2", "a3miss5", "a8"])
def test_full_em(oracle_mod, name):
    """HaploModel::run: iteration count, per-iteration LL / R_E / R_M / pattern
    counts and the accepted haplotype pair of every individual."""
    p = panel(name)
    m = gpu_model(p, max_iteration=30)
    res = m.run()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=30)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert [x["r_e"] for x in m.log] == r["R_E"].tolist()
    assert m.m0["r_m"] == r["R_M"][0] and m.m0["n_patterns"] == r["n_patterns"][0]
    for k in range(r["iterations"] - 1):
        assert m.log[k]["r_m"] == r["R_M"][k + 1]
        assert m.log[k]["n_patterns"] == r["n_patterns"][k + 1]
    assert np.array_equal(res, r["resolutions"])
    # HaploComp log line of every iteration (HaploModel.cpp:134-136): integer
    # counts, so the ratios are bit-equal
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])
    np.testing.assert_array_equal(np.array(m.haplocomp()), r["haplocomp"][-1])


@pytest.mark.parametrize("name,S", [("n60", 40), ("a3miss5", 64)])
def test_full_em_large_sample_size(oracle_mod, name, S):
    """sample_size above one wavefront's lists (S = 40, 64: lists of up to 2S
    links over two lanes' selection slots, HaploPair.cpp:63-89): whole-EM
    parity with the restatement (LL, R_E, R_M, HaploComp, accepted pairs)."""
    p = panel(name)
    m = gpu_model(p, S, max_iteration=30)
    res = m.run()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=S, max_iter=30)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert [x["r_e"] for x in m.log] == r["R_E"].tolist()
    for k in range(r["iterations"] - 1):
        assert m.log[k]["r_m"] == r["R_M"][k + 1]
    assert np.array_equal(res, r["resolutions"])
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])


@pytest.mark.timeout(600)
def test_wide_frontier_over_65535_states(oracle_mod):
    """An individual whose frontier passes 65 535 states at a locus (no
    genotype at all on a panel of 8 alleles per locus, patterns mined down to
    a low threshold: pairs of ~400 patterns per locus): state ids take 21 bits
    in the structure records and list links, the state capacity grows by
    doubling, the contribution capacity too (amax^2 contributions per state
    where both alleles are missing).  The E-step equals
    HaploModel::resolveAll bit for bit."""
    rng = np.random.default_rng(1)
    N, L, A = 100, 6, 8
    al = (rng.integers(0, A, size=(N, 2, L)) + ord("1")).astype(np.int32)
    al[0] = -1
    p = synth.Panel(al, "S" * L)
    o = oracle_mod.Oracle(p.alleles, p.types, min_freq_abs=0.3, max_len=L, sample_size=10)
    o.find_patterns()
    m = gpu_model(p, min_freq_abs=0.3, max_pattern_len=L)
    m.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())
    ll_g, H, re_g = m.resolve_all()
    fr = m.estep_frontier()
    assert fr["max_states"] > 65535, fr
    o.reset_counters()
    assert_estep_equal(m, o, ll_g, o.resolve_all(), H, re_g)


@pytest.mark.parametrize("missing", [0.0, 0.03])
def test_many_alleles(oracle_mod, missing):
    """Loci with 40 alleles (microsatellite 'M' loci; GenoData's allele tables
    are unbounded, GenoData.cpp:78-118): whole-EM parity with the restatement
    (LL, R_E, R_M, HaploComp, accepted pairs), missing alleles included."""
    rng = np.random.default_rng(40)
    base = synth.founder_mosaic(60, 30, A=2, seed=11, missing=missing)
    a = np.where(base.alleles < 0, -1, base.alleles - ord("1") + 1).astype(np.int32)
    for k in (5, 17, 25):
        a[:, :, k] = rng.integers(1, 41, size=(60, 2))
    a[:, :, 17][rng.random((60, 2)) < missing] = -1
    p = synth.Panel(alleles=a, types="M" * 30)
    m = gpu_model(p, max_iteration=10)
    res = m.run()
    assert m.amax > 32
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert [x["r_e"] for x in m.log] == r["R_E"].tolist()
    for k in range(r["iterations"] - 1):
        assert m.log[k]["r_m"] == r["R_M"][k + 1]
    assert np.array_equal(res, r["resolutions"])
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])


@pytest.mark.parametrize("name", ["cfg1", "miss2"])
def test_em_iteration_drives_the_same_chain(oracle_mod, name):
    """hmc_em_iteration (one HaploModel::run iteration, HaploModel.cpp:130-144)
    driven from the host until the continue rule stops: the same iterations,
    LL, R_E / R_M, HaploComp lines and accepted pairs as HaploModel::run."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=30)
    r = o.run()
    m = gpu_model(p)
    m.find_patterns()
    old, logs = -np.finfo(np.float64).max, []
    for it in range(1, 31):
        log, old, go = m.em_iteration(it, old, always_mstep=False, max_iteration=30)
        logs.append(log)
        if not go:
            break
    assert len(logs) == r["iterations"]
    assert [x["log_likelihood"] for x in logs] == r["ll"].tolist()
    assert [x["r_e"] for x in logs] == r["R_E"].tolist()
    for k in range(r["iterations"] - 1):
        assert logs[k]["r_m"] == r["R_M"][k + 1]
    np.testing.assert_array_equal(np.array([(x["switch_error"], x["ihp"], x["igp"]) for x in logs]), r["haplocomp"])
    best = np.zeros((p.N, 2, p.L), np.int32)
    assert hmc_amd.lib().hmc_get_best_resolutions(m._h, best.ctypes.data_as(__import__("ctypes").POINTER(
        __import__("ctypes").c_int32))) == 0
    assert np.array_equal(best, r["resolutions"])


@pytest.mark.parametrize("name,width", [("n300", 31), ("n300", 77), ("n300", 5), ("a4", 31), ("a4", 13),
                                        ("a3miss5", 45), ("miss2", 60), ("miss2", 1)])
def test_mining_in_start_blocks(oracle_mod, name, width):
    """hmc_set_mine_block: the search by blocks of start loci from L-1 down
    (roots of searchPattern's DFS are independent, PatternManager.cpp:90-108)
    gives the restatement's table exactly — ids, allele strings, frequencies,
    prefix frequencies, transition probabilities, successors, R_M — for M0 and
    for the M-step on the samples, and the E-step in between agrees too.
    Blocks narrower than the patterns are long (widths 1, 5, 13) need the
    successors of the block above (mine_succ_level)."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    m = gpu_model(p)
    m.set_mine_block(width)
    for step in range(2):
        o.reset_counters()
        P = o.find_patterns()
        Pg, rm = m.find_patterns()
        st = m.mine_stats()
        assert st["blocks"] == -(-p.L // width), st
        ref, got = o.patterns(maxlen=30), m.patterns(maxlen=30)
        assert Pg == P
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        assert rm == o.counters()[1]
        ll_o = o.resolve_all()
        ll, H, re = m.resolve_all()
        assert ll == ll_o


@pytest.mark.parametrize("name,cap", [("n300", 2 << 20), ("a3miss5", 1 << 20)])
def test_mining_splits_blocks_over_memory_cap(oracle_mod, name, cap):
    """A block whose matching lists exceed the cap (hmc_set_mine_memory, the
    path taken when device memory runs out) is re-run with half the width:
    several blocks, and still the restatement's table, R_M and E-step."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    m = gpu_model(p)
    m.set_mine_memory(cap)
    for step in range(2):
        o.reset_counters()
        P = o.find_patterns()
        Pg, rm = m.find_patterns()
        assert m.mine_stats()["blocks"] >= 2
        ref, got = o.patterns(maxlen=30), m.patterns(maxlen=30)
        assert Pg == P
        for k in ref:
            np.testing.assert_array_equal(got[k], ref[k], err_msg=k)
        assert rm == o.counters()[1]
        assert m.resolve_all()[0] == o.resolve_all()


@pytest.mark.parametrize("name", ["n60", "miss2"])
def test_em_rewind_repeats_the_chain(oracle_mod, name):
    """hmc_model_save after M0 + hmc_em_rewind (bench.py's restart of the
    converged chain): the chain run after a rewind — after a whole first chain
    and extra forced iterations — is the restatement's HaploModel::run chain
    again (LL, R_E, R_M, HaploComp, accepted pairs), and get_patterns returns
    M0's table again."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=30)
    r = o.run()
    m = gpu_model(p)
    m.find_patterns()
    m.model_save()
    pt0 = m.patterns(maxlen=30)

    def chain(extra=0):
        old, logs = -np.finfo(np.float64).max, []
        for it in range(1, 31):
            log, old, go = m.em_iteration(it, old, always_mstep=False, max_iteration=30)
            logs.append(log)
            if not go:
                break
        for it in range(extra):  # forced iterations past the stop (the bench's steady leg)
            m.em_iteration(len(logs) + 1 + it, old, always_mstep=True)
        return logs

    first = chain(extra=2)
    m.em_rewind()
    pt = m.patterns(maxlen=30)
    for k in pt0:  # allele strings included: spelled from the prefix ids, not the replaced tree
        np.testing.assert_array_equal(pt[k], pt0[k])
    again = chain()
    for logs in (first, again):
        assert [x["log_likelihood"] for x in logs] == r["ll"].tolist()
        assert [x["r_e"] for x in logs] == r["R_E"].tolist()
        for k in range(r["iterations"] - 1):
            assert logs[k]["r_m"] == r["R_M"][k + 1]
        np.testing.assert_array_equal(np.array([(x["switch_error"], x["ihp"], x["igp"]) for x in logs]),
                                      r["haplocomp"])
    best = np.zeros((p.N, 2, p.L), np.int32)
    assert hmc_amd.lib().hmc_get_best_resolutions(m._h, best.ctypes.data_as(__import__("ctypes").POINTER(
        __import__("ctypes").c_int32))) == 0
    assert np.array_equal(best, r["resolutions"])


@pytest.mark.parametrize("name,model,order,min_len", [
    ("n60", "MC", 1, 1), ("a3miss5", "MC", 1, 1), ("n60", "MC", 2, 1), ("a4", "MC", 1, 1),
    ("miss2", "MA", 1, 1), ("n60", "MV", 1, 2), ("a3miss5", "MV", 1, 3)])
def test_full_em_models(oracle_mod, name, model, order, min_len):
    """The other models of HaploModel::setModel (HaploModel.cpp:26-36, 65-76) and
    min_pattern_len > 1: MC mines every length-(order+1) candidate
    (findPatternBlock, PatternManager.cpp:72-88) and starts the E-step from
    length-(order+1) heads (initHeadList, HaploBuilder.cpp:153-224, on the host);
    MA is MV plus range checks.  Whole-EM parity as in test_full_em, including the
    per-iteration pattern tables' sizes, R_E / R_M and the HaploComp log."""
    p = panel(name)
    m = gpu_model(p, max_iteration=12, model=model, mc_order=order, min_pattern_len=min_len)
    res = m.run()
    o = oracle_mod.Oracle(p.alleles, p.types, min_len=min_len, sample_size=10, max_iter=12)
    o.set_model(model, order)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert [x["r_e"] for x in m.log] == r["R_E"].tolist()
    assert m.m0["r_m"] == r["R_M"][0] and m.m0["n_patterns"] == r["n_patterns"][0]
    for k in range(r["iterations"] - 1):
        assert m.log[k]["r_m"] == r["R_M"][k + 1]
        assert m.log[k]["n_patterns"] == r["n_patterns"][k + 1]
    assert np.array_equal(res, r["resolutions"])
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])


def test_mc_model_estep_and_table(oracle_mod):
    """MC, one E-step and one M-step compared in full: pattern table (every
    length-2 candidate, zero-frequency ones included), head pairs through the
    traceback (samples), weights and the next table."""
    p = panel("a3miss5")
    m = gpu_model(p, model="MC", mc_order=1)
    m._push_params()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.set_model("MC", 1)
    m.find_patterns()
    o.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())
    assert m.head_len() == o.head_len() == 2
    o.reset_counters()
    ll_g, H, re_g = m.resolve_all()
    ll_o = o.resolve_all()
    assert_estep_equal(m, o, ll_g, ll_o, H, re_g)
    m.find_patterns()
    o.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())


@pytest.mark.parametrize("K,N,L,min_len,num", [
    (2, 40, 30, 1, 20), (2, 40, 30, 1, 150), (2, 40, 30, 1, 400), (2, 40, 30, 2, 150), (2, 40, 30, 2, 400),
    (3, 50, 40, 1, 150), (3, 50, 40, 1, 400), (3, 50, 40, 2, 60)])
def test_find_pattern_by_num(oracle_mod, K, N, L, min_len, num):
    """findPatternByNum (PatternManager.cpp:44-70): rounds of searchPattern(true)
    at thresholds 1.0, 0.9, ... with reserved candidates, the last round sorted
    by frequency (std::sort) and cut at num_patterns.  Low-diversity panels
    (K founders, monomorphic stretches) make the rounds and the cut matter.
    Pattern tables after M0 and M1 in full, then the whole EM."""
    p = synth.founder_mosaic(N, L, A=2, K=K, seed=5)
    m = gpu_model(p, num_patterns=num, min_pattern_len=min_len)
    o = oracle_mod.Oracle(p.alleles, p.types, min_len=min_len, sample_size=10)
    o.set_num_patterns(num)
    o.reset_counters()
    P0, rm0 = m.find_patterns()
    o.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())
    assert rm0 == o.counters()[1]
    o.reset_counters()
    ll_g, H, re_g = m.resolve_all()
    ll_o = o.resolve_all()
    assert_estep_equal(m, o, ll_g, ll_o, H, re_g)
    o.reset_counters()
    P1, rm1 = m.find_patterns()
    o.find_patterns()
    assert_tables_equal(m.patterns(), o.patterns())
    assert rm1 == o.counters()[1]
    m2 = gpu_model(p, max_iteration=10, num_patterns=num, min_pattern_len=min_len)
    res = m2.run()
    o2 = oracle_mod.Oracle(p.alleles, p.types, min_len=min_len, sample_size=10, max_iter=10)
    o2.set_num_patterns(num)
    r = o2.run()
    assert m2.iterations == r["iterations"]
    assert [x["ll"] for x in m2.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])


@pytest.mark.parametrize("gname", ["cfg1", "miss_a3", "snp_miss", "s3"])
def test_against_golden_fixtures(gname):
    sys.path.insert(0, os.path.join(HERE, "golden"))
    import make_golden

    c = make_golden.CASES[gname]
    g = np.load(os.path.join(HERE, "golden", f"{gname}.npz"))
    p = synth.founder_mosaic(c["N"], c["L"], A=c["A"], missing=c["missing"], seed=c["seed"])
    assert np.array_equal(p.alleles, g["alleles"])
    m = gpu_model(p, c["S"])
    m.find_patterns()
    pt = m.patterns(maxlen=g["m0_alleles"].shape[1])
    for k in ("start", "len", "freq", "prefix", "tp", "succ", "alleles"):
        assert np.array_equal(pt[k], g["m0_" + k]), k
    ll, H, _ = m.resolve_all()
    assert ll == g["e1_ll"][0]
    er = m.estep_results()
    assert np.array_equal(er["ncand"], g["e1_ncand"]) and np.array_equal(er["total"], g["e1_total"])
    al, w, tw = m.samples(H)
    assert np.array_equal(al, g["e1_samples"]) and np.array_equal(w, g["e1_w"]) and tw == g["e1_tw"][0]
    m2 = gpu_model(p, c["S"], max_iteration=20)
    res = m2.run()
    assert m2.iterations == g["em_iterations"][0]
    assert np.array_equal(np.array([x["ll"] for x in m2.log]), g["em_ll"])
    assert np.array_equal(res, g["em_resolutions"])


def test_phase_file_io(tmp_path, oracle_mod):
    p = panel("a3miss5")
    f = tmp_path / "in.phase"
    synth.write_phase(p, str(f))
    m = hmc_amd.HaploModel()
    m.max_iteration = 10
    m.load_phase(str(f))  # HaploFile::readGenoData
    res = m.run()
    m2 = gpu_model(p, max_iteration=10)
    assert np.array_equal(res, m2.run())
    out = tmp_path / "out.phase"
    m.write_phase(str(out))  # HaploFile::writeGenoData
    back = synth.read_phase(str(out))
    assert np.array_equal(back.alleles, res)


def test_edge_cases(oracle_mod):
    """L = 1, monomorphic loci, an all-missing locus and individual, missing at
    locus 0 (initHeadList's missing-complement branch)."""
    rng = np.random.default_rng(9)
    base = synth.founder_mosaic(30, 12, A=3, missing=0.0, seed=9).alleles.copy()
    base[:, :, 3] = ord("2")        # monomorphic locus
    base[:, :, 5] = -1              # all missing at one locus
    base[4, :, :] = -1              # one individual entirely missing
    base[7, 0, 0] = -1              # one missing allele at locus 0
    base[8, :, 0] = -1              # both missing at locus 0
    cases = [base, base[:, :, :1].copy(), base[:5, :, 2:4].copy()]
    for a in cases:
        o = oracle_mod.Oracle(a, "S" * a.shape[2], sample_size=10, max_iter=10)
        r = o.run()
        m = hmc_amd.HaploModel()
        m.max_iteration = 10
        res = m.run(hmc_amd.GenoData(a, "S" * a.shape[2]))
        assert m.iterations == r["iterations"]
        assert [x["ll"] for x in m.log] == r["ll"].tolist()
        assert np.array_equal(res, r["resolutions"])


@pytest.mark.parametrize("vpass,S,sv", [("classic", 4, 1), ("classic", 40, 1),
                                        pytest.param("dataflow", 4, 2, marks=pytest.mark.variants)])
def test_underflow_unresolved(oracle_mod, vpass, S, sv):
    """Raw double products underflow on long i.i.d. panels; those individuals
    are unresolved (HaploBuilder.cpp:117-124), LL = -inf and the EM stops —
    both implementations must agree on all of it.  The individuals whose
    forward likelihoods reach 0 are re-built with extend()'s forward test
    (HaploBuilder.cpp:237): any sample size, either value-pass schedule."""
    rng = np.random.default_rng(5)
    a = (rng.integers(0, 2, (6, 2, 2500)) + ord("1")).astype(np.int32)
    o = oracle_mod.Oracle(a, "S" * 2500, sample_size=S, max_iter=3)
    r = o.run()
    m = hmc_amd.HaploModel()
    m.set_value_pass(vpass)
    m.set_structure_pass(sv)
    m.sample_size = S
    m.max_iteration = 3
    res = m.run(hmc_amd.GenoData(a, "S" * 2500))
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.isneginf(r["ll"][0])
    assert np.array_equal(res, r["resolutions"])
    # the split E-step hands the underflowing individuals to the fused kernel
    assert m.estep_split_stats()["n_fallback"] > 0


def _digest_patterns(pt):
    h = hashlib.sha256()
    for k in ("start", "len", "freq", "prefix", "tp", "succ"):
        h.update(np.ascontiguousarray(pt[k]).tobytes())
    return h.hexdigest()


def test_cfg2_full_size_against_oracle_digest():
    """BASELINE configs[1] (1000 x 500) at full size: per-iteration LL,
    pattern counts, R_E, R_M and SHA-256 of the M0 table and of the accepted
    resolutions equal the restatement's (tests/golden/cfg2_digest.json)."""
    d = json.load(open(os.path.join(HERE, "golden", "cfg2_digest.json")))
    p = synth.config_panel(2)
    m = gpu_model(p)
    m.find_patterns()
    assert _digest_patterns(m.patterns(maxlen=1)) == d["m0_patterns_sha256"]
    m2 = gpu_model(p, max_iteration=50)
    res = m2.run()
    assert m2.iterations == d["iterations"]
    assert [float(x["ll"]).hex() for x in m2.log] == d["ll_hex"]
    assert [x["r_e"] for x in m2.log] == d["R_E"]
    assert m2.m0["r_m"] == d["R_M"][0] and m2.m0["n_patterns"] == d["n_patterns"][0]
    for k in range(d["iterations"] - 1):
        assert m2.log[k]["r_m"] == d["R_M"][k + 1]
        assert m2.log[k]["n_patterns"] == d["n_patterns"][k + 1]
    assert hashlib.sha256(np.ascontiguousarray(res, np.int32).tobytes()).hexdigest() == d["resolutions_sha256"]


def test_cfg5_full_size_properties():
    """BASELINE config 5 at full size (10 000 individuals x 1 000 loci, 8 alleles
    per locus: the divergent multi-allelic frontier): every selected pair is a
    phasing of its genotype, priors sorted, weights sum to 1 per individual,
    the M1 table is a proper pattern table (checked successors are suffixes),
    and E1 repeats bit for bit."""
    import time
    t0 = time.time()
    p = synth.config_panel(5)
    m = gpu_model(p)
    m.find_patterns()
    ll, H, re1 = m.resolve_all()
    print(f"cfg5 M0+E1 {time.time() - t0:.1f} s", flush=True)
    er = m.estep_results()
    g = p.alleles
    nc = er["ncand"]
    assert np.all(nc > 0) and np.isfinite(ll) and H == int(2 * nc.sum())
    k = np.arange(er["prior"].shape[1])
    valid = k[None, :] < nc[:, None]
    pr = np.where(valid, er["prior"], 0.0)  # slots past ncand are not compared (valid[:, 1:] implies both valid)
    assert np.all(np.diff(pr, axis=1)[valid[:, 1:]] <= 0)
    assert np.all(np.abs(np.where(valid, er["weight"], 0.0).sum(1) - 1.0) < 1e-12)
    res = m.resolutions()
    ok = ((res[:, 0] == g[:, 0]) & (res[:, 1] == g[:, 1])) | ((res[:, 0] == g[:, 1]) & (res[:, 1] == g[:, 0]))
    assert ok.all()
    ll2, H2, re2 = m.resolve_all()
    assert (ll2, H2, re2) == (ll, H, re1)
    print(f"cfg5 E1 again {time.time() - t0:.1f} s", flush=True)
    P, _ = m.find_patterns()
    pt = m.patterns()
    print(f"cfg5 M1 {P} patterns {time.time() - t0:.1f} s", flush=True)
    num, sym, _ = m.allele_table()
    assert np.all(pt["freq"] > 0) and np.all(pt["freq"] <= 1) and np.all(pt["tp"] <= 1)
    rng = np.random.default_rng(5)
    for i in rng.choice(P, 500, replace=False):
        e = pt["start"][i] + pt["len"][i]
        if e >= p.L:
            continue
        for j in range(num[e]):
            s = pt["succ"][i, j]
            if s < 0:
                continue
            ext = np.append(pt["alleles"][i, :pt["len"][i]], sym[e, j])
            assert pt["start"][s] + pt["len"][s] == e + 1
            assert np.array_equal(pt["alleles"][s, :pt["len"][s]], ext[len(ext) - pt["len"][s]:])


def test_cfg2_properties():
    """Size-independent properties at full size: samples are phasings of the
    genotypes, weights of each individual sum to 1, priors are sorted, successors
    are suffixes, frequencies in (0, 1], tp <= 1, and the run is deterministic."""
    p = synth.config_panel(2)
    m = gpu_model(p)
    m.find_patterns()
    ll, H, _ = m.resolve_all()
    er = m.estep_results()
    al, w, tw = m.samples(H)
    g = p.alleles
    base = 0
    for i in range(p.N):
        n = er["ncand"][i]
        assert n > 0
        assert np.all(np.diff(er["prior"][i, :n]) <= 0)
        assert abs(er["weight"][i, :n].sum() - 1.0) < 1e-12
        for c in range(n):
            h0, h1 = al[base + 2 * c], al[base + 2 * c + 1]
            ok = ((h0 == g[i, 0]) & (h1 == g[i, 1])) | ((h0 == g[i, 1]) & (h1 == g[i, 0]))
            assert ok.all()
        base += 2 * n
    assert base == H and abs(tw - 2 * p.N) < 1e-9  # two haplotypes per individual, weights sum to 1 each
    P, _ = m.find_patterns()
    pt = m.patterns()
    num, sym, _ = m.allele_table()
    assert np.all(pt["freq"] > 0) and np.all(pt["freq"] <= 1) and np.all(pt["tp"] <= 1)
    rng = np.random.default_rng(0)
    for i in rng.choice(P, 2000, replace=False):
        e = pt["start"][i] + pt["len"][i]
        if e >= p.L:
            continue
        for j in range(num[e]):
            s = pt["succ"][i, j]
            if s < 0:
                continue
            ext = np.append(pt["alleles"][i, :pt["len"][i]], sym[e, j])
            assert pt["start"][s] + pt["len"][s] == e + 1
            assert np.array_equal(pt["alleles"][s, :pt["len"][s]], ext[len(ext) - pt["len"][s]:])
    m3 = gpu_model(p)
    m3.find_patterns()
    assert m3.resolve_all()[0] == ll


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.parametrize("reduction", ["ordered", "allreduce"])
@pytest.mark.parametrize("variant", ["MV", "MC", "BYNUM", "WIN"])
def test_two_ranks_one_gpu_host_collective(oracle_mod, tmp_path, variant, reduction):
    """The sharded multi-rank path (individual shards, per-level cross-rank
    candidate sums, LL / total weight, the HaploComp counters) with 2 ranks on
    one GPU and a gloo host collective, for MV, MC, findPatternByNum and MV
    with every E-step windowed (WIN: windows of 7 loci on each rank's shard).
    Ordered reduction (default) continues every sum rank by rank in the
    reference's item order: tolerance 0 — LL, every accepted pair and the
    HaploComp log equal the single-rank restatement's.  All-reduce mode
    reassociates the sums: LL to 1e-10 relative, and the fraction of differing
    resolutions is reported."""
    script = os.path.join(HERE, "_two_rank_worker.py")
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE="2")
    procs = [subprocess.Popen([sys.executable, script, str(r), str(tmp_path), variant, reduction],
                              env=dict(env, RANK=str(r))) for r in range(2)]
    for pr in procs:
        assert pr.wait(timeout=300) == 0
    p = panel("a3miss5")
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10,
                          min_len=2 if variant == "BYNUM" else 1)
    if variant == "MC":
        o.set_model("MC", 1)
    elif variant == "BYNUM":
        o.set_num_patterns(150)
    r = o.run()
    outs = [np.load(tmp_path / f"rank{k}.npz") for k in range(2)]
    ll = outs[0]["ll"]
    assert np.array_equal(ll, outs[1]["ll"])  # every rank sees the same LL
    assert len(ll) == r["iterations"]
    res = np.concatenate([outs[0]["res"], outs[1]["res"]])
    same = np.mean(np.all(res == r["resolutions"], axis=(1, 2)))
    assert np.array_equal(outs[0]["m0_freq"], outs[1]["m0_freq"])
    assert np.array_equal(outs[0]["comp"], outs[1]["comp"])  # HaploComp over both shards
    if reduction == "ordered":
        assert np.array_equal(ll, r["ll"])
        assert same == 1.0
        np.testing.assert_array_equal(outs[0]["comp"], r["haplocomp"])
        o0 = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, min_len=2 if variant == "BYNUM" else 1)
        if variant == "MC":
            o0.set_model("MC", 1)
        elif variant == "BYNUM":
            o0.set_num_patterns(150)
        o0.find_patterns()
        assert np.array_equal(outs[0]["m0_freq"], o0.patterns()["freq"])
    else:
        print(f"all-reduce mode: {100 * (1 - same):.1f}% of resolutions differ from one rank", flush=True)
        assert np.allclose(ll, r["ll"], rtol=1e-10, atol=0)
        assert same >= 0.97, same


def _rccl_comm_one_rank():
    """A one-rank RCCL communicator owned by the caller (hmc_ctx_create_comm),
    made with the RCCL libhmc_amd is linked with (torch may have loaded a
    second librccl into the process; its communicators are not interchangeable)."""
    import ctypes as C
    L = hmc_amd.lib()
    uid = C.create_string_buffer(hmc_amd.HaploModel.unique_id(), 128)
    comm = C.c_void_p()
    assert L.hmc_rccl_comm_init(0, 1, 0, C.cast(uid, C.c_void_p), C.byref(comm)) == 0
    return L, comm


@pytest.mark.parametrize("how", ["unique_id", "caller_comm"])
@pytest.mark.parametrize("reduction", ["ordered", "allreduce"])
def test_rccl_collectives_one_rank(oracle_mod, how, reduction):
    """The RCCL branch (ncclCommInitRank, ncclBroadcast of the ordered
    reduction, ncclAllReduce) run on a one-rank communicator: with
    hmc_set_force_collectives a one-rank context executes every collective, so
    the whole EM goes through RCCL on a one-GPU machine — LL, resolutions and
    the HaploComp log equal the restatement's."""
    p = panel("a3miss5")
    if how == "unique_id":
        m = hmc_amd.HaploModel(device=0, rank=0, world=1, unique_id=hmc_amd.HaploModel.unique_id())
        rccl = None
    else:
        rccl, comm = _rccl_comm_one_rank()
        m = hmc_amd.HaploModel(device=0, rccl_comm=comm.value)
    m.set_force_collectives(True)
    m.set_reduction(reduction)
    m.max_iteration = 10
    res = m.run(hmc_amd.GenoData.from_panel(p))
    r = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10).run()
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])
    np.testing.assert_array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])
    cs = m.comm_stats()
    if reduction == "ordered":
        # every mining level's sums and every E-step's LL / weight went through
        # a grouped ncclSend + ncclRecv hop (to this rank itself) into a
        # NaN-poisoned buffer: the run above is bit-exact through that path
        assert cs["sends"] == cs["recvs"] > 0 and cs["bytes_received"] > 0, cs
        print(f"ordered chain over RCCL send/recv: {cs}", flush=True)
    else:
        assert cs["sends"] == cs["recvs"] == 0, cs
    m.close()
    if rccl is not None:
        assert rccl.hmc_rccl_comm_destroy(comm) == 0  # the caller's communicator outlives the context


@pytest.mark.parametrize("name,kw", [("cfg1", {}), ("a3miss5", {}), ("n300", {"model": "MC"})])
def test_rccl_send_recv_chain_full_em(oracle_mod, name, kw):
    """The ordered reduction's point-to-point path (ctx.hpp ordered_chain:
    ncclRecv -> continue -> ncclSend -> ncclBroadcast) on a one-rank RCCL
    communicator: each hop is a grouped ncclSend/ncclRecv to the rank itself
    into a NaN-poisoned buffer.  Whole EMs equal the restatement's bit for bit
    (every LL, every accepted pair, the M0 table)."""
    p = panel(name)
    m = hmc_amd.HaploModel(device=0, rank=0, world=1, unique_id=hmc_amd.HaploModel.unique_id())
    m.set_force_collectives(True)
    m.set_comm_timeout(600)
    o0 = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10)
    if kw.get("model") == "MC":
        m.model, m.mc_order = "MC", 1
        o0.set_model("MC", 1)
    m.max_iteration = 10
    res = m.run(hmc_amd.GenoData.from_panel(p))
    r = o0.run()
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])
    cs = m.comm_stats()
    assert cs["sends"] == cs["recvs"] > 0, cs
    m.close()


HMC_ERCCL = -6  # include/hmc_amd.h


def test_rccl_bounded_wait_aborts():
    """A stream that does not drain within the communicator timeout ends the
    call with HMC_ERCCL (the communicator is aborted, ncclCommAbort) instead
    of waiting forever; later collectives of the context fail the same way.
    The stall is a bounded one-wavefront kernel (hmc_debug_stall)."""
    import ctypes as C
    m = hmc_amd.HaploModel(device=0, rank=0, world=1, unique_id=hmc_amd.HaploModel.unique_id())
    m.set_force_collectives(True)
    L = hmc_amd.lib()
    m.set_comm_timeout(30)
    assert L.hmc_debug_stall(m._h, C.c_double(50.0)) == 0  # drains inside the timeout
    m.set_comm_timeout(0.2)
    t0 = time.time()
    rc = L.hmc_debug_stall(m._h, C.c_double(2000.0))
    dt = time.time() - t0
    msg = L.hmc_ctx_error(m._h).decode()
    assert rc == HMC_ERCCL, (rc, msg)
    assert "timeout" in msg, msg
    assert dt < 10, dt
    p = panel("cfg1")
    with pytest.raises(hmc_amd.HMCError) as ei:
        m.run(hmc_amd.GenoData.from_panel(p))
    assert ei.value.code == HMC_ERCCL, ei.value
    m.close()


def test_shard_ranges_balanced_and_tiling():
    """Every rank's [i0, i1) from the library equals the documented rule
    (hmc_amd.model.balanced_shard) and the ranges tile [0, N)."""
    import ctypes as C
    from hmc_amd.model import balanced_shard
    p = panel("miss2")
    L = hmc_amd.lib()
    world, prev = 3, 0
    noop = hmc_amd._lib.ALLREDUCE_FN(lambda buf, n, user: 0)
    for r in range(world):
        h = C.c_void_p()
        assert L.hmc_ctx_create_hostcoll(0, r, world, noop, None, C.byref(h)) == 0
        al = np.ascontiguousarray(p.alleles, dtype=np.int32)
        assert L.hmc_load_genotypes(h, p.N, p.L, al.ctypes.data_as(C.POINTER(C.c_int32)), p.types.encode()) == 0
        i0, i1 = C.c_int(), C.c_int()
        assert L.hmc_shard_range(h, C.byref(i0), C.byref(i1)) == 0
        assert (i0.value, i1.value) == balanced_shard(p.alleles, r, world)
        assert i0.value == prev
        prev = i1.value
        L.hmc_ctx_destroy(h)
    assert prev == p.N


@pytest.mark.parametrize("name", ["a3miss5", "cfg1", "n300"])
def test_estep_shape_invariance(oracle_mod, name):
    """1, 2 and 4 wavefronts per individual (and any LDS split) of the
    split E-step give the identical E-step: same LL, resolutions, weights
    and link count."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    pt = o.patterns()
    ref = None
    for mode, nw, ipc in [(0, 1, 4), (0, 2, 4), (0, 4, 2), (0, 2, 1), (0, 2, 16), (0, 3, 32)]:
        m = gpu_model(p, 10)
        m.set_estep_mode(mode)
        m.set_estep_shape(nw, ipc)
        m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
        ll, H, re = m.resolve_all()
        er = m.estep_results()
        got = (ll, H, re, m.resolutions().tobytes(), er["weight"].tobytes(), er["prior"].tobytes())
        if ref is None:
            ref = got
        assert got == ref, (mode, nw, ipc)


@pytest.mark.parametrize("mode", [0, pytest.param(1, marks=pytest.mark.variants)], ids=["split", "fused"])
def test_small_frontier_capacity_retries(oracle_mod, mode):
    """A frontier capacity far below the panel's frontiers: the batch is re-run
    with doubled capacities (HBM tiers, key tables, contribution lists) until
    it fits, with results identical to the restatement."""
    p = panel("n300")
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    pt = o.patterns()
    m = gpu_model(p, 10)
    m.set_estep_mode(mode)
    m.set_tuning(frontier_cap=8)
    m.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last_symbols(pt))
    ll_g, H, re_g = m.resolve_all()
    o.reset_counters()
    ll_o = o.resolve_all()
    assert_estep_equal(m, o, ll_g, ll_o, H, re_g)


@pytest.mark.parametrize("sw", [32, 20, 8, 2])
def test_segmented_nth_element_matches_libstdcxx(oracle_mod, sw):
    """The segmented wave selection of the E-step kernel (coop_select.hpp),
    64/sw lists per wavefront, permutes every list exactly like
    std::nth_element (ties, NaN, sorted and organ-pipe inputs, n up to the
    segment width; 32 = 2 x the largest sample size)."""
    import ctypes as C

    rng = np.random.default_rng(77 + sw)
    liks, ns, nths = [], [], []
    for n in list(range(1, sw + 1)) * 24:
        kind = rng.integers(0, 6)
        if kind == 0:
            v = rng.random(n)
        elif kind == 1:
            v = rng.integers(0, 3, n).astype(np.float64)
        elif kind == 2:
            v = np.zeros(n)
        elif kind == 3:
            v = np.arange(n, dtype=np.float64)[:: (1 if rng.random() < 0.5 else -1)].copy()
        elif kind == 4:
            v = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(np.float64)
        else:
            v = rng.integers(0, 4, n).astype(np.float64) * 1e-300
            v[rng.integers(0, n)] = np.nan
        liks.append(v)
        ns.append(n)
        nths.append(int(rng.integers(0, n + 1)))  # nth == n is a no-op in libstdc++
    perm = rng.permutation(len(ns))  # mix lengths inside each wavefront
    liks = [liks[i] for i in perm]
    ns = [ns[i] for i in perm]
    nths = [nths[i] for i in perm]
    off = np.cumsum([0] + ns[:-1]).astype(np.int32)
    lik = np.concatenate(liks)
    tag = np.concatenate([np.arange(n, dtype=np.uint32) for n in ns])
    l2, t2 = lik.copy(), tag.copy()
    n_a, nth_a = np.array(ns, np.int32), np.array(nths, np.int32)
    rc = hmc_amd.lib().hmc_test_coop_nth_element(
        0, l2.ctypes.data_as(C.POINTER(C.c_double)), t2.ctypes.data_as(C.POINTER(C.c_uint32)),
        off.ctypes.data_as(C.POINTER(C.c_int32)), n_a.ctypes.data_as(C.POINTER(C.c_int32)),
        nth_a.ctypes.data_as(C.POINTER(C.c_int32)), len(ns), len(lik), sw)
    assert rc == 0
    for b, n in enumerate(ns):
        o = off[b]
        _, ref = oracle_mod.std_nth_element(lik[o:o + n], tag[o:o + n].astype(np.int32), nths[b])
        assert np.array_equal(t2[o:o + n].astype(np.int32), ref), (n, nths[b], lik[o:o + n])


# ---------------------------------------------------------------- exact M-step
EXACT_PANELS = ["cfg1", "n60", "a4", "miss2", "a3miss5", "a8"]


def _rel_close(a, b, rtol=1e-6, atol=1e-12):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= atol + rtol * np.abs(b))


def _assert_table_bits(pg, po):
    """The exact M-step's table equals the restatement's bit for bit: the
    restatement walks in the device walk's order (oracle/hmc_oracle.cpp
    xwalk: gathers in add order, 64 strided partials and the butterfly, 2^-44
    fixed-point totals) — the reference's own order is std::map pointer order,
    reproducible by neither."""
    for k in ("start", "len", "alleles", "succ"):
        assert np.array_equal(pg[k], po[k]), k
    for k in ("freq", "prefix", "tp"):
        d = np.max(np.abs(pg[k] - po[k]) / np.maximum(np.abs(po[k]), 1e-300)) if len(po[k]) else 0.0
        assert np.array_equal(pg[k], po[k]), (k, d, int(np.sum(pg[k] != po[k])))


@pytest.mark.parametrize("name", EXACT_PANELS)
def test_exact_mstep_against_oracle(oracle_mod, name):
    """--exact-estimate (PatternManager::estimatePatterns, HaploBuilder::
    estimateFrequency): after M0 and E1, one exact M-step gives the
    restatement's table — the same patterns in the same (candidate) order,
    successors, frequencies, prefix frequencies and transition probabilities
    bit for bit (_assert_table_bits; the north star's bar is 1e-6: the
    reference sums its match lists in pointer order)."""
    p = panel(name)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    o.resolve_all()
    P_o, _ = o.estimate_patterns()
    po = o.patterns()
    m = gpu_model(p)
    m.exact_estimate = True
    m.find_patterns()  # M0 mines the genotypes
    m.resolve_all()
    P_g, _ = m.find_patterns()  # after an E-step: estimatePatterns
    pg = m.patterns()
    st = m.exact_stats()
    assert st["rounds"] >= 1 and st["candidates"] >= P_g
    assert P_g == P_o
    _assert_table_bits(pg, po)


def test_exact_mstep_wide_trie(oracle_mod):
    """The exact walk's wide-trie paths: microsatellite loci with up to 20
    alleles (trie width 20 > 10), so marking reads each target's header
    instead of the allele-pair ballot and no per-depth child or non-zero-mask
    cache is kept (exact.hip, exact_walk_cache_w) — the table still equals the
    restatement's bit for bit."""
    rng = np.random.default_rng(20)
    base = synth.founder_mosaic(40, 30, A=2, seed=11)
    a = np.where(base.alleles < 0, -1, base.alleles - ord("1") + 1).astype(np.int32)
    for k in (4, 11, 19, 26):
        a[:, :, k] = rng.integers(1, 21, size=(40, 2))
    p = synth.Panel(alleles=a, types="M" * 30)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.find_patterns()
    o.resolve_all()
    P_o, _ = o.estimate_patterns()
    po = o.patterns()
    m = gpu_model(p)
    m.exact_estimate = True
    m.find_patterns()
    m.resolve_all()
    P_g, _ = m.find_patterns()
    assert m.amax > 10
    assert P_g == P_o
    _assert_table_bits(m.patterns(), po)


RARE = dict(N=80, L=50, A=2, K=40, rho=0.05, seed=12)  # patterns down to min_freq = 0.2 / 2N = 1.25e-3


@pytest.mark.parametrize("name", EXACT_PANELS + ["rare"])
def test_exact_mstep_against_reference_order(oracle_mod, name):
    """The north star's bar against an independent restatement: the GPU's
    exact M-step table vs the restatement that sums in the reference's own
    grouping in double (oracle rwalk: HaploBuilder.cpp:369-434 — list 0's
    terms, then list 1's, then list 2's, predecessors in creation order for
    std::map's pointer order; frequencies and prefixes added in double in
    visiting order, :437-441), not a copy of the device's arithmetic.  Same
    patterns, order and successors; freq / prefix / tp within 1e-6 relative,
    including `rare`, whose patterns sit at the min_freq threshold."""
    if name == "rare":
        p, mfa = synth.founder_mosaic(**RARE), 0.2
    else:
        p, mfa = panel(name), 1.5
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, min_freq_abs=mfa)
    o.set_exact_order("reference")
    o.find_patterns()
    o.resolve_all()
    P_o, _ = o.estimate_patterns()
    po = o.patterns()
    m = gpu_model(p, min_freq_abs=mfa)
    m.exact_estimate = True
    m.find_patterns()
    m.resolve_all()
    P_g, _ = m.find_patterns()
    pg = m.patterns()
    assert P_g == P_o
    for k in ("start", "len", "alleles", "succ"):
        assert np.array_equal(pg[k], po[k]), k
    for k in ("freq", "prefix", "tp"):
        rel = np.abs(pg[k] - po[k]) / np.maximum(np.abs(po[k]), 1e-300)
        print(f"{name} {k}: max rel {rel.max():.2e} over {len(rel)} patterns (min {po[k].min():.3g})", flush=True)
        assert _rel_close(pg[k], po[k], rtol=1e-6, atol=0.0), (k, rel.max())


@pytest.mark.variants
@pytest.mark.parametrize("name", ["n60"])
def test_exact_walk_four_items_per_wave(oracle_mod, name):
    """hmc_set_exact_walk(4): the depth-first walk with four (individual, start
    locus) items per wavefront, 16 lanes each — the fixed-point frequency sums
    are the same integers, so the table equals the default walk's (mode 1) bit
    for bit; (2) the breadth-first walk, one trie node per lane, sums each
    child's frequency in state order instead of the wavefront's butterfly:
    the same table within 1e-12."""
    p = panel(name)
    tabs = []
    for ipw in (1, 4, 2):
        m = gpu_model(p)
        m.exact_estimate = True
        m.set_exact_walk(ipw)
        m.find_patterns()
        m.resolve_all()
        m.find_patterns()
        tabs.append(m.patterns())
        m.close()
    for k in ("start", "len", "alleles", "succ", "freq", "prefix", "tp"):
        assert np.array_equal(tabs[0][k], tabs[1][k]), k
    for k in ("start", "len", "alleles", "succ"):
        assert np.array_equal(tabs[0][k], tabs[2][k]), k
    for k in ("freq", "prefix", "tp"):
        assert np.allclose(tabs[0][k], tabs[2][k], rtol=1e-12, atol=1e-15), k


@pytest.mark.timeout(900)
def test_exact_mstep_300x200_against_oracle(oracle_mod):
    """The exact M-step on a 300 x 200 panel (the survey's probe size):
    after M0 and E1, one exact M-step equals the restatement's table — same
    patterns, order and successors, frequencies / prefix / tp bit for bit."""
    p = panel("n300")
    oracle_mod.set_threads(16)
    try:
        o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
        o.find_patterns()
        o.resolve_all()
        P_o, _ = o.estimate_patterns()
        po = o.patterns()
    finally:
        oracle_mod.set_threads(1)
    m = gpu_model(p)
    m.exact_estimate = True
    m.find_patterns()
    m.resolve_all()
    P_g, _ = m.find_patterns()
    pg = m.patterns()
    assert P_g == P_o
    _assert_table_bits(pg, po)


@pytest.mark.timeout(900)
def test_exact_mstep_with_pruned_individual(oracle_mod):
    """An individual some of whose pairs' forward likelihoods underflow to 0
    (extend() skips them, HaploBuilder.cpp:237) while its genotype probability
    stays positive — founder mosaic 60 x 1 600, seed 1, found with the
    restatement's skip counter: E1 rebuilds it with the pruned structure pass
    (n_fallback > 0) at a finite LL equal to the restatement's, and the exact
    M-step walks its pruned records (HaploBuilder.cpp:291-314): the table
    equals the restatement's bit for bit."""
    p = synth.founder_mosaic(60, 1600, A=2, seed=1)
    oracle_mod.set_threads(16)
    try:
        o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
        o.find_patterns()
        ll_o = o.resolve_all()
        _, gp = o.estep_summary()
        sk = o.skip_counts()
        assert np.isfinite(ll_o) and np.all(gp > 0) and np.any(sk > 0)
        P_o, _ = o.estimate_patterns()
        po = o.patterns()
    finally:
        oracle_mod.set_threads(1)
    m = gpu_model(p)
    m.exact_estimate = True
    m.find_patterns()
    ll_g, H, re = m.resolve_all()
    assert ll_g == ll_o and m.estep_split_stats()["n_fallback"] > 0
    P_g, _ = m.find_patterns()
    assert m.exact_stats()["pruned"] > 0
    pg = m.patterns()
    assert P_g == P_o
    _assert_table_bits(pg, po)


def test_exact_single_allele_frequencies(oracle_mod):
    """Known answer: with nothing missing, every phasing carries the same
    alleles, so the exact frequency of a length-1 pattern is the allele
    frequency (2 n_aa + n_ab) / 2N of its locus."""
    p = panel("a4")
    m = gpu_model(p)
    m.exact_estimate = True
    m.find_patterns()
    m.resolve_all()
    m.find_patterns()
    pt = m.patterns()
    num, sym, fr = m.allele_table()
    one = np.where(pt["len"] == 1)[0]
    assert len(one) > 0
    for i in one:
        k = pt["start"][i]
        j = list(sym[k]).index(pt["alleles"][i, 0])
        assert abs(pt["freq"][i] - fr[k, j]) <= 1e-12
        assert pt["prefix"][i] == 1.0


@pytest.mark.parametrize("K,N,L,num", [(2, 40, 30, 150), (3, 50, 40, 400)])
def test_exact_mstep_after_find_pattern_by_num(oracle_mod, K, N, L, num):
    """--exact-estimate with num_patterns > 0: M0 by findPatternByNum, E1,
    then estimatePatterns at the search's last threshold (m_min_freq,
    PatternManager.cpp:53-60, 364-408) — the restatement's table bit for bit
    — and the whole EM (LL and resolutions bit for bit)."""
    p = synth.founder_mosaic(N, L, A=2, K=K, seed=5)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10)
    o.set_num_patterns(num)
    o.find_patterns()
    o.resolve_all()
    P_o, _ = o.estimate_patterns()
    po = o.patterns()
    m = gpu_model(p, num_patterns=num)
    m.exact_estimate = True
    m.find_patterns()
    m.resolve_all()
    P_g, _ = m.find_patterns()
    pg = m.patterns()
    assert P_g == P_o
    _assert_table_bits(pg, po)
    m2 = gpu_model(p, max_iteration=6, num_patterns=num)
    m2.exact_estimate = True
    res = m2.run()
    o2 = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=6)
    o2.set_num_patterns(num)
    o2.set_exact(True)
    r = o2.run()
    assert m2.iterations == r["iterations"]
    assert [x["ll"] for x in m2.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])


@pytest.mark.parametrize("name", ["cfg1", "n60", "miss2"])
def test_exact_em_against_oracle(oracle_mod, name):
    """HaploModel::run with --exact-estimate: iteration count, every
    iteration's LL and the accepted pairs, bit for bit (the restatement walks
    in the device walk's order, _assert_table_bits)."""
    p = panel(name)
    m = gpu_model(p, max_iteration=10)
    m.exact_estimate = True
    res = m.run()
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=10)
    o.set_exact(True)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(res, r["resolutions"])


def test_exact_em_estep_after_store_shrink(oracle_mod):
    """The E-step after an exact M-step (HaploModel.cpp:139-145) when HBM is
    shorter than the stores the first E-step grew (cfg 3's OOM in round 3):
    budgets cut to about an eighth of E1's trace make the stores give way to
    the pass scratch and the E-step run in groups; E2 equals the run with
    automatic budgets bit for bit (LL, R_E, totals, resolutions)."""
    p = panel("n60")
    runs = []
    for shrink in (False, True):
        m = gpu_model(p)
        m.exact_estimate = True
        m.find_patterns()
        ll1, H1, re1 = m.resolve_all()
        m.find_patterns()  # estimatePatterns
        if shrink:
            m.set_store_budgets(trace_bytes=max(1 << 16, re1 // 2), record_bytes=max(1 << 16, re1 // 2))
        ll, H, re = m.resolve_all()
        st = m.estep_split_stats()
        runs.append((float(ll).hex(), H, re, m.estep_results()["total"].copy(), m.resolutions().copy(), st))
        m.close()
    (a, b) = runs
    assert b[5]["structure_passes"] + b[5]["value_passes"] > a[5]["structure_passes"] + a[5]["value_passes"], (a[5], b[5])
    assert a[:3] == b[:3]
    assert np.array_equal(a[3], b[3]) and np.array_equal(a[4], b[4])


# ------------------------------------------------ full-size chain digests
def _sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a, dt).tobytes()).hexdigest()


def _total_weight(m):
    import ctypes as C
    tw = C.c_double()
    assert hmc_amd.lib().hmc_get_samples(m._h, None, None, C.byref(tw)) == 0
    return tw.value


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cfg", [2, 5, 3])
def test_full_size_chain_against_oracle_digest(cfg):
    """BASELINE configs 3 (10 000 x 2 000) and 5 (10 000 x 1 000, 8 alleles)
    at full size against the restatement's digests
    (tests/golden/cfg{3,5}_chain_digest.json, make_full_digest.py): the EM
    chain M0, E1, M1, E2, M2, E3 that bench.py times — every pattern table
    (SHA-256 of ids' start, length, frequency, prefix, tp, successors), R_M,
    and per E-step the LL, R_E, samples, total weight, and SHA-256 of the
    per-individual totals, candidate counts and selected pairs.  Tolerance 0."""
    path = os.path.join(HERE, "golden", f"cfg{cfg}_chain_digest.json")
    if not os.path.exists(path):
        pytest.skip(f"{path} not generated")
    d = json.load(open(path))
    p = synth.config_panel(cfg)
    assert (p.N, p.L) == (d["N"], d["L"])
    m = gpu_model(p)

    def check_m(k):
        P, rm = m.find_patterns()
        want = d["m"][k]
        assert (P, rm) == (want["P"], want["R_M"]), (k, P, rm)
        assert _digest_patterns(m.patterns(maxlen=1)) == want["table_sha256"], k

    def check_e(k):
        ll, H, re = m.resolve_all()
        want = d["e"][k - 1]
        assert (float(ll).hex(), re, H) == (want["ll_hex"], want["R_E"], want["H"]), k
        assert float(_total_weight(m)).hex() == want["total_weight_hex"]
        er = m.estep_results()
        assert _sha(er["total"], np.float64) == want["totals_sha256"], k
        assert _sha(er["ncand"], np.int32) == want["ncand_sha256"], k
        assert [float(er["total"][i]).hex() for i in want["subset"]] == want["subset_totals_hex"]
        assert _sha(m.resolutions(), np.int32) == want["resolutions_sha256"], k

    check_m(0)
    for k in range(1, len(d["e"]) + 1):
        check_e(k)
        if k < len(d["m"]):
            check_m(k)


def _estep_properties(m, p, ll, H):
    """Samples phase the genotypes (both haplotypes of each candidate, every
    non-missing locus), candidates' priors are sorted, each individual's
    weights sum to 1, total weight = 2N — vectorised over all candidates."""
    er = m.estep_results()
    n = er["ncand"]
    assert np.all(n > 0) and np.isfinite(ll) and ll < 0
    S = er["prior"].shape[1]
    live = np.arange(S)[None, :] < n[:, None]
    pr = np.where(live, er["prior"], -np.inf)
    assert np.all(np.diff(pr, axis=1)[live[:, 1:]] <= 0)
    assert np.all(np.abs(np.where(live, er["weight"], 0.0).sum(axis=1) - 1.0) < 1e-12)
    al, w, tw = m.samples(H)
    assert H == 2 * int(n.sum()) and abs(tw - 2 * p.N) < 1e-6
    owner = np.repeat(np.arange(p.N), n)  # individual of each candidate (samples in individual order)
    h0, h1 = al[0::2], al[1::2]
    g0, g1 = p.alleles[owner, 0], p.alleles[owner, 1]
    ok = ((h0 == g0) & (h1 == g1)) | ((h0 == g1) & (h1 == g0))
    assert ok.all()


def _table_properties(m, L):
    pt = m.patterns(maxlen=1)
    assert np.all(pt["freq"] > 0) and np.all(pt["freq"] <= 1) and np.all(pt["tp"] <= 1)
    e = pt["start"] + pt["len"]
    assert np.all(pt["len"] >= 1) and np.all(e <= L)
    s = pt["succ"]
    has = s >= 0
    rows = np.nonzero(has)[0]
    assert np.all(e[s[has]] == e[rows] + 1)  # a successor ends one locus further
    return _digest_patterns(pt)


@pytest.mark.timeout(1100)
def test_cfg4_rank_slice_properties():
    """cfg 4's per-rank workload (6 250 x 5 000, seed 4: one GPU's share of the
    8-GPU run): M0 mined in blocks of start loci (the automatic width: several
    blocks here) equals M0 mined in one block (pattern count, R_M and table
    digest); E1, M1 and E2 keep the full-size properties (samples phase the
    genotypes, weights sum to 1, priors sorted, frequencies in (0, 1],
    successors end one locus further); a fresh context repeats M0 and E1 bit
    for bit (table digest, LL, R_E, resolutions)."""
    p = synth.founder_mosaic(6250, 5000, A=2, seed=4)
    one = gpu_model(p)
    one.set_mine_block(p.L)
    P1, rm1 = one.find_patterns()
    assert one.mine_stats()["blocks"] == 1
    d1 = _digest_patterns(one.patterns(maxlen=1))
    one.close()

    m = gpu_model(p)
    P, rm = m.find_patterns()
    st = m.mine_stats()
    assert st["blocks"] >= 2, st
    assert (P, rm) == (P1, rm1)
    d0 = _table_properties(m, p.L)
    assert d0 == d1
    ll1, H1, re1 = m.resolve_all()
    _estep_properties(m, p, ll1, H1)
    res1 = m.resolutions()
    m.find_patterns()
    _table_properties(m, p.L)
    ll2, H2, _ = m.resolve_all()
    _estep_properties(m, p, ll2, H2)
    m.close()

    r = gpu_model(p)
    assert r.find_patterns() == (P, rm)
    assert _digest_patterns(r.patterns(maxlen=1)) == d0
    ll, H, re = r.resolve_all()
    assert (float(ll).hex(), H, re) == (float(ll1).hex(), H1, re1)
    assert np.array_equal(r.resolutions(), res1)
    r.close()
