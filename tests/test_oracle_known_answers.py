"""Known-answer tests for the CPU restatement, derived by hand from the
reference source (no reference build exists here: parity unpinned, see
DESIGN.md §Oracle).  The expected values below are worked out step by step
from PatternManager.cpp:100-144/267-291/293-318 and HaploBuilder.cpp:35-126 for
a 2-individual x 2-locus panel, with every floating-point operation written in
the reference's order."""
import math

import numpy as np

ONE, TWO = ord("1"), ord("2")


def tiny_panel():
    # individual A: 11 / 11 (homozygous); individual B: 12 / 21 (het at both loci)
    a = np.array([[[ONE, ONE], [ONE, ONE]], [[ONE, TWO], [TWO, ONE]]], np.int32)
    return a


def test_allele_tables(oracle_mod):
    o = oracle_mod.Oracle(tiny_panel(), "SS")
    num, sym, fr = o.allele_table()
    assert num.tolist() == [2, 2]
    assert sym.tolist() == [[ONE, TWO], [ONE, TWO]]
    assert fr.tolist() == [[0.75, 0.25], [0.75, 0.25]]  # GenoData.cpp:101-117: count / non-missing


def test_m0_pattern_table(oracle_mod):
    o = oracle_mod.Oracle(tiny_panel(), "SS")
    assert o.find_patterns() == 5
    pt = o.patterns()
    # DFS pre-order: start 1 first, descending allele index (PatternManager.cpp:94-97,112-113)
    assert pt["start"].tolist() == [1, 1, 0, 0, 0]
    assert pt["len"].tolist() == [1, 1, 1, 1, 2]
    assert pt["alleles"][:, 0].tolist() == [TWO, ONE, TWO, ONE, ONE]
    assert pt["alleles"][4, :2].tolist() == [ONE, ONE]
    # genotype-branch frequencies (getMatchingFrequency, PatternManager.cpp:267-291), N = 2
    f11 = (1.0 * (0.5 * 2.0) * (1.0 * (0.5 * 2.0)) + (1.0 * (0.5 * 1.0)) * (1.0 * (0.5 * 1.0))) / 2
    assert pt["freq"].tolist() == [0.25, 0.75, 0.25, 0.75, f11]
    assert pt["prefix"].tolist() == [1.0, 1.0, 1.0, 1.0, 0.75]
    assert pt["tp"].tolist() == [0.25, 0.75, 0.25, 0.75, f11 / 0.75]
    # "12" starting at 0 has frequency 0.125 < min_freq 1.5/4 and is rejected;
    # successors = longest stored suffix (PatternManager.cpp:308-317)
    assert pt["succ"].tolist() == [[-1, -1], [-1, -1], [1, 0], [4, 0], [-1, -1]]


def test_e1_known_answer(oracle_mod):
    o = oracle_mod.Oracle(tiny_panel(), "SS", sample_size=10)
    o.find_patterns()
    ll = o.resolve_all()
    tp4 = 0.625 / 0.75
    # A: head pair (P3,P3) homozygous, extended to (P4,P4)
    fwd_a = (0.75 * 0.75) * (tp4 * tp4)
    # B: head pair (P2,P3): fwd doubled; extensions (0,4) and reversed (1,0)->(0,1)
    head_b = 0.25 * 0.75
    fwd_b0 = (head_b * 2.0) * (0.25 * tp4)
    fwd_b1 = (head_b * 2.0) * (0.25 * 0.75)
    total_b = fwd_b0 + fwd_b1
    nc, gp = o.estep_summary()
    assert nc.tolist() == [1, 2]
    assert gp.tolist() == [fwd_a, total_b]
    assert ll == math.log(fwd_a) + math.log(total_b)
    hap, prior, post = o.candidate(1, 0)
    assert hap.tolist() == [[TWO, TWO], [ONE, ONE]]
    assert prior == (head_b * (0.25 * tp4)) * 2.0
    hap, prior1, _ = o.candidate(1, 1)
    assert hap.tolist() == [[ONE, TWO], [TWO, ONE]]  # reversed link swaps the roles
    assert prior1 == (head_b * (0.25 * 0.75)) * 2.0
    hap, prior_a, post_a = o.candidate(0, 0)
    assert hap.tolist() == [[ONE, ONE], [ONE, ONE]] and prior_a == fwd_a and post_a == 1.0
    al, w, tw = o.samples()
    assert al.shape == (6, 2)
    p0, p1 = prior / total_b, prior1 / total_b
    cov = p0 + p1
    assert w.tolist() == [1.0, 1.0, p0 / cov, p0 / cov, p1 / cov, p1 / cov]
    assert tw == ((((1.0 + 1.0) + p0 / cov) + p0 / cov) + p1 / cov) + p1 / cov
    # the selected pair is the first candidate (HaploBuilder.cpp:115)
    assert o.resolutions()[1].tolist() == [[TWO, TWO], [ONE, ONE]]


def test_m1_from_samples(oracle_mod):
    o = oracle_mod.Oracle(tiny_panel(), "SS", sample_size=10)
    o.find_patterns()
    o.resolve_all()
    al, w, tw = o.samples()
    o.find_patterns()
    pt = o.patterns()
    # sample-branch frequency = ordered sum of matching weights / total weight
    for i in range(len(pt["start"])):
        s, l = pt["start"][i], pt["len"][i]
        m = np.all(al[:, s:s + l] == pt["alleles"][i, :l], axis=1)
        acc = 0.0
        for h in np.nonzero(m)[0]:
            acc += w[h]
        assert pt["freq"][i] == acc / tw


def test_missing_allele_head_quirk(oracle_mod):
    # genotype (?, 2) at locus 0 and a head '1': the complement is the missing
    # allele, which findLongestMatchPattern resolves to the first child (allele
    # index 0) of the locus-1 trie (HaploBuilder.cpp:193-201, PatternTree.cpp:102-114)
    a = np.array([[[-1, ONE], [TWO, ONE]], [[ONE, TWO], [ONE, TWO]], [[TWO, ONE], [TWO, TWO]]], np.int32)
    o = oracle_mod.Oracle(a, "SS", sample_size=4)
    o.find_patterns()
    o.resolve_all()
    nc, gp = o.estep_summary()
    assert nc[0] > 0 and gp[0] > 0


def test_haplocomp_known_answers(oracle_mod):
    """HaploComp (HaploComp.cpp:29-155, Genotype.cpp:160-266) worked by hand on
    one individual: loci (1,2) (2,1) (1,2) (2,1) (1,1) (1,2), five heterozygous."""
    A = np.array([[[49, 50, 49, 50, 49, 49], [50, 49, 50, 49, 49, 50]]], np.int32)
    o = oracle_mod.Oracle(A, "S" * 6)
    assert o.haplocomp(A).tolist() == [0.0, 0.0, 0.0]
    B = A.copy()
    B[0, :, 3:] = B[0, ::-1, 3:]  # phase flipped from locus 3 on
    # one switch over 5-1 heterozygous steps; the haplotype is wrong; the best
    # orientation mismatches loci 3 and 5 of the 6 non-missing loci
    assert o.haplocomp(B).tolist() == [0.25, 1.0, 2 / 6]
    C = A.copy()
    C[0, 0, 0] = 50  # not the input genotype: the reference exits
    assert o.haplocomp(C) is None
    # a missing allele: locus 1 leaves every count, the wildcard matches
    M = A.copy()
    M[0, 0, 1] = -1
    o2 = oracle_mod.Oracle(M, "S" * 6)
    F = A.copy()
    F[0, :, 2:] = F[0, ::-1, 2:]
    # heterozygous: loci 0,2,3,5 (locus 1 has a missing allele, which matches
    # anything); switch at locus 2; mismatches of the best orientation: locus 0
    assert o2.haplocomp(F).tolist() == [1 / 3, 1.0, 1 / 5]


def test_haplocomp_logged_per_iteration(oracle_mod):
    from hmc_amd import synth

    p = synth.founder_mosaic(40, 30, A=2, seed=4)
    o = oracle_mod.Oracle(p.alleles, p.types, sample_size=10, max_iter=5)
    r = o.run()
    assert r["haplocomp"].shape == (r["iterations"], 3)
    assert np.isfinite(r["haplocomp"]).all() and (r["haplocomp"] >= 0).all()
    np.testing.assert_array_equal(o.haplocomp(r["resolutions"]), r["haplocomp"][-1])
