import numpy as np

from hmc_amd import synth


def test_deterministic_and_shaped():
    a = synth.founder_mosaic(50, 80, A=3, seed=7)
    b = synth.founder_mosaic(50, 80, A=3, seed=7)
    c = synth.founder_mosaic(50, 80, A=3, seed=8)
    assert a.alleles.shape == (50, 2, 80)
    assert np.array_equal(a.alleles, b.alleles)
    assert not np.array_equal(a.alleles, c.alleles)
    assert set(np.unique(a.alleles)) <= {ord("1"), ord("2"), ord("3")}


def test_missing_rate():
    p = synth.founder_mosaic(200, 200, missing=0.02, seed=3)
    r = (p.alleles < 0).mean()
    assert 0.015 < r < 0.025


def test_mosaic_has_ld():
    # short windows of a founder mosaic show about K distinct haplotypes, not 2^w
    p = synth.founder_mosaic(100, 400, A=2, K=8, seed=1, rho=0.002)
    h = p.alleles.reshape(200, 400)
    for s in (0, 150, 390):
        distinct = {tuple(r) for r in h[:, s:s + 10].tolist()}
        assert len(distinct) <= 8 + 4


def test_phase_roundtrip(tmp_path, oracle_mod):
    p = synth.founder_mosaic(12, 30, A=4, missing=0.05, seed=5)
    f = tmp_path / "p.phase"
    synth.write_phase(p, str(f))
    q = synth.read_phase(str(f))
    assert np.array_equal(p.alleles, q.alleles) and q.types == p.types
    o = oracle_mod.Oracle(phase_path=str(f))  # HaploFile::readGenoData restatement
    assert np.array_equal(o.genotypes(), p.alleles)


def test_config_table():
    assert synth.CONFIGS[2] == dict(N=1000, L=500, A=2)
    p = synth.config_panel(1)
    assert p.alleles.shape == (10, 2, 20)
