"""HaploFile formats besides PHASE (HaploFile.cpp:205-640) through the C-ABI:
hmc_parse_file needs no device, so the readers are checked here on the CPU
against panels worked out by hand from the reference's parsing rules; the
writers are checked by a GPU round trip (load -> EM -> write -> parse)."""
import ctypes as C

import numpy as np
import pytest

import hmc_amd
from hmc_amd import synth


def parse(fmt, path, path2=None):
    L = hmc_amd.lib()
    n, l = C.c_int(), C.c_int()
    p2 = path2.encode() if path2 else None
    rc = L.hmc_parse_file(fmt.encode(), path.encode(), p2, C.byref(n), C.byref(l), None, None)
    if rc:
        return None
    al = np.zeros((n.value, 2, l.value), np.int32)
    ty = C.create_string_buffer(l.value + 1)
    rc = L.hmc_parse_file(fmt.encode(), path.encode(), p2, None, None, al.ctypes.data_as(C.POINTER(C.c_int32)), ty)
    assert rc == 0
    return al, ty.value.decode()


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return str(p)


def test_hpm_reader(tmp_path):
    # HPM: integer alleles, 0 = missing; loci with <= 2 alleles become 'S'
    # loci with 1..9 -> '1'..'9' (HaploFile.cpp:238-247, 253-257); a Status
    # column before the markers is skipped (checkHeader, :345-387)
    f = write(tmp_path, "a.hpm", "Id\tStatus\tM1 M2 M3\n"
                                 "ind1\t0\t1 2 3\n"
                                 "ind1\t0\t2 2 1\n"
                                 "ind2\t1\t0 1 12\n"
                                 "ind2\t1\t1 2 12\n")
    al, ty = parse("HPM", f)
    assert ty == "SSM"
    o1, o2 = ord("1"), ord("2")
    assert al.tolist() == [[[o1, o2, 3], [o2, o2, 1]], [[-1, o1, 12], [o1, o2, 12]]]


def test_hpm2_reader(tmp_path):
    # HPM2: one character per allele, '0' = missing, letters = 10.. (:389-416)
    f = write(tmp_path, "a.hpm2", "Id M1 M2 M3\n"
                                  "x\t1 A 1\n"
                                  "x\t2 0 3\n"
                                  "y\t2 A 4\n"
                                  "y\t1 A 2\n")
    al, ty = parse("HPM2", f)
    assert ty == "SSM"
    o = ord
    assert al.tolist() == [[[o("1"), o("A"), 1], [o("2"), -1, 3]], [[o("2"), o("A"), 4], [o("1"), o("A"), 2]]]


def test_bench2_reader(tmp_path):
    # BENCH: L characters per haplotype, '0' missing, '9' = heterozygous
    # placeholder -> '1' on the first haplotype of a pair and '2' on the second
    # (readHaplotype, :605-624); then "number 0 id" (:528-564)
    g = write(tmp_path, "g.txt", "1290   0 0 fam1\n2190   1 0 fam1\n1111   2 0 fam2\n2221   3 0 fam2\n")
    p = write(tmp_path, "p.txt", " 0   rs1   100\n 1   rs2   250\n 2   rs3   400\n 3   rs4   900\n")
    al, ty = parse("BENCH2", g, p)
    assert ty == "SSSS"
    o = ord
    assert al.tolist() == [[[o("1"), o("2"), o("1"), -1], [o("2"), o("1"), o("2"), -1]],
                           [[o("1"), o("1"), o("1"), o("1")], [o("2"), o("2"), o("2"), o("1")]]]


def parse_files(fmt, paths):
    L = hmc_amd.lib()
    arr = (C.c_char_p * len(paths))(*[x.encode() for x in paths])
    n, l, u = C.c_int(), C.c_int(), C.c_int()
    if L.hmc_parse_files(fmt.encode(), arr, len(paths), C.byref(n), C.byref(l), None, None, C.byref(u)):
        return None
    al = np.zeros((n.value, 2, l.value), np.int32)
    ty = C.create_string_buffer(l.value + 1)
    assert L.hmc_parse_files(fmt.encode(), arr, len(paths), None, None, al.ctypes.data_as(C.POINTER(C.c_int32)),
                             ty, None) == 0
    return al, ty.value.decode(), u.value


def test_bench3_reader(tmp_path):
    # BENCH3 = BENCH2 + a children file read the same way and appended as
    # ordinary genotypes (HaploFile.cpp:446-484): the heterozygous placeholder
    # restarts at '1' in the children file, unphased_num = the parents (:475)
    g = write(tmp_path, "g.txt", "129   0 0 p1\n219   1 0 p1\n")
    p = write(tmp_path, "p.txt", " 0 rs1 10\n 1 rs2 20\n 2 rs3 30\n")
    c = write(tmp_path, "c.txt", "912   2 0 c1\n902   3 0 c1\n111   4 0 c2\n221   5 0 c2\n")
    al, ty, unph = parse_files("BENCH3", [g, p, c])
    o = ord
    assert ty == "SSS" and unph == 1 and al.shape == (3, 2, 3)
    assert al.tolist() == [[[o("1"), o("2"), o("1")], [o("2"), o("1"), o("2")]],
                           [[o("1"), o("1"), o("2")], [o("2"), -1, o("2")]],
                           [[o("1"), o("1"), o("1")], [o("2"), o("2"), o("1")]]]
    # BENCH2 of the same genotype file: every genotype unphased
    assert parse_files("BENCH2", [g, p])[2] == 1
    assert parse_files("BENCH3", [g, p]) is None  # needs the children file


def test_phase_reader_via_files(tmp_path):
    # PHASE through the multi-file seam: P line, ids, 'S' and 'M' loci
    f = write(tmp_path, "a.inp", "2\n3\nP 100 250 400\nSSM\nfam1\n1 2 12\n2 2 3\n#7\n? 1 -\n1 1 4\n")
    al, ty, unph = parse_files("PHASE", [f])
    o = ord
    assert ty == "SSM" and unph == 2
    assert al.tolist() == [[[o("1"), o("2"), 12], [o("2"), o("2"), 3]], [[-1, o("1"), -1], [o("1"), o("1"), 4]]]


def test_reader_errors(tmp_path):
    odd = write(tmp_path, "odd.hpm", "Id M1\nx\t1\ny\t2\nz\t1\n")
    assert parse("HPM", odd) is None  # "Incorrect haplotype data"
    bad = write(tmp_path, "bad.hpm", "Name M1\nx\t1\nx\t2\n")
    assert parse("HPM", bad) is None  # "Not a valid HPM file!"
    assert parse("BENCH9", bad) is None  # unknown format
    assert parse("HPM", str(tmp_path / "missing.hpm")) is None


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["HPM", "HPM2", "BENCH2"])
def test_write_read_round_trip(tmp_path, fmt):
    """Load a panel from the format, run the EM, write the accepted
    resolutions in the same format and parse them back."""
    p = synth.founder_mosaic(40, 30, A=2, seed=9)
    sym = p.alleles  # '1'/'2' characters
    lines_hpm = ["Id\t" + " ".join(f"M{k + 1}" for k in range(p.L))]
    lines_bench = []
    for i in range(p.N):
        for h in range(2):
            s = "".join(chr(a) for a in sym[i, h])
            lines_hpm.append(f"i{i}\t" + " ".join(s))
            lines_bench.append(f"{s}   {2 * i + h} 0 i{i}")
    if fmt == "BENCH2":
        src = write(tmp_path, "in.txt", "\n".join(lines_bench) + "\n")
        src2 = write(tmp_path, "in.pos", "".join(f" {k}   rs{k}   {10 * k}\n" for k in range(p.L)))
    else:
        src = write(tmp_path, "in.hpm", "\n".join(lines_hpm) + "\n")
        src2 = None
    m = hmc_amd.HaploModel()
    m.max_iteration = 5
    L = hmc_amd.lib()
    assert L.hmc_load_file(m._h, fmt.encode(), src.encode(), src2.encode() if src2 else None) == 0
    m._info()
    res = m.run()  # [N][2][L] symbols
    out = str(tmp_path / "out.txt")
    out2 = str(tmp_path / "out.pos") if fmt == "BENCH2" else None
    assert L.hmc_write_file(m._h, fmt.encode(), out.encode(), out2.encode() if out2 else None) == 0
    al, ty = parse(fmt, out, out2)
    assert np.array_equal(al, res)
    if fmt == "BENCH2":
        assert open(out2).read().splitlines()[3].split() == ["3", "rs3", "30"]


@pytest.mark.gpu
@pytest.mark.parametrize("block", [0, 3])
def test_write_patterns(tmp_path, block):
    """writePattern (.patterns): one line per pattern in id order with freq/N,
    the length and the long-format alleles; checked against the table.
    block = 3: the search runs in blocks of 3 start loci, which leaves no
    complete candidate tree — the strings come from the prefix ids."""
    p = synth.founder_mosaic(30, 20, A=2, seed=3)
    m = hmc_amd.HaploModel()
    m.load(hmc_amd.GenoData.from_panel(p))
    if block:
        m.set_mine_block(block)
    m.find_patterns()
    if block:
        assert m.mine_stats()["blocks"] > 1
    out = str(tmp_path / "x.patterns")
    assert hmc_amd.lib().hmc_write_patterns(m._h, out.encode()) == 0
    pt = m.patterns()
    lines = open(out).read().splitlines()
    assert lines[0].split("\t")[:2] == ["Frequency", "Length"]
    assert len(lines) == 1 + len(pt["start"])
    for i in list(range(0, len(lines) - 1, max(1, len(lines) // 40))) + [len(lines) - 2]:
        f, ln, al = lines[i + 1].split("\t")
        assert float(f) == pytest.approx(pt["freq"][i] / p.N, abs=5e-7) and int(ln) == pt["len"][i]
        v = [int(x) for x in al.split()]
        s, n = pt["start"][i], pt["len"][i]
        assert len(v) == p.L and v[:s] == [-1] * s and v[s + n:] == [-1] * (p.L - s - n)
        assert v[s:s + n] == pt["alleles"][i, :n].tolist()


@pytest.mark.gpu
def test_bench3_em_against_oracle(tmp_path, oracle_mod):
    """BENCH3: parents + children resolved together (children are ordinary
    unphased genotypes, Genotype.cpp:40), HaploComp over the parents only
    (HaploComp.cpp:40): per-iteration LL, HaploComp triple and accepted pairs
    equal the restatement's."""
    p = synth.founder_mosaic(50, 40, A=2, seed=11)
    sym = p.alleles
    par, kid = [], []
    for i in range(p.N):
        for h in range(2):
            line = "".join(chr(a) for a in sym[i, h]) + f"   {2 * i + h} 0 i{i}"
            (par if i < 30 else kid).append(line)
    g = write(tmp_path, "g.txt", "\n".join(par) + "\n")
    c = write(tmp_path, "c.txt", "\n".join(kid) + "\n")
    pos = write(tmp_path, "p.txt", "".join(f" {k} rs{k} {7 * k}\n" for k in range(p.L)))
    m = hmc_amd.HaploModel()
    m.max_iteration = 20
    m.load_files("BENCH3", [g, pos, c])
    assert m.unphased_num() == 30 and m.N == 50
    res = m.run()
    o = oracle_mod.Oracle(sym, p.types, sample_size=10, max_iter=20)
    o.set_unphased(30)
    r = o.run()
    assert m.iterations == r["iterations"]
    assert [x["ll"] for x in m.log] == r["ll"].tolist()
    assert np.array_equal(np.array([x["haplocomp"] for x in m.log]), r["haplocomp"])
    assert np.array_equal(res, r["resolutions"])
    out, outp = str(tmp_path / "o.txt"), str(tmp_path / "o.pos")
    m.write_files("BENCH3", [out, outp])
    al, _, _ = parse_files("BENCH2", [out, outp])
    assert np.array_equal(al, res)
    assert open(outp).read().splitlines()[2] == " 2   rs2   14"


@pytest.mark.gpu
def test_write_phase_text(tmp_path, oracle_mod):
    """writeGenoData (HaploFile.cpp:120-153) text: the input's P line and ids
    ('#' only before an id that starts with a digit), the type line and one
    "a a a " line per haplotype, checked against text built from the
    restatement's accepted pairs."""
    p = synth.founder_mosaic(6, 12, A=2, seed=4)
    ids = ["fam1", "#2", "33", "x-4", "5b", "#six"]
    pos = [100 + 37 * k for k in range(p.L)]
    lines = [str(p.N), str(p.L), "P " + " ".join(map(str, pos)), p.types]
    for i in range(p.N):
        lines.append(ids[i] + "  trailing")
        for h in range(2):
            lines.append(" ".join(chr(a) for a in p.alleles[i, h]))
    src = write(tmp_path, "in.inp", "\n".join(lines) + "\n")
    m = hmc_amd.HaploModel()
    m.max_iteration = 10
    m.load_phase(src)
    m.run()
    o = oracle_mod.Oracle(phase_path=src, sample_size=10, max_iter=10)
    r = o.run()
    best = r["resolutions"]
    exp = [str(p.N), str(p.L), "P " + " ".join(map(str, pos)), p.types]
    for i in range(p.N):
        exp.append(("#" if ids[i][0].isdigit() else "") + ids[i])
        for h in range(2):
            exp.append("".join(chr(a) + " " for a in best[i, h]))
    out = str(tmp_path / "out.inp")
    m.write_phase(out)
    assert open(out).read() == "\n".join(exp) + "\n"
