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


def test_reader_errors(tmp_path):
    odd = write(tmp_path, "odd.hpm", "Id M1\nx\t1\ny\t2\nz\t1\n")
    assert parse("HPM", odd) is None  # "Incorrect haplotype data"
    bad = write(tmp_path, "bad.hpm", "Name M1\nx\t1\nx\t2\n")
    assert parse("HPM", bad) is None  # "Not a valid HPM file!"
    assert parse("BENCH3", bad) is None  # phased children: not on the GPU path
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
def test_write_patterns(tmp_path):
    """writePattern (.patterns): one line per pattern in id order with freq/N,
    the length and the long-format alleles; checked against the table."""
    p = synth.founder_mosaic(30, 20, A=2, seed=3)
    m = hmc_amd.HaploModel()
    m.load(hmc_amd.GenoData.from_panel(p))
    m.find_patterns()
    out = str(tmp_path / "x.patterns")
    assert hmc_amd.lib().hmc_write_patterns(m._h, out.encode()) == 0
    pt = m.patterns()
    lines = open(out).read().splitlines()
    assert lines[0].split("\t")[:2] == ["Frequency", "Length"]
    assert len(lines) == 1 + len(pt["start"])
    for i in (0, len(lines) // 2, len(lines) - 2):
        f, ln, al = lines[i + 1].split("\t")
        assert float(f) == pytest.approx(pt["freq"][i] / p.N, abs=5e-7) and int(ln) == pt["len"][i]
        v = [int(x) for x in al.split()]
        s, n = pt["start"][i], pt["len"][i]
        assert len(v) == p.L and v[:s] == [-1] * s and v[s + n:] == [-1] * (p.L - s - n)
        assert v[s:s + n] == pt["alleles"][i, :n].tolist()
