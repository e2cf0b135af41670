"""The C++ host driver tools/hmc_resolve (HMC's resolve mode, HMC.cpp:179-233,
on the C-ABI): run as a separate program on PHASE and BENCH3 inputs; its
<input>.reconstructed is compared with text built from the CPU restatement's
accepted pairs in the writeGenoData layout (HaploFile.cpp:120-153), and its
per-iteration log lines with the restatement's HaploComp / LL."""
import os
import re
import subprocess

import numpy as np
import pytest

import hmc_amd
from hmc_amd import synth

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "tools", "hmc_resolve")


def run_cli(*args):
    r = subprocess.run([CLI, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    return r.stdout


def write_phase(path, p, ids, pos):
    lines = [str(p.N), str(p.L), "P " + " ".join(map(str, pos)), p.types]
    for i in range(p.N):
        lines.append(ids[i])
        for h in range(2):
            lines.append(" ".join(chr(a) for a in p.alleles[i, h]))
    path.write_text("\n".join(lines) + "\n")


def log_lines(out):
    rx = re.compile(r"Switch Error = ([-\d.naninf]+), IHP = ([-\d.naninf]+), IGP = ([-\d.naninf]+), LL = ([-\d.]+)")
    return [tuple(float(x) for x in m.groups()) for m in rx.finditer(out)]


def test_cli_phase_reconstructed_text(tmp_path, oracle_mod):
    p = synth.founder_mosaic(40, 30, A=2, seed=12)
    ids = [f"ind{i}" if i % 3 else f"{100 + i}" for i in range(p.N)]
    pos = [17 + 123 * k for k in range(p.L)]
    src = tmp_path / "in.inp"
    write_phase(src, p, ids, pos)
    out = run_cli("-i", "10", "--output-patterns", "x", str(src))
    r = oracle_mod.Oracle(phase_path=str(src), sample_size=10, max_iter=10).run()
    got = log_lines(out)
    assert len(got) == r["iterations"]
    for (se, ihp, igp, ll), comp, llo in zip(got, r["haplocomp"], r["ll"]):
        assert (se, ihp, igp) == tuple(float(f"{x:f}") for x in comp) and ll == float(f"{llo:f}")
    best = r["resolutions"]
    exp = [str(p.N), str(p.L), "P " + " ".join(map(str, pos)), p.types]
    for i in range(p.N):
        exp.append(("#" if ids[i][0].isdigit() else "") + ids[i])  # HaploFile.cpp:141-147
        for h in range(2):
            exp.append("".join(chr(a) + " " for a in best[i, h]))
    assert (tmp_path / "in.inp.reconstructed").read_text() == "\n".join(exp) + "\n"
    pat = (tmp_path / "in.inp.patterns").read_text().splitlines()
    assert pat[0].startswith("Frequency\tLength\t") and len(pat) > 1


def test_cli_exact_estimate(tmp_path, oracle_mod):
    p = synth.founder_mosaic(30, 24, A=2, seed=13)
    src = tmp_path / "x.inp"
    write_phase(src, p, [f"#{i + 1}" for i in range(p.N)], [1000 * k for k in range(p.L)])
    out = run_cli("-i", "6", "--exact-estimate", str(src))
    o = oracle_mod.Oracle(phase_path=str(src), sample_size=10, max_iter=6)
    o.set_exact(True)
    r = o.run()
    got = log_lines(out)
    assert len(got) == r["iterations"]
    assert np.allclose([g[3] for g in got], r["ll"], rtol=1e-6, atol=2e-6)


def test_cli_bench3(tmp_path):
    p = synth.founder_mosaic(24, 20, A=2, seed=14)
    par, kid = [], []
    for i in range(p.N):
        for h in range(2):
            line = "".join(chr(a) for a in p.alleles[i, h]) + f"   {2 * i + h} 0 f{i // 3}"
            (par if i < 16 else kid).append(line)
    g, c, pos = tmp_path / "g.txt", tmp_path / "c.txt", tmp_path / "p.txt"
    g.write_text("\n".join(par) + "\n")
    c.write_text("\n".join(kid) + "\n")
    pos.write_text("".join(f" {k}   rs{k}   {5 * k}\n" for k in range(p.L)))
    run_cli("-f", "BENCH3", "-i", "5", str(g), str(pos), str(c))
    m = hmc_amd.HaploModel()
    m.max_iteration = 5
    m.load_files("BENCH3", [str(g), str(pos), str(c)])
    res = m.run()
    lines = (tmp_path / "g.txt.reconstructed").read_text().splitlines()
    assert len(lines) == 2 * p.N
    for i in range(p.N):
        for h in range(2):
            hap, rest = lines[2 * i + h][:p.L], lines[2 * i + h][p.L:].split()
            assert [ord(ch) for ch in hap] == res[i, h].tolist()
            assert rest == [str(2 * i + h), "0", f"f{i // 3}"]
