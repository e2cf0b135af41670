"""Synthetic genotype panels (founder mosaics) for tests and the benchmark.

SURVEY.md §8(d): K founders with i.i.d. uniform alleles; every haplotype starts
on a uniform founder and at each later locus switches (with probability rho) to
a uniform founder; optional per-allele missing rate.  The draws come from a
counter-based SplitMix64 stream so that any machine regenerates the identical
panel from (config, seed) without shipping data files.

The PHASE text layout written here is the one HaploFile::readGenoData parses
(HaploFile.cpp:54-118): N, L, a `P` positions line, a type line, then per
individual an id line and two allele lines.
"""
from __future__ import annotations

import dataclasses
import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def _mix64(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * _M1
    z = (z ^ (z >> np.uint64(27))) * _M2
    return z ^ (z >> np.uint64(31))


def _uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    """U[0,1) doubles for counters `idx` of (seed, stream)."""
    with np.errstate(over="ignore"):
        base = _mix64(np.array([seed * 1000003 + stream], dtype=np.uint64) * _GAMMA + _GAMMA)
        v = _mix64(base + (idx.astype(np.uint64) + np.uint64(1)) * _GAMMA)
    return (v >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


@dataclasses.dataclass
class Panel:
    """Genotype panel: alleles[N][2][L] as symbol codes (ASCII for SNP), -1 = missing."""

    alleles: np.ndarray
    types: str

    @property
    def N(self) -> int:
        return self.alleles.shape[0]

    @property
    def L(self) -> int:
        return self.alleles.shape[2]


def founder_mosaic(N: int, L: int, A: int = 2, K: int = 8, rho: float = 0.002,
                   missing: float = 0.0, seed: int = 1) -> Panel:
    if not (1 <= A <= 9):
        raise ValueError("A must be in 1..9 for single-character SNP symbols")
    H = 2 * N
    fidx = np.arange(K * L, dtype=np.uint64)
    founders = np.minimum((_uniform(seed, 1, fidx) * A).astype(np.int64), A - 1).reshape(K, L)
    hidx = np.arange(H, dtype=np.uint64) * np.uint64(L)
    cur = np.minimum((_uniform(seed, 2, hidx) * K).astype(np.int64), K - 1)
    out = np.empty((H, L), dtype=np.int32)
    out[:, 0] = founders[cur, 0]
    for l in range(1, L):
        ctr = hidx + np.uint64(l)
        sw = _uniform(seed, 3, ctr) < rho
        if sw.any():
            nf = np.minimum((_uniform(seed, 4, ctr) * K).astype(np.int64), K - 1)
            cur = np.where(sw, nf, cur)
        out[:, l] = founders[cur, l]
    sym = out + ord("1")
    if missing > 0:
        m = _uniform(seed, 5, np.arange(H * L, dtype=np.uint64)).reshape(H, L) < missing
        sym = np.where(m, -1, sym)
    return Panel(alleles=sym.reshape(N, 2, L).astype(np.int32), types="S" * L)


# BASELINE.json configs (1-5); seed = config index.
CONFIGS = {
    1: dict(N=10, L=20, A=2),
    2: dict(N=1000, L=500, A=2),
    3: dict(N=10000, L=2000, A=2),
    4: dict(N=50000, L=5000, A=2),
    5: dict(N=10000, L=1000, A=8),
}


def config_panel(cfg: int, missing: float = 0.0) -> Panel:
    c = CONFIGS[cfg]
    return founder_mosaic(c["N"], c["L"], A=c["A"], seed=cfg, missing=missing)


def write_phase(panel: Panel, path: str) -> None:
    """Write a PHASE file in the layout HaploFile::writeGenoData emits (HaploFile.cpp:120-153)."""
    N, L = panel.N, panel.L
    lines = [str(N), str(L), "P " + " ".join(str(i * 1000) for i in range(L)), panel.types]
    for i in range(N):
        lines.append(f"#{i + 1}")
        for h in range(2):
            row = panel.alleles[i, h]
            lines.append(" ".join("?" if a < 0 else chr(a) for a in row.tolist()))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def read_phase(path: str) -> Panel:
    """Parse a PHASE file with SNP ('S') loci (HaploFile.cpp:54-118 semantics)."""
    with open(path) as f:
        toks = f.read().split("\n")
    N, L = int(toks[0]), int(toks[1])
    r = 2
    if toks[r].lstrip().startswith("P"):
        r += 1
    types = "".join(toks[r].split())[:L]
    r += 1
    al = np.full((N, 2, L), -1, dtype=np.int32)
    for i in range(N):
        r += 1  # id line
        for h in range(2):
            chars = "".join(toks[r].split())
            for k in range(L):
                c = chars[k]
                al[i, h, k] = -1 if c in "?-" else ord(c)
            r += 1
    return Panel(alleles=al, types=types)
