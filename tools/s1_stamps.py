"""Diagnostic build: the structure pass's phase cycles (lane 0, summed over
individuals) for E_1..E_k of a BASELINE config, per individual-locus.

    make -C hmc_amd/csrc diag && python tools/s1_stamps.py CFG ITERS
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HMC_AMD_LIB"] = os.path.join(ROOT, "hmc_amd", "libhmc_amd_diag.so")
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

cfg = int(sys.argv[1]) if len(sys.argv) > 1 else 2
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
p = synth.config_panel(cfg)
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
m.find_patterns()
names = {0: "pairs", 14: "chunk: gathers", 15: "chunk: keys+lanes", 16: "chunk: rank sync",
         17: "chunk: new-state scan", 7: "chunk: states+records", 1: "after the chunks", 18: "counts scan",
         19: "record alloc", 2: "per-state loop", 3: "chains/order", 4: "clear", 5: "head", 6: "epilogue"}
for it in range(iters):
    m.resolve_all()
    st = (C.c_uint64 * 40)()
    hmc_amd.lib().hmc_get_stamps(m._h, st)
    s1 = st[20:40]
    s = m.estep_split_stats()
    nl = max(1, s1[13])
    tot = sum(s1[:8]) + sum(s1[14:20])
    print(f"E{it + 1}: structure {s['structure_ms']:.1f} ms in {s['structure_passes']} passes; per individual-locus "
          f"(lane-0 cycles, summed over all passes):")
    for k, nm in names.items():
        print(f"   {nm:24s} {s1[k] / nl:9.0f}  {100 * s1[k] / max(tot, 1):5.1f}%")
    print(f"   C {s1[8] / nl:.1f}  F {s1[9] / nl:.1f}  chunks {s1[10] / nl:.2f}  HBM-tier keys {s1[11] / nl:.1f}  "
          f"HBM-tier states {s1[12] / nl:.1f}  loci walked {s1[13]}", flush=True)
    m.find_patterns()
