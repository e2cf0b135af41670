"""cfg 4's M0 (50 000 x 5 000, seed 4) mined on one GPU over every
individual, in blocks of start loci (the automatic block width): the global
pattern count, the candidate-node window and the time — the replicated part
of each rank's memory in the 8-GPU run.  HMC_DEBUG_MEM=1 prints
every block.

    python tools/cfg4_m0.py [BLOCK_WIDTH]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

t0 = time.perf_counter()
p = synth.config_panel(4)
print(f"panel {p.N} x {p.L} built in {time.perf_counter() - t0:.0f} s", flush=True)
m = hmc_amd.HaploModel()
if len(sys.argv) > 1:
    m.set_mine_block(int(sys.argv[1]))
m.load(hmc_amd.GenoData.from_panel(p))
t0 = time.perf_counter()
P, rm = m.find_patterns()
wall = time.perf_counter() - t0
st = m.mine_stats()
print(f"cfg4 M0: {P} patterns, R_M {rm}, {wall:.1f} s wall, {m.timings()['mstep_ms']:.0f} ms device; "
      f"{st['blocks']} blocks, {st['nodes']} candidate nodes, node window {st['node_window_gb']:.1f} GB", flush=True)
m.close()
