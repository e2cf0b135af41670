"""Diagnostic build: block-critical-path cycles per phase of the split E-step's
value pass (estep_values), averaged per individual-locus, for E1..E3 of a
BASELINE config (env CFG, default 2; ITERS E-steps, default 3)."""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["HMC_AMD_LIB"] = os.path.join(ROOT, "hmc_amd", "libhmc_amd_diag.so")
sys.path.insert(0, ROOT)
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

p = synth.config_panel(int(os.environ.get("CFG", "2")))
m = hmc_amd.HaploModel()
nw, ipc = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "0:0").split(":"))
m.set_pass_shapes(0, 0, nw, ipc)  # value-pass shape (0 = automatic)
m.load(hmc_amd.GenoData.from_panel(p))
m.find_patterns()
names = ["record hdr", "phase A", "phase B", "trace", "final sync", "final select"]
for it in range(int(os.environ.get("ITERS", "3"))):
    ll, H, re = m.resolve_all()
    print(f"  R_E {re}", flush=True)
    st = (C.c_uint64 * 40)()
    hmc_amd.lib().hmc_get_stamps(m._h, st)
    s = m.estep_split_stats()
    print(f"  passes: structure {s['structure_passes']} value {s['value_passes']}", flush=True)
    nl = p.N * (p.L - 1)
    tot = sum(st[:6])
    print(f"E{it + 1}: structure {s['structure_ms']:.2f} ms values {s['values_ms']:.2f} ms; "
          f"mean per individual-locus cycles (thread 0):")
    for k in range(6):
        print(f"   {names[k]:14s} {st[k] / nl:9.0f}  {100 * st[k] / max(tot, 1):5.1f}%")
    print(f"   states past the LDS tier (frontier HBM-tier writes) {st[7] / nl:.1f} per locus of {st[9] / nl:.1f}; "
          f"loci {st[11]}; R_E {m.last_re if hasattr(m, 'last_re') else 'see log'}")
    print(f"   chains/locus {st[8] / nl:.1f}  states/locus {st[9] / nl:.1f}  "
          f"wave-0 chain steps/locus {st[10] / nl:.2f}  critical-path steps/locus {st[12] / nl:.2f}  "
          f"phase-B cycles per critical step {st[2] / max(st[12], 1):.0f}")
    print(f"   wave 0 per chain step: selection {st[13] / max(st[10], 1):.0f} cycles, "
          f"rest (pop/loads/transform/store) {st[14] / max(st[10], 1):.0f} cycles")
    m.find_patterns()
