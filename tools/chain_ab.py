"""A/B of library builds or E-step options over a config's converged chain:
M0 once, then twice (hmc_em_rewind) E1, M1, E2, M2, E3 with device ms of
every E-step's passes.  Pick the build with HMC_AMD_LIB and the value mode
with HMC_VALUE_MODE (exact | fast: value-only k-best lists, the exact pass
re-run only for individuals with ties); LL and R_E must not change.

    HMC_AMD_LIB=... HMC_VALUE_MODE=fast python tools/chain_ab.py TAG [CFG]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 3
vmode = os.environ.get("HMC_VALUE_MODE", "exact")
m = hmc_amd.HaploModel()
m.set_value_mode(vmode)
if os.environ.get("HMC_VALUE_SHAPE") or os.environ.get("HMC_STRUCT_SHAPE"):  # "waves,individuals_per_cu"
    vw, vi = (int(x) for x in os.environ.get("HMC_VALUE_SHAPE", "0,0").split(","))
    sw, si = (int(x) for x in os.environ.get("HMC_STRUCT_SHAPE", "0,0").split(","))
    m.set_pass_shapes(sw, si, vw, vi)
    tag += f"/vshape{vw}x{vi}/sshape{sw}x{si}"
if os.environ.get("HMC_VALUE_LAYOUT"):  # 0 one link per lane, 1 two for heavy groups, 2 two everywhere
    m.set_value_layout(int(os.environ["HMC_VALUE_LAYOUT"]))
    tag += f"/layout{os.environ['HMC_VALUE_LAYOUT']}"
if os.environ.get("HMC_S1_TIER"):  # "key_mult10,contrib_mult10"
    km, cm = (int(x) for x in os.environ["HMC_S1_TIER"].split(","))
    m.set_structure_tier(km, cm)
    tag += f"/tier{km},{cm}"
if os.environ.get("HMC_KEY_PROBES"):
    m.set_key_probes(int(os.environ["HMC_KEY_PROBES"]))
    tag += f"/probes{os.environ['HMC_KEY_PROBES']}"
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(cfg)))
t0 = time.perf_counter()
P, _ = m.find_patterns()
print(f"{tag}: cfg {cfg} value mode {vmode}: M0 {P} patterns {time.perf_counter() - t0:.1f} s "
      f"lib {hmc_amd.lib_identity()}", flush=True)
m.model_save()
n = m.i1 - m.i0
for rep in range(2):
    m.em_rewind()
    for k in range(1, 4):
        t0 = time.perf_counter()
        ll, H, re = m.resolve_all()
        wall = time.perf_counter() - t0
        s = m.estep_split_stats()
        print(f"{tag} chain {rep} E{k}: wall {wall * 1e3:.0f} ms structure {s['structure_ms']:.0f} ms "
              f"({s['structure_passes']}) values {s['values_ms']:.0f} ms ({s['value_passes']}) "
              f"order re-runs {s['n_order_rerun']} of {n} ({s['order_ms']:.0f} ms) "
              f"ll={ll!r} R_E={re}", flush=True)
        if k < 3:
            m.find_patterns()
