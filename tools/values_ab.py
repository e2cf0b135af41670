"""A/B of value-pass builds and shapes at cfg 3: M0, E1, M1, then the E-step
with the M1 model repeated (runs after the first use exact region sizes, one
group).  Pick the library with HMC_AMD_LIB and the value-pass shape with
HMC_VP_SHAPE ("nw:ipc"); LL and R_E must not change."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "run"
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(synth.config_panel(int(os.environ.get("CFG", "3")))))
m.find_patterns()
m.resolve_all()
m.find_patterns()
for r in range(4):
    ll, H, re = m.resolve_all()
    s = m.estep_split_stats()
    print(f"{tag} run {r}: structure {s['structure_ms']:.1f} ms values {s['values_ms']:.1f} ms "
          f"({s['value_passes']} passes) ll={ll!r} re={re}", flush=True)
