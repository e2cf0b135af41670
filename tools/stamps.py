import sys, os, ctypes as C
os.environ["HMC_AMD_LIB"] = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "hmc_amd", "libhmc_amd_diag.so")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, hmc_amd
from hmc_amd import synth
names = ["pairs/loop", "decode+fwd", "succ gather", "tp/last gather", "key insert", "grouping", "cnt/state", "rounds(create/add)", "trace+clear", "final select", "-", "-"]
p = synth.config_panel(2)
wpc = int(sys.argv[1]) if len(sys.argv) > 1 else 4
m = hmc_amd.HaploModel(); m.set_estep_shape(int(os.environ.get('HMC_NW', '3')), wpc); m.load(hmc_amd.GenoData.from_panel(p)); m.find_patterns()
for it in range(2):
    ll, H, re = m.resolve_all()
    st = (C.c_uint64 * 40)()
    hmc_amd.lib().hmc_get_stamps(m._h, st)
    tot = sum(st)
    print(f"E{it+1} fwd {m.timings()['estep_forward_ms']:.1f} ms; cycles per wave-locus (divide by N_waves):")
    tot = sum(st[:10])
    for k in range(10):
        print(f"   {names[k]:22s} {st[k]/1000/500:10.0f}  {100*st[k]/tot:5.1f}%")
    na, nr, ns = max(st[10], 1), max(st[11], 1), max(st[18], 1)
    print(f"   per round: lane part {st[13]/nr:.0f} (own part per add {st[14]/na:.0f})  sync {st[16]/nr:.0f}; Y in LDS {st[17]/na:.2f}")
    print(f"   per selection step: params+load {st[15]/ns:.0f}  nth {st[19]/ns:.0f}  store {st[12]/ns:.0f};  steps per round {ns/nr:.2f}")
    print(f"   adds per wave-locus {st[10]/1000/500:.1f}; rounds per wave-locus {st[11]/1000/500:.2f}")
    m.find_patterns()
