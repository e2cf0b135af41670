"""Per-rank E-step of a sharded run, on one GPU: the value/structure pass times
of rank 0's shard of cfg 3 (hmc_shard_range's balanced cut) for world sizes W,
under each launch shape "W:I" (waves per individual : individuals per CU;
"0:0" = the library's automatic choice).  The E-step is independent per
individual given the model, so the shard is loaded as a panel of its own with
the full panel's M1 model (hmc_set_patterns): the same work rank 0 does in
E_2 of `bench.py --gpus W`.  Results must not depend on the shape.
usage: python tools/shard_shapes.py "2,4,8" 0:0 1:16 2:8 4:4 ..."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402
from hmc_amd.model import balanced_shard  # noqa: E402

worlds = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8").split(",")]
shapes = sys.argv[2:] or ["0:0", "2:8", "4:4"]
p = synth.config_panel(int(os.environ.get("CFG", "3")))
m = hmc_amd.HaploModel()
m.load(hmc_amd.GenoData.from_panel(p))
m.find_patterns()
m.resolve_all()
P, _ = m.find_patterns()
pt = m.patterns(maxlen=30)
last = pt["alleles"][np.arange(P), pt["len"] - 1].astype(np.int32)
t = time.time()
ll, H, re = m.resolve_all()
s = m.estep_split_stats()
print(f"full N={p.alleles.shape[0]}: structure {s['structure_ms']:.1f} ms values {s['values_ms']:.1f} ms", flush=True)
m.close()
del m

for W in worlds:
    i0, i1 = balanced_shard(p.alleles, 0, W)
    g = hmc_amd.GenoData(np.ascontiguousarray(p.alleles[i0:i1]), p.types)
    r = hmc_amd.HaploModel()
    r.load(g)
    r.set_patterns(pt["start"], pt["len"], pt["freq"], pt["tp"], pt["succ"], last)
    ref = None
    for shape in shapes:
        nw, ipc = (int(x) for x in shape.split(":"))
        r.set_estep_shape(nw, ipc)
        for k in range(2):
            t = time.time()
            key = r.resolve_all()
            wall = (time.time() - t) * 1e3
            ref = ref or key
            assert key == ref, (W, shape, key, ref)
            s = r.estep_split_stats()
            print(f"W={W} shard [{i0},{i1}) shape {shape} run {k}: structure {s['structure_ms']:.1f} ms "
                  f"values {s['values_ms']:.1f} ms ({s['value_passes']} passes) wall {wall:.0f} ms", flush=True)
    r.close()
