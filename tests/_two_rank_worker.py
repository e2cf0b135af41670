"""Worker for test_gpu_parity.test_two_ranks_one_gpu_host_collective: one
rank of a 2-rank HaploModel sharing GPU 0, collectives over gloo."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402


def main():
    rank, out = int(sys.argv[1]), sys.argv[2]
    variant = sys.argv[3] if len(sys.argv) > 3 else "MV"
    reduction = sys.argv[4] if len(sys.argv) > 4 else "ordered"
    dist.init_process_group("gloo", rank=rank, world_size=2)

    def allreduce(arr):
        t = torch.from_numpy(arr)
        dist.all_reduce(t)

    p = synth.founder_mosaic(80, 60, A=3, missing=0.05, seed=5)
    m = hmc_amd.HaploModel(device=0, rank=rank, world=2, host_allreduce=allreduce)
    m.max_iteration = 10
    m.set_reduction(reduction)
    if variant == "MC":
        m.model = "MC"
    elif variant == "BYNUM":
        m.num_patterns, m.min_pattern_len = 150, 2
    m.load(hmc_amd.GenoData.from_panel(p))
    if variant == "WIN":  # every E-step of each rank's shard in windows of 7 loci
        m.set_estep_windows("always", 7)
    m.find_patterns()
    m0_freq = m.patterns()["freq"]
    m.clear_samples()
    res = m.run()
    np.savez(os.path.join(out, f"rank{rank}.npz"), ll=np.array([x["ll"] for x in m.log]), res=res, m0_freq=m0_freq,
             comp=np.array([x["haplocomp"] for x in m.log]))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
