"""World-size-2 check (gloo, CPU) of the decomposition the multi-GPU path
relies on: individuals sharded in contiguous blocks,
E-steps independent per shard, and M-step frequencies formed as the all-reduced
sum of per-shard ordered partial sums.  Each rank runs the CPU restatement on
its shard; the reductions go through torch.distributed (gloo)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _shard(alleles, rank, world):  # the library's rule (Ctx::shard / hmc_shard_range)
    from hmc_amd.model import balanced_shard
    return balanced_shard(alleles, rank, world)


def _worker(rank, world, port, q):
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle
        from hmc_amd import synth

        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        p = synth.founder_mosaic(40, 40, A=2, missing=0.02, seed=21)
        N = p.N
        full = oracle.Oracle(p.alleles, p.types, sample_size=10)
        full.find_patterns()
        ll_full = full.resolve_all()
        al_full, w_full, tw_full = full.samples()
        full.find_patterns()  # M1 on all samples
        pt = full.patterns()
        min_freq = 1.5 / (2.0 * N)

        i0, i1 = _shard(p.alleles, rank, world)
        o = oracle.Oracle(p.alleles, p.types, sample_size=10)
        o.find_patterns()
        ll_loc = o.resolve_range(i0, i1)
        al, w, tw_loc = o.samples()
        # E-step shards concatenate to the full E-step (exact)
        sizes = torch.zeros(world, dtype=torch.int64)
        sizes[rank] = len(w)
        dist.all_reduce(sizes)
        off = int(sizes[:rank].sum())
        assert np.array_equal(al, al_full[off:off + len(w)])
        assert np.array_equal(w, w_full[off:off + len(w)])
        red = torch.tensor([ll_loc, tw_loc], dtype=torch.float64)
        dist.all_reduce(red)
        assert abs(red[0].item() - ll_full) <= 1e-12 * abs(ll_full)
        tw = red[1].item()
        assert abs(tw - tw_full) <= 1e-12 * tw_full
        # M-step: per-pattern ordered local sums, all-reduced
        P = len(pt["start"])
        loc = np.zeros(P)
        for k in range(P):
            s, l = pt["start"][k], pt["len"][k]
            m = np.all(al[:, s:s + l] == pt["alleles"][k, :l], axis=1)
            acc = 0.0
            for h in np.nonzero(m)[0]:
                acc += w[h]
            loc[k] = acc
        t = torch.from_numpy(loc)
        dist.all_reduce(t)
        freq = t.numpy() / tw
        rel = np.abs(freq - pt["freq"]) / np.maximum(pt["freq"], 1e-300)
        assert rel.max() <= 1e-12, rel.max()
        # no accept/reject decision sits within rounding of min_freq here
        assert np.array_equal(freq >= min_freq, pt["freq"] >= min_freq)
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_sharded_decomposition_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res
