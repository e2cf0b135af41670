#!/usr/bin/env python3
"""Benchmark: individual·loci per second per EM iteration of the HaploModel EM
(BASELINE.json metric) on synthetic founder-mosaic panels.

    python bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1]): 1000 individuals x 500
biallelic SNP loci per GPU (weak scaling: the panel has 1000*N individuals),
reference parameters (min-freq-abs 1.5, pattern length 1..30, sample size 10).
A "step" is one EM iteration, E-step (HaploModel::resolveAll) + M-step
(PatternManager::findPatternByFreq on the weighted samples), continuing the
EM chain from the genotype-mined model M0: step k = E_k + M_k.  Before the
timed region the panel is resident in HBM and M0 has been mined (its time is
reported separately); the warmup steps run the same chain,
after which the samples are dropped and M0 is mined again so that the timed
steps start from M0.

Multi-GPU: launched by torch.distributed.run, one process per GPU.
Individuals are sharded in contiguous blocks; the M-step all-reduces the
per-level candidate sums over RCCL inside libhmc_amd.  torch.distributed
(gloo) only bootstraps the RCCL id, the barriers and the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hmc_amd  # noqa: E402
from hmc_amd import synth  # noqa: E402

METRIC = "individuals×loci/sec per EM iter, synthetic panel, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s HBM3E (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--individuals", type=int, default=1000, help="per GPU")
    ap.add_argument("--loci", type=int, default=500)
    ap.add_argument("--sample-size", type=int, default=10)
    ap.add_argument("--alleles", type=int, default=2, help="alleles per locus of the synthetic panel (cfg 5: 8)")
    ap.add_argument("--missing", type=float, default=0.0, help="missing-allele rate of the synthetic panel")
    ap.add_argument("--seed", type=int, default=2, help="panel seed (= BASELINE config index)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=100, help="individuals timed for the CPU E-step")
    return ap.parse_args()


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, local, world


def main():
    args = parse()
    rank, local, world = dist_env()
    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(x: float) -> float:
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())

    N = args.individuals * world
    L = args.loci
    panel = synth.founder_mosaic(N, L, A=args.alleles, missing=args.missing, seed=args.seed)
    genos = hmc_amd.GenoData.from_panel(panel)

    uid = None
    if world > 1:
        obj = [hmc_amd.HaploModel.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    m = hmc_amd.HaploModel(device=local, rank=rank, world=world, unique_id=uid)
    m.sample_size = args.sample_size
    m.load(genos)
    n_local = m.i1 - m.i0

    # M0 on the genotypes (reported separately)
    barrier()
    t0 = time.perf_counter()
    P0, rm0 = m.find_patterns()
    barrier()
    t_m0 = max_over_ranks(time.perf_counter() - t0)

    # CPU baseline (rank 0, N = 1 only): the oracle restatement on this host
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, panel, args)
        m.clear_samples()
        m.find_patterns()

    def em_step():
        ll, H, re = m.resolve_all()
        t = m.timings()
        P, rm = m.find_patterns()
        sp = m.estep_split_stats()
        return dict(ll=ll, H=H, r_e=re, r_m=rm, P=P, fwd_ms=t["estep_forward_ms"], struct_ms=sp["structure_ms"],
                    values_ms=sp["values_ms"], fallback_ms=sp["fallback_ms"], n_fallback=sp["n_fallback"],
                    tb_ms=t["estep_traceback_ms"], mstep_ms=m.timings()["mstep_ms"])

    warm = [em_step() for _ in range(args.warmup)]
    m.clear_samples()
    m.find_patterns()  # back to M0 so the timed chain is E1+M1, E2+M2, ...

    barrier()
    t0 = time.perf_counter()
    steps = [em_step() for _ in range(args.steps)]
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    # roofline of the dominant kernel, the E-step value pass (estep_values):
    # SURVEY.md §8d prices the E-step at 2 B per genotype allele (2*n*L, read by
    # the structure pass) + 8 B per retained k-best link (R_E); the value pass
    # owns the R_E term.  Duration = its HIP-event time on the context stream.
    val_ms = sum(s["values_ms"] for s in steps)
    alg_bytes = sum(8.0 * s["r_e"] for s in steps)
    achieved = alg_bytes / (val_ms * 1e-3) / 1e9 if val_ms > 0 else 0.0
    traffic = pmc_traffic()

    ms_per_step = elapsed / args.steps * 1e3
    value = N * L / (elapsed / args.steps)
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "individual·loci/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic founder-mosaic panel (K=8 founders, rho=0.002, A={args.alleles}, "
                    f"missing={args.missing}, seed={args.seed}), generated in-process",
            "config": {
                "workload": f"{'cfg2 ' if (args.individuals, L, args.alleles) == (1000, 500, 2) else ''}per GPU: "
                            f"{args.individuals} individuals x {L} SNP loci, {args.alleles} alleles/locus; "
                            f"step = one EM iteration (E_k + M_k) from the genotype-mined model M0",
                "individuals": N, "loci": L, "sample_size": args.sample_size,
                "min_freq_abs": 1.5, "pattern_len": [1, 30],
                "parallelism": f"individual-sharded x{world}, RCCL all-reduce per mining level",
            },
            "roofline": {
                "bound": "hbm", "kernel": "estep_values",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "avg_launch_ms": val_ms / args.steps,
                # every launch of the process incl. warmup: the figure rocprofv3 --stats averages
                "avg_launch_ms_all": (val_ms + sum(w["values_ms"] for w in warm)) / (args.steps + len(warm)),
                "estep_ms_per_step": sum(s["fwd_ms"] for s in steps) / args.steps,
                "alg_bytes_per_launch": alg_bytes / args.steps,
            },
            "cpu_baseline": cpu,
            "m0": {"seconds": t_m0, "patterns": P0, "r_m": rm0},
            "per_step": [{k: (round(v, 6) if isinstance(v, float) else v) for k, v in s.items()} for s in steps],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def pmc_traffic():
    """HBM bytes per estep_values launch from the committed rocprofv3 PMC
    summary (profiles/pmc_estep_values.json), or None."""
    p = os.path.join(ROOT, "profiles", "pmc_estep_values.json")
    try:
        with open(p) as f:
            return json.load(f).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(m, panel, args):
    """Time the CPU restatement (oracle/, 1 thread) on a bounded sample of the
    same EM iteration: E_1 over the first `cpu_sample` individuals with the M0
    model (scaled to all individuals) + M_1 over all E_1 samples."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the baseline, never as the product

    pt = m.patterns()
    o = oracle.Oracle(panel.alleles, panel.types, sample_size=args.sample_size)
    o.set_patterns(pt)
    ns = min(args.cpu_sample, panel.N)
    t_e = o.time_resolve_range(0, ns)
    ll, H, re = m.resolve_all()  # E_1 samples on the GPU (bit-identical to the oracle's)
    al, w, _ = m.samples(H)
    o.set_samples(al, w)
    t_m = o.time_find_patterns()
    t_iter = t_e * panel.N / ns + t_m
    return {
        "value": panel.N * panel.L / t_iter, "unit": "individual·loci/s", "cores": 1, "kind": "port",
        "sample": f"E_1 over {ns}/{panel.N} individuals (scaled x{panel.N / ns:g}) + full M_1 over {H} samples, "
                  f"oracle/hmc_oracle.cpp g++ -O2, 1 thread",
        "t_estep_sample_s": t_e, "t_mstep_s": t_m, "t_iter_s": t_iter,
    }


if __name__ == "__main__":
    main()
