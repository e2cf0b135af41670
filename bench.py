#!/usr/bin/env python3
"""Benchmark: individual·loci per second per EM iteration of the HaploModel EM
(BASELINE.json metric) on synthetic founder-mosaic panels.

    python bench.py --gpus N --steps K --warmup W

Workload: BASELINE.json configs[2] — 10 000 individuals x 2 000 biallelic SNP
loci (cfg 3, seed 3; the largest configuration quoted for one MI355X), reference
parameters (min-freq-abs 1.5, pattern length 1..30, sample size 10).  A "step"
is one EM iteration, E-step (HaploModel::resolveAll) + M-step
(PatternManager::findPatternByFreq on the weighted samples), continuing the EM
chain from the genotype-mined model M0: step k = E_k, accept + HaploComp, M_k
(hmc_em_iteration: one HaploModel::run iteration).  Before the timed
region the panel is resident in HBM and M0 has been mined (its time is
reported separately); the warmup steps run the same chain, then
the samples are dropped and M0 is mined again so that the timed steps start
from M0 (E1 included).  --config 2 / 5 select the other single-GPU configs.

Multi-GPU: launched by torch.distributed.run, one process per GPU.  The panel
is the same (strong scaling): individuals are sharded in contiguous blocks; the
M-step's per-level candidate sums are reduced in rank order over RCCL inside
libhmc_amd (chained ncclBroadcast of seeded partial sums: bit-identical to one
GPU; hmc_set_reduction selects a single ncclAllReduce instead).
torch.distributed (gloo) only bootstraps the RCCL id, the barriers and the
max-over-ranks time.
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
PMC_DIR = os.path.join(ROOT, "profiles", "r02")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 5],
                    help="BASELINE config (synth.CONFIGS); the options below override it")
    ap.add_argument("--individuals", type=int, default=0, help="total individuals (all ranks)")
    ap.add_argument("--loci", type=int, default=0)
    ap.add_argument("--alleles", type=int, default=0, help="alleles per locus of the synthetic panel (cfg 5: 8)")
    ap.add_argument("--missing", type=float, default=0.0, help="missing-allele rate of the synthetic panel")
    ap.add_argument("--seed", type=int, default=0, help="panel seed (default = config index)")
    ap.add_argument("--sample-size", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-indiv", type=int, default=40, help="individuals timed for the CPU E-step sample")
    ap.add_argument("--cpu-roots", type=int, default=0, help="start loci timed for the CPU M-step sample (0: L/40)")
    ap.add_argument("--trace-bytes", type=int, default=0, help="E-step store budget per store (0: automatic)")
    ap.add_argument("--reduction", default="ordered", choices=["ordered", "allreduce"],
                    help="cross-rank M-step sums: rank-ordered (bit-identical to one GPU) or one all-reduce")
    ap.add_argument("--collective", default="rccl", choices=["rccl", "host"],
                    help="M-step collective: RCCL (the product), or a gloo host all-reduce with every rank on "
                         "GPU LOCAL_RANK %% device_count (rehearses the multi-rank bench on one GPU; not a measurement)")
    a = ap.parse_args()
    c = synth.CONFIGS[a.config]
    a.N = a.individuals or c["N"]
    a.L = a.loci or c["L"]
    a.A = a.alleles or c["A"]
    a.seed = a.seed or a.config
    a.tag = f"cfg{a.config}" if (a.N, a.L, a.A, a.seed, a.missing) == (c["N"], c["L"], c["A"], a.config, 0.0) else "custom"
    return a


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
    dev = local % max(1, torch.cuda.device_count()) if args.collective == "host" else local
    torch.cuda.set_device(dev)

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

    N, L = args.N, args.L
    panel = synth.founder_mosaic(N, L, A=args.A, missing=args.missing, seed=args.seed)
    genos = hmc_amd.GenoData.from_panel(panel)

    if world > 1 and args.collective == "host":
        def host_allreduce(arr):  # in place, float64, summed over ranks by gloo
            dist.all_reduce(torch.from_numpy(arr))

        m = hmc_amd.HaploModel(device=dev, rank=rank, world=world, host_allreduce=host_allreduce)
    else:
        uid = None
        if world > 1:
            obj = [hmc_amd.HaploModel.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(obj, src=0)
            uid = obj[0]
        m = hmc_amd.HaploModel(device=local, rank=rank, world=world, unique_id=uid)
    m.set_reduction(args.reduction)
    m.sample_size = args.sample_size
    if args.trace_bytes:
        m.set_tuning(trace_bytes=args.trace_bytes)
    m.load(genos)

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
        print(f"[bench] cpu baseline {cpu['value']:.4g} {cpu['unit']} ({cpu['t_iter_s']:.0f} s/iteration)",
              file=sys.stderr, flush=True)
        m.clear_samples()
        m.find_patterns()

    def progress(msg):
        if rank == 0:
            print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)

    progress(f"M0 {P0} patterns in {t_m0:.1f} s")

    chain = {"it": 0, "old_ll": -float("inf")}

    def em_step():
        # one HaploModel::run iteration (HaploModel.cpp:130-144): E-step, accept,
        # HaploComp, M-step (always: a fixed number of steps is timed)
        chain["it"] += 1
        log, chain["old_ll"], _ = m.em_iteration(chain["it"], chain["old_ll"], always_mstep=True)
        ll, H, re, rm, P = log["log_likelihood"], log["n_samples"], log["r_e"], log["r_m"], log["n_patterns"]
        t = m.timings()
        sp = m.estep_split_stats()
        progress(f"EM step: LL {ll:.6f}, R_E {re}, E {t['estep_forward_ms']:.0f} ms, M {t['mstep_ms']:.0f} ms")
        return dict(ll=ll, H=H, r_e=re, r_m=rm, P=P, estep_ms=t["estep_forward_ms"] + t["estep_traceback_ms"],
                    struct_ms=sp["structure_ms"], values_ms=sp["values_ms"], fallback_ms=sp["fallback_ms"],
                    n_fallback=sp["n_fallback"], struct_passes=sp["structure_passes"],
                    value_passes=sp["value_passes"], tb_ms=t["estep_traceback_ms"], mstep_ms=m.timings()["mstep_ms"])

    warm = [em_step() for _ in range(args.warmup)]
    m.clear_samples()
    m.find_patterns()  # back to M0 so the timed chain is E1+M1, E2+M2, ...
    chain.update(it=0, old_ll=-float("inf"))

    barrier()
    t0 = time.perf_counter()
    steps = [em_step() for _ in range(args.steps)]
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms_per_step = elapsed / args.steps * 1e3
    value = N * L / (elapsed / args.steps)

    # Roofline of the dominant kernel, the E-step value pass (estep_values):
    # SURVEY.md §8d prices the E-step at 8 B per retained k-best link (R_E); the
    # value pass owns that term.  Per launch: algorithmic bytes / HIP-event
    # duration on the context stream, summed over the timed launches (a large
    # E-step runs its individuals in several groups, one launch each).
    r_e_all = sum_over_ranks(float(sum(s["r_e"] for s in steps)))
    val_ms = max_over_ranks(sum(s["values_ms"] for s in steps))
    n_launch = sum(s["value_passes"] for s in steps)
    achieved = 8.0 * r_e_all / (val_ms * 1e-3) / 1e9 / world if val_ms > 0 else 0.0
    # Roofline of the whole iteration: B_iter = 2NL (genotypes)
    # + 2HL (samples written by E, read by M) + 8 R_E + 1 R_M, over t_iter.
    H_all = sum_over_ranks(float(sum(s["H"] for s in steps)))
    r_m_all = sum_over_ranks(float(sum(s["r_m"] for s in steps)))  # each rank scans its own samples
    b_iter = (2.0 * N * L * args.steps + 2.0 * H_all * L + 8.0 * r_e_all + r_m_all) / args.steps
    ach_iter = b_iter / (elapsed / args.steps) / 1e9
    pmc = pmc_summary(args.tag)

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
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic founder-mosaic panel (K=8 founders, rho=0.002, A={args.A}, "
                    f"missing={args.missing}, seed={args.seed}), generated in-process",
            "config": {
                "workload": f"{args.tag}: {N} individuals x {L} SNP loci, {args.A} alleles/locus; "
                            f"step = one EM iteration (E_k, accept, HaploComp, M_k) from the genotype-mined model M0",
                "individuals": N, "loci": L, "sample_size": args.sample_size,
                "min_freq_abs": 1.5, "pattern_len": [1, 30],
                "parallelism": f"individual-sharded x{world}, " + ("ordered RCCL reduction (chained broadcasts)" if args.reduction == "ordered"
                                                                     else "RCCL all-reduce") + " per mining level"
                               + (" [REHEARSAL: gloo host collective, ranks sharing GPUs - not a measurement]"
                                  if world > 1 and args.collective == "host" else ""),
            },
            "roofline": {
                "bound": "hbm", "kernel": "estep_values",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": pmc.get("hbm_bytes_per_launch") if pmc else None,
                "traffic_source": pmc.get("source") if pmc else None,
                "alg_bytes_per_launch": 8.0 * r_e_all / world / max(1, n_launch),
                "avg_launch_ms": val_ms / max(1, n_launch),
                "launches": n_launch,
                "per_unit": "8 B per retained k-best link (R_E)",
            },
            "roofline_iter": {
                "bound": "hbm", "achieved": ach_iter, "peak": HBM_PEAK_GBS * world, "unit": "GB/s",
                "frac": ach_iter / (HBM_PEAK_GBS * world), "bytes_per_iter": b_iter,
                "formula": "B_iter = 2NL + 2HL + 8 R_E + R_M (SURVEY.md 8d), / t_iter",
            },
            "cpu_baseline": cpu,
            "m0": {"seconds": t_m0, "patterns": P0, "r_m": rm0},
            "per_step": [{k: (round(v, 6) if isinstance(v, float) else v) for k, v in s.items()} for s in steps],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def pmc_summary(tag):
    """rocprofv3 PMC summary (HBM bytes per estep_values launch) of this
    workload, committed under profiles/r02/ by tools/profile_round.sh; None
    when this configuration has not been profiled."""
    p = os.path.join(PMC_DIR, f"pmc_estep_values_{tag}.json")
    try:
        with open(p) as f:
            d = json.load(f)
        d["source"] = os.path.relpath(p, ROOT)
        return d
    except (OSError, ValueError):
        return None


def cpu_baseline(m, panel, args):
    """Time the CPU restatement (oracle/, 1 thread) on a bounded sample of EM
    iteration 2 of the same chain: E_2 over the first `cpu_indiv` individuals
    with the M1 model (scaled to all individuals) + M_2 over `cpu_roots` start
    loci (each root's DFS subtree is independent, PatternManager.cpp:94-97;
    scaled to all L roots).  The GPU supplies M1 and the E_2 samples, which are
    bit-identical to the restatement's (tests/test_gpu_parity.py)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the baseline, never as the product

    m.resolve_all()  # E1
    m.find_patterns()  # M1
    pt = m.patterns(maxlen=30)
    o = oracle.Oracle(panel.alleles, panel.types, sample_size=args.sample_size)
    o.set_patterns(pt)
    del pt
    ns = min(args.cpu_indiv, panel.N)
    t_e = o.time_resolve_range(0, ns)
    ll, H, re = m.resolve_all()  # E2 samples on the GPU
    al, w, _ = m.samples(H)
    o.set_samples(al, w)
    del al
    k = args.cpu_roots or max(1, panel.L // 40)
    t_m = o.time_find_patterns_roots(panel.L - k, panel.L)
    t_iter = t_e * panel.N / ns + t_m * panel.L / k
    return {
        "value": panel.N * panel.L / t_iter, "unit": "individual·loci/s", "cores": 1, "kind": "port",
        "sample": f"EM iteration 2: E_2 over {ns}/{panel.N} individuals (scaled x{panel.N / ns:g}) + M_2 over "
                  f"start loci [{panel.L - k}, {panel.L}) of {panel.L} (scaled x{panel.L / k:g}), "
                  f"oracle/hmc_oracle.cpp g++ -O2, 1 thread",
        "t_estep_sample_s": t_e, "t_mstep_sample_s": t_m, "t_iter_s": t_iter,
    }


if __name__ == "__main__":
    main()
