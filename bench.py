#!/usr/bin/env python3
"""Benchmark: individual·loci per second per EM iteration of the HaploModel EM
(BASELINE.json metric) on synthetic founder-mosaic panels.

    python bench.py --gpus N --steps K --warmup W

Workload: BASELINE.json configs[2] — 10 000 individuals x 2 000 biallelic SNP
loci (cfg 3, seed 3; the largest configuration quoted for one MI355X), reference
parameters (min-freq-abs 1.5, pattern length 1..30, sample size 10).

A step is one EM iteration of the reference's converged chain
(HaploModel::run, HaploModel.cpp:130-153): E_k, accept + HaploComp, and M_k
when the chain continues ((old_ll - ll) / old_ll > 1e-4 with ll >= old_ll).
The iteration that stops the chain has no M-step; the next step starts the
chain again from the genotype-mined model M0 (hmc_em_rewind: M0's table
restored, no samples, resolutions = input — inside the timed step).  At cfg 3
the chain is E1+M1, E2+M2, E3, so the K timed steps cycle through it; M0 is
mined once before the timed region and reported separately.
value = N·L·K / timed seconds (K need not be a multiple of the chain length:
the leftover steps are the chain's first, heaviest ones, so this is the
conservative figure); `value_chain` is the same over whole chains only, and
`value_steady` the forced iterations after the chain's end (E4, E5, ...).

Multi-GPU: one process per GPU, launched by torch.distributed.run — or, when
WORLD_SIZE is not set and --gpus N > 1, by this script itself: it starts N
fresh worker processes (rank env set, 127.0.0.1 rendezvous) before anything
touches a GPU and exits with their status.  The panel is the same (strong
scaling): individuals are sharded in contiguous blocks; the M-step's per-level
candidate sums are reduced in rank order over RCCL inside libhmc_amd (a
point-to-point chain: rank r receives the running sums from r-1, continues
them over its own items and sends them to r+1, then rank W-1 broadcasts the
totals once — bit-identical to one GPU; hmc_set_reduction selects a single
ncclAllReduce instead).  torch.distributed
(gloo) only bootstraps the RCCL id, the barriers and the max-over-ranks time.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import hmc_amd  # noqa: E402  (ctypes binding; loads nothing until first use)
from hmc_amd import synth  # noqa: E402

METRIC = "individuals×loci/sec per EM iter, synthetic panel, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s HBM3E (spec)
PMC_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r06", "r05", "r04", "r03")]  # newest profile of the workload first
DBL_MAX = sys.float_info.max
# What bounds estep_values (SQ counters under profiles/): the
# roofline prices it against HBM as the contract asks, but the kernel moves a
# few % of peak; its VALU issue (SQ_INSTS_VALU, tools/sq_summary.py) is the
# roof it runs against.
# The sampled CPU estimate checked against the whole single-thread chain at
# cfg 2 (bench.py --config 2 --cpu-validate on a GPU box, same run).
VALIDATION_NOTE = "profiles/r04/cpu_validate_cfg2.json"
LIMITER = ("VALU issue of the segmented k-best selection: the SIMDs' VALU issue slots measured busy "
           "(4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) over 32 SIMDs x SQ_BUSY_CYCLES per SE; dual issue calibrated "
           "by tools/diag/issue_bench.hip, DESIGN.md 9), not HBM bandwidth")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed steps (default 20; cfg 4: 3, one chain)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 5; cfg 4: 1)")
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5],
                    help="BASELINE config (synth.CONFIGS); the options below override it.  cfg 4 (50 000 x 5 000) is "
                         "the 8-GPU configuration: --gpus 8 gives each rank ~6 250 individuals")
    ap.add_argument("--individuals", type=int, default=0, help="total individuals (all ranks)")
    ap.add_argument("--loci", type=int, default=0)
    ap.add_argument("--alleles", type=int, default=0, help="alleles per locus of the synthetic panel (cfg 5: 8)")
    ap.add_argument("--missing", type=float, default=0.0, help="missing-allele rate of the synthetic panel")
    ap.add_argument("--seed", type=int, default=0, help="panel seed (default = config index)")
    ap.add_argument("--sample-size", type=int, default=10)
    ap.add_argument("--steady-steps", type=int, default=None,
                    help="forced iterations after the chain's end, timed for value_steady (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-indiv", type=int, default=20, help="individuals per CPU E-step sample (E_k, k >= 2)")
    ap.add_argument("--cpu-indiv-e1", type=int, default=24,
                    help="individuals of the CPU E_1 sample (M0 model); timed in two interleaved halves for the spread")
    ap.add_argument("--cpu-roots", type=int, default=30, help="start loci per CPU M-step sample")
    ap.add_argument("--cpu-validate", action="store_true",
                    help="also time the whole chain on the CPU restatement (1 thread) next to the sampled "
                         "estimate: minutes at cfg 2, hours at cfg 3")
    ap.add_argument("--trace-bytes", type=int, default=0, help="E-step store budget per store (0: automatic)")
    ap.add_argument("--reduction", default="ordered", choices=["ordered", "allreduce"],
                    help="cross-rank M-step sums: rank-ordered (bit-identical to one GPU) or one all-reduce")
    ap.add_argument("--collective", default="rccl", choices=["rccl", "host"],
                    help="M-step collective: RCCL (the product), or a gloo host all-reduce with every rank on "
                         "GPU LOCAL_RANK %% device_count (rehearses the multi-rank bench on one GPU; not a measurement)")
    a = ap.parse_args()
    big = a.config == 4  # an E1 of ~25 s per rank at 8 ranks: one chain, no steady leg, no CPU sample
    a.steps = a.steps if a.steps is not None else (3 if big else 20)
    a.warmup = a.warmup if a.warmup is not None else (1 if big else 5)
    a.steady_steps = a.steady_steps if a.steady_steps is not None else (0 if big else 8)
    if big:
        a.no_cpu_baseline = True
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


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without a launcher: N fresh worker processes of this
    script, one per GPU, with the torch.distributed env a launcher would set.
    Runs before anything in this process touches a GPU (no exec from here)."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0 and rc == 0:
                    rc = c
                    for q in procs:  # one rank failed: the others would wait forever in a collective
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    rank, local, world = dist_env()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
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

    def progress(msg):
        if rank == 0:
            print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)

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
    ident = hmc_amd.lib_identity()
    progress(f"library {ident['path']} sha256 {ident['sha256_16']} ({ident['build']})")

    # M0 on the genotypes (reported separately), kept for the rewinds
    barrier()
    t0 = time.perf_counter()
    P0, rm0 = m.find_patterns()
    barrier()
    t_m0 = max_over_ranks(time.perf_counter() - t0)
    m.model_save()
    progress(f"M0 {P0} patterns in {t_m0:.1f} s")

    # CPU baseline (rank 0, N = 1 only): the oracle restatement on this host,
    # sampled along the same chain
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(m, panel, args)
        print(f"[bench] cpu baseline {cpu['value']:.4g} {cpu['unit']} ({cpu['t_iter_s']:.0f} s/iteration)",
              file=sys.stderr, flush=True)
        m.em_rewind()

    chain = {"it": 0, "old_ll": -DBL_MAX, "ended": False}
    run_log = []  # (R_E, value-pass launches) of every E-step this process runs after M0, in order (PMC pairing)

    def em_step(force_m: bool = False):
        """One step of the converged chain (or, force_m, an iteration that
        always runs its M-step: the steady leg)."""
        t_s = time.perf_counter()
        if chain["ended"]:  # the previous step stopped the chain: start again from M0
            m.em_rewind()
            chain.update(it=0, old_ll=-DBL_MAX, ended=False)
        chain["it"] += 1
        it = chain["it"]
        log, chain["old_ll"], go = m.em_iteration(it, chain["old_ll"], always_mstep=force_m)
        if not go and not force_m:
            chain["ended"] = True
        wall = time.perf_counter() - t_s
        t = m.timings()
        sp = m.estep_split_stats()
        ms_stats = m.mine_stats() if go or force_m else {"reduction_ms": 0.0, "reduction_levels": 0}
        win = m.estep_windows()
        run_log.append([int(log["r_e"]), int(sp["value_passes"])])
        progress(f"EM iteration {it}: LL {log['log_likelihood']:.6f}, R_E {log['r_e']}, "
                 f"E {t['estep_forward_ms'] + t['estep_traceback_ms']:.0f} ms "
                 f"(structure {sp['structure_ms']:.0f} in {sp['structure_passes']}, values {sp['values_ms']:.0f} in "
                 f"{sp['value_passes']}), M {t['mstep_ms'] if go or force_m else 0:.0f} ms, step {wall * 1e3:.0f} ms"
                 + ("" if go or force_m else "  [chain stops]"))
        return dict(iteration=it, go=bool(go), wall_ms=wall * 1e3, ll=log["log_likelihood"], H=log["n_samples"],
                    r_e=log["r_e"], r_m=log["r_m"] if go or force_m else 0, P=log["n_patterns"],
                    estep_ms=t["estep_forward_ms"] + t["estep_traceback_ms"], struct_ms=sp["structure_ms"],
                    values_ms=sp["values_ms"], fallback_ms=sp["fallback_ms"], n_fallback=sp["n_fallback"],
                    struct_passes=sp["structure_passes"], value_passes=sp["value_passes"],
                    tb_ms=t["estep_traceback_ms"], mstep_ms=t["mstep_ms"] if go or force_m else 0.0,
                    value_dataflow=m.last_value_pass_dataflow(), reduction_ms=ms_stats["reduction_ms"],
                    reduction_levels=ms_stats["reduction_levels"], windows=win["windows"],
                    collection_ms=win["collection_ms"])

    for _ in range(args.warmup):
        em_step()
    m.em_rewind()  # the timed region starts a fresh chain at E1
    chain.update(it=0, old_ll=-DBL_MAX, ended=False)

    barrier()
    t0 = time.perf_counter()
    steps = [em_step() for _ in range(args.steps)]
    barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms_per_step = elapsed / args.steps * 1e3
    value = N * L / (elapsed / args.steps)

    # whole chains inside the timed region (per-step walls are this rank's;
    # every step ends in a collective, so ranks stay in step)
    chains, cur = [], []
    for s in steps:
        cur.append(s)
        if not s["go"]:
            chains.append(cur)
            cur = []
    chain_iters = sum(len(c) for c in chains)
    chain_s = max_over_ranks(sum(s["wall_ms"] for c in chains for s in c) / 1e3)
    value_chain = N * L * chain_iters / chain_s if chain_iters else None

    # steady leg (not the headline): a fresh chain to its end, then forced iterations
    steady = None
    if args.steady_steps > 0:
        m.em_rewind()
        chain.update(it=0, old_ll=-DBL_MAX, ended=False)
        while True:
            s = em_step(force_m=True)
            if not s["go"]:
                break
        barrier()
        t1 = time.perf_counter()
        st = [em_step(force_m=True) for _ in range(args.steady_steps)]
        barrier()
        el = max_over_ranks(time.perf_counter() - t1)
        steady = {"value": N * L / (el / args.steady_steps), "ms_per_step": el / args.steady_steps * 1e3,
                  "iterations": [s["iteration"] for s in st]}

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
    pmc = pmc_summary(args.tag, ident)
    sq = sq_summary(args.tag, ident)
    # the bound from the evidence: the fraction of the VALU issue roof the SQ
    # pass measured against the fraction of HBM bandwidth the PMC pass measured
    hbm_frac_meas = None
    if pmc and pmc.get("hbm_bytes_per_launch") and val_ms > 0 and n_launch:
        hbm_frac_meas = pmc["hbm_bytes_per_launch"] / (val_ms * 1e-3 / n_launch) / 1e9 / HBM_PEAK_GBS
    # (only counters of the library this process loaded count as evidence;
    # without them the line prices against HBM and says the bound is unmeasured)
    bound, bound_basis = "hbm", "no same-build counters: priced against HBM, limiter unmeasured"
    if sq and sq["same_build"] and sq.get("valu_issue_frac") is not None:
        hbm_f = hbm_frac_meas or achieved / HBM_PEAK_GBS
        bound = "valu-issue" if sq["valu_issue_frac"] > hbm_f else "hbm"
        if max(sq["valu_issue_frac"], hbm_f) < 0.5:  # neither roof near: the waves wait (SQ_WAIT_ANY)
            bound = "latency"
        bound_basis = (f"measured VALU issue occupancy {sq['valu_issue_frac']:.2f} vs HBM fraction {hbm_f:.2f} "
                       f"({'PMC' if hbm_frac_meas else 'algorithmic bytes'}), same build")

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
                            f"step = one iteration of the reference's converged EM chain from M0 "
                            f"(E_k, accept, HaploComp, M_k while continuing; restart from M0 after the stop)",
                "individuals": N, "loci": L, "sample_size": args.sample_size,
                "min_freq_abs": 1.5, "pattern_len": [1, 30],
                "parallelism": f"individual-sharded x{world}, " + ("ordered RCCL reduction (send/recv chain + one broadcast)" if args.reduction == "ordered"
                                                                     else "RCCL all-reduce") + " per mining level"
                               + (" [REHEARSAL: gloo host collective, ranks sharing GPUs - not a measurement]"
                                  if world > 1 and args.collective == "host" else ""),
            },
            "value_chain": value_chain,
            "chain": {"iterations": [len(c) for c in chains],
                      "ms_per_iteration": chain_s / chain_iters * 1e3 if chain_iters else None},
            "value_steady": steady,
            "roofline": {
                "bound": bound, "bound_basis": bound_basis, "kernel": "estep_values",
                "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                "traffic": pmc.get("hbm_bytes_per_launch") if pmc and pmc["same_build"] else None,
                "traffic_over_alg": pmc.get("traffic_over_alg") if pmc and pmc["same_build"] else None,
                "traffic_source": pmc.get("source") if pmc else None,
                "traffic_same_build": pmc["same_build"] if pmc else None,
                "hbm_frac_measured": hbm_frac_meas if pmc and pmc["same_build"] else None,
                "valu_issue_frac": sq["valu_issue_frac"] if sq and sq["same_build"] else None,
                "valu_dual_issue_share": sq["valu_dual_issue_share"] if sq and sq["same_build"] else None,
                "valu_issue_frac_nominal_4cyc": sq["valu_issue_frac_nominal_4cyc"] if sq and sq["same_build"] else None,
                "valu_issue_frac_nominal_2cyc": sq["valu_issue_frac_nominal_2cyc"] if sq and sq["same_build"] else None,
                "lds_bank_conflict_ratio": sq["lds_bank_conflict_ratio"] if sq and sq["same_build"] else None,
                "valu_issue_source": sq.get("source") if sq else None,
                "valu_issue_same_build": sq["same_build"] if sq else None,
                "valu_issue_formula": "4 * (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / (32 SIMDs per SE * SQ_BUSY_CYCLES): "
                                      "measured VALU issue-slot occupancy (one instruction per quad-cycle, two when "
                                      "they dual-issue; profiles/r06/issue/)",
                "limiter": LIMITER,
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
            "library": ident,
            "per_step": [{k: (round(v, 6) if isinstance(v, float) else v) for k, v in s.items()} for s in steps],
            "run_estep_log": run_log,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _profile_json(name, ident):
    """The newest committed profile summary `name` under profiles/rNN/
    (tools/profile_round.sh), with `same_build`: whether it was measured on
    the library this process loaded (SHA-256 prefix).  Counters of another
    build are reported as null in the line, not paired with this run's times."""
    for d in PMC_DIRS:
        p = os.path.join(d, name)
        try:
            with open(p) as f:
                out = json.load(f)
        except (OSError, ValueError):
            continue
        out["source"] = os.path.relpath(p, ROOT)
        lib = out.get("library") or {}
        out["same_build"] = bool(lib) and lib.get("sha256_16") == ident.get("sha256_16")
        return out
    return None


def pmc_summary(tag, ident):
    """rocprofv3 PMC summary (HBM bytes per estep_values launch) of this workload."""
    return _profile_json(f"pmc_estep_values_{tag}.json", ident)


def sq_summary(tag, ident):
    """SQ summary of estep_values (tools/sq_summary.py): VALU issue fraction and
    LDS bank-conflict ratio summed over the instantiations the pass launched."""
    d = _profile_json(f"sq_estep_values_{tag}.json", ident)
    if not d or not d.get("kernels"):
        return None
    ks = list(d["kernels"].values())
    t = sum(k["kernel_seconds"] for k in ks)
    cap = 1024 * 2.4e9 * t
    valu = sum(k["valu_insts"] for k in ks)
    lds_conf = max(k["lds_bank_conflict_ratio"] for k in ks)
    meas, dual = None, None
    bp = [k.get("busy_pass") for k in ks]
    if all(b and b.get("SQ_BUSY_CYCLES") for b in bp):  # measured issue over every instantiation the pass launched
        v1 = sum(b["SQ_INSTS_VALU"] for b in bp)
        v2 = sum(b["SQ_ACTIVE_INST_VALU2"] or 0.0 for b in bp)
        meas = 4.0 * (v1 - v2) / (32.0 * sum(b["SQ_BUSY_CYCLES"] for b in bp))
        dual = 2.0 * v2 / v1 if v1 else None
    return {"valu_issue_frac": meas, "valu_dual_issue_share": dual,
            "valu_issue_frac_nominal_4cyc": 4.0 * valu / cap if cap else None,
            "valu_issue_frac_nominal_2cyc": 2.0 * valu / cap if cap else None,
            "lds_bank_conflict_ratio": lds_conf, "source": d["source"], "same_build": d["same_build"]}


def cpu_baseline(m, panel, args):
    """Time the CPU restatement (oracle/, 1 thread) on bounded, stratified
    samples of the same converged chain: each E_k over a sample of individuals
    spread evenly over the E-step's own cost order (heterozygous-or-missing
    loci, heaviest first), each M_k over start loci spread evenly over [0, L)
    (each root's DFS subtree is independent, PatternManager.cpp:94-97), with
    the GPU's model and samples of that step (bit-identical to the
    restatement's, tests/test_gpu_parity.py).  Every sample is scaled to the
    whole panel; t_iter = the chain's scaled time / its iterations."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # test infrastructure: timed as the baseline, never as the product

    N, L = panel.N, panel.L
    a = panel.alleles
    het = ((a[:, 0, :] != a[:, 1, :]) | (a[:, 0, :] < 0)).sum(axis=1)
    order = np.argsort(-het, kind="stable")

    def strat_indiv(k):
        k = max(1, min(k, N))
        return np.sort(order[(np.arange(k) * N) // k + N // (2 * k)])

    kr = max(1, min(args.cpu_roots, L))
    roots = (np.arange(kr) * L) // kr + L // (2 * kr)
    o = oracle.Oracle(panel.alleles, panel.types, sample_size=args.sample_size)
    old_ll, it, parts = -DBL_MAX, 1, []
    e1_spread = None
    while True:
        pt = m.patterns(maxlen=30)
        P = len(pt["start"])
        o.set_patterns(pt)
        del pt
        ids = strat_indiv(args.cpu_indiv_e1 if it == 1 else args.cpu_indiv)
        if it == 1 and len(ids) >= 2:  # two interleaved halves of the stratified sample: the estimate's spread
            ta, tb = o.time_resolve_list(ids[0::2]), o.time_resolve_list(ids[1::2])
            te = ta + tb
            e1_spread = {"half_a_scaled_s": ta * N / len(ids[0::2]), "half_b_scaled_s": tb * N / len(ids[1::2]),
                         "rel_diff": abs(ta / len(ids[0::2]) - tb / len(ids[1::2])) / max(1e-12, te / len(ids))}
        else:
            te = o.time_resolve_list(ids)
        parts.append({"step": f"E{it}", "sample": len(ids), "seconds": te, "scale": N / len(ids)})
        # HaploBuilder::initialize clears P maps before every individual
        # (HaploBuilder.cpp:25-33); the restatement's resolve skips that, so it
        # is timed on its own (one pass) and charged N times
        tr = oracle.Oracle.time_best_pair_reset(P)
        parts.append({"step": f"E{it} reset", "sample": 1, "seconds": tr, "scale": float(N), "patterns": P})
        ll, H, _ = m.resolve_all()  # the same E-step on the GPU (its samples feed the next M-step)
        go = ll >= old_ll and (old_ll - ll) / old_ll > 1e-4  # HaploModel.cpp:139
        if not go:
            break
        al, w, _ = m.samples(H)
        o.set_samples(al, w)
        del al
        tm = o.time_find_patterns_root_list(roots)
        parts.append({"step": f"M{it}", "sample": int(kr), "seconds": tm, "scale": L / kr})
        m.find_patterns()
        old_ll, it = ll, it + 1
    t_chain = sum(p["seconds"] * p["scale"] for p in parts)
    t_iter = t_chain / it
    t_iter_port = sum(p["seconds"] * p["scale"] for p in parts if not p["step"].endswith("reset")) / it
    validation = None
    if args.cpu_validate:  # the same chain in full, M0 to the stop, one thread (HaploModel::run)
        oracle.set_threads(1)
        full = oracle.Oracle(panel.alleles, panel.types, sample_size=args.sample_size, max_iter=100).run()
        n_e, n_m = len(full["t_e"]), max(0, full["iterations"] - 1)
        t_full = float(sum(full["t_e"][:n_e]) + sum(full["t_m"][:n_m]))
        validation = {"full_chain_iterations": int(full["iterations"]), "full_chain_seconds": t_full,
                      "full_t_iter_s": t_full / full["iterations"], "sampled_t_iter_s": t_iter_port,
                      "sampled_over_full": t_iter_port / (t_full / full["iterations"]),
                      "full_parts_s": {"E": [float(x) for x in full["t_e"][:n_e]],
                                       "M": [float(x) for x in full["t_m"][:n_m]]}}
    return {
        "value": N * L / t_iter, "unit": "individual·loci/s", "cores": 1, "kind": "port",
        "host_cores": os.cpu_count(),
        "host_cores_note": "os.cpu_count() of the host; the reference and the restatement are single-threaded, so one "
                           "core is timed (a box's CPU share for this job is 16)",
        "sample": f"converged chain of {it} EM iterations ({', '.join(p['step'] for p in parts)}): E_1 over "
                  f"{min(args.cpu_indiv_e1, N)} and E_k over {min(args.cpu_indiv, N)} individuals spread over the "
                  f"cost order, M_k over {kr} start loci spread over [0, {L}), each scaled to the panel; plus "
                  f"HaploBuilder::initialize's per-individual clear of P maps (HaploBuilder.cpp:25-33), which the "
                  f"restatement's resolve omits, timed once per E-step and charged N times; "
                  f"oracle/hmc_oracle.cpp g++ -O2, 1 thread",
        "e1_spread": e1_spread,
        "parts": parts, "t_iter_s": t_iter, "sample_seconds": sum(p["seconds"] for p in parts),
        "validation": validation if validation else VALIDATION_NOTE,
    }


if __name__ == "__main__":
    main()
