"""Python mirror of the reference's HaploModel interface over libhmc_amd.so.

Names, parameters and defaults follow HaploModel (HaploModel.h:15-33) and the
HMC command line (HMC.cpp:35-47):

    m = HaploModel()
    m.sample_size = 10; m.max_iteration = 50
    resolutions = m.run(genos)            # HaploModel::run (HaploModel.cpp:117-155)

Lower-level seams (used by the parity tests) mirror the reference's internal
calls: find_patterns() = PatternManager::findPatternByFreq + initialize,
resolve_all() = HaploModel::resolveAll.  Every call goes through the C-ABI of
include/hmc_amd.h; errors the reference reports with Logger::error + exit(1)
raise HMCError here.
"""
from __future__ import annotations

import ctypes as C
import dataclasses

import numpy as np

from ._lib import ALLREDUCE_FN, HMCError, IterLog, lib

_P = C.POINTER


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(_P(t))


@dataclasses.dataclass
class GenoData:
    """Genotype panel: alleles[N][2][L] allele symbols (-1 missing), per-locus types."""

    alleles: np.ndarray
    types: str

    @property
    def genotype_num(self) -> int:
        return self.alleles.shape[0]

    @property
    def genotype_len(self) -> int:
        return self.alleles.shape[2]

    @classmethod
    def from_panel(cls, panel) -> "GenoData":
        return cls(np.ascontiguousarray(panel.alleles, dtype=np.int32), panel.types)


def balanced_shard(alleles: np.ndarray, rank: int, world: int) -> tuple[int, int]:
    """Individuals [i0, i1) of `rank`: contiguous blocks whose E-step cost
    (L/8 + heterozygous-or-missing loci per individual) splits evenly — the
    rule of the library's Ctx::shard (hmc_shard_range)."""
    a = np.asarray(alleles)
    N, _, L = a.shape
    if world == 1:
        return 0, N
    het = ((a[:, 0, :] != a[:, 1, :]) | (a[:, 0, :] < 0)).sum(axis=1)
    pre = np.concatenate([[0.0], np.cumsum(L / 8.0 + het)])

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return N
        return int(np.searchsorted(pre, pre[N] * r / world, side="left"))

    return cut(rank), cut(rank + 1)


class HaploModel:
    """HaploModel (model "MV", sampling EM) on one MI355X, or one rank of a sharded run."""

    def __init__(self, device: int = 0, rank: int = 0, world: int = 1, unique_id: bytes | None = None,
                 host_allreduce=None, rccl_comm: int | None = None):
        """world > 1 shards individuals over ranks.  The M-step collective is
        RCCL (unique_id from HaploModel.unique_id() on rank 0, or an RCCL
        communicator the caller owns, `rccl_comm` = its ncclComm_t address), or,
        when `host_allreduce(np.ndarray)` is given, that callable, which must
        sum the float64 array across ranks in place (e.g. torch.distributed
        gloo)."""
        L = lib()
        h = C.c_void_p()
        self._cb = None
        if host_allreduce is not None:
            def _cb(buf, n, _user):
                try:
                    arr = np.ctypeslib.as_array(buf, shape=(n,))
                    host_allreduce(arr)
                    return 0
                except Exception:  # noqa: BLE001 — reported to the library as failure
                    return 1
            self._cb = ALLREDUCE_FN(_cb)
            rc = L.hmc_ctx_create_hostcoll(device, rank, world, self._cb, None, C.byref(h))
        elif rccl_comm is not None:
            rc = L.hmc_ctx_create_comm(device, C.c_void_p(rccl_comm), C.byref(h))
        elif world > 1 or unique_id is not None:
            uid = C.create_string_buffer(unique_id, 128)
            rc = L.hmc_ctx_create_dist(device, rank, world, C.cast(uid, C.c_void_p), C.byref(h))
        else:
            rc = L.hmc_ctx_create(device, C.byref(h))
        self._h = h
        self.rank, self.world = rank, world
        self._comm_keepalive = rccl_comm
        if rc:
            msg = L.hmc_ctx_error(h).decode() if h else ""
            self.close()
            raise HMCError(rc, msg)
        # HaploModel public fields (HaploModel.h:15-26) with the CLI defaults (HMC.cpp:35-47)
        self.min_freq = -1.0
        self.min_freq_abs = 1.5
        self.min_pattern_len = 1
        self.max_pattern_len = 30
        self.sample_size = 10
        self.max_iteration = 1
        self.model = "MV"  # HaploModel::setModel: MV, MC or MA (HMC.cpp:35)
        self.mc_order = 1  # HMC.cpp:41
        self.num_patterns = -1  # HMC.cpp:38: > 0 mines with findPatternByNum
        self.exact_estimate = False  # HMC.cpp:42 --exact-estimate: M-steps by estimatePatterns
        self.N = self.L = self.amax = 0
        self.iterations = 0
        self.log: list[dict] = []

    # ------------------------------------------------------------------ util
    def _check(self, rc: int):
        if rc:
            raise HMCError(rc, lib().hmc_ctx_error(self._h).decode())

    def _push_params(self):
        self._check(lib().hmc_set_params(self._h, float(self.min_freq_abs), float(self.min_freq),
                                         int(self.min_pattern_len), int(self.max_pattern_len),
                                         int(self.sample_size)))
        self._check(lib().hmc_set_model(self._h, str(self.model).encode(), int(self.mc_order)))
        self._check(lib().hmc_set_num_patterns(self._h, int(self.num_patterns)))
        self._check(lib().hmc_set_exact_estimate(self._h, 1 if self.exact_estimate else 0))

    def close(self):
        if getattr(self, "_h", None) and self._h.value:
            lib().hmc_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def unique_id() -> bytes:
        buf = C.create_string_buffer(128)
        rc = lib().hmc_rccl_unique_id(C.cast(buf, C.c_void_p))
        if rc:
            raise HMCError(rc, "ncclGetUniqueId failed")
        return buf.raw

    def set_tuning(self, frontier_cap: int = 0, trace_bytes: int = 0, waves: int = 0):
        self._check(lib().hmc_set_tuning(self._h, frontier_cap, trace_bytes, waves))

    def set_estep_shape(self, waves_per_individual: int = 0, individuals_per_cu: int = 0):
        """E-step launch shape (results are identical for every shape)."""
        self._check(lib().hmc_set_estep_shape(self._h, waves_per_individual, individuals_per_cu))

    def set_pass_shapes(self, structure_waves: int = 0, structure_ipc: int = 0, value_waves: int = 0,
                        value_ipc: int = 0):
        """Launch shapes of the split E-step's passes (0 = automatic)."""
        self._check(lib().hmc_set_pass_shapes(self._h, structure_waves, structure_ipc, value_waves, value_ipc))

    def set_store_budgets(self, trace_bytes: int = 0, record_bytes: int = 0):
        """E-step store budgets in bytes (0 = automatic)."""
        self._check(lib().hmc_set_store_budgets(self._h, int(trace_bytes), int(record_bytes)))

    def set_mine_block(self, start_loci: int = 0):
        """Start loci per block of the pattern search (0 = automatic)."""
        self._check(lib().hmc_set_mine_block(self._h, int(start_loci)))

    def estep_frontier(self) -> dict:
        """Largest frontier of the last E-step and the state capacity it ran with."""
        ms, fc = C.c_int(), C.c_int()
        self._check(lib().hmc_last_estep_frontier(self._h, C.byref(ms), C.byref(fc)))
        return dict(max_states=ms.value, capacity=fc.value)

    def set_mine_memory(self, list_bytes: int = 0):
        """Cap one search level's matching lists (bytes; 0 = device memory):
        a block over it is re-run with half the width."""
        self._check(lib().hmc_set_mine_memory(self._h, int(list_bytes)))

    def mine_stats(self) -> dict:
        b, n, g = C.c_int(), C.c_int64(), C.c_double()
        self._check(lib().hmc_last_mine_stats(self._h, C.byref(b), C.byref(n), C.byref(g)))
        ms, lv = C.c_double(), C.c_int()
        self._check(lib().hmc_last_mine_reduction(self._h, C.byref(ms), C.byref(lv)))
        return dict(blocks=b.value, nodes=n.value, node_window_gb=g.value, reduction_ms=ms.value,
                    reduction_levels=lv.value)

    def model_save(self):
        """Keep a device copy of the current pattern table (hmc_model_save)."""
        self._check(lib().hmc_model_save(self._h))

    def em_rewind(self):
        """Restore the saved table and the EM state right after it was built
        (HaploModel::run after build(), HaploModel.cpp:121-129)."""
        self._check(lib().hmc_em_rewind(self._h))

    def set_reduction(self, mode: str):
        """Cross-rank sums: "ordered" (default, bit-exact with one rank) or
        "allreduce" (one collective per mining level, last-bit drift)."""
        self._check(lib().hmc_set_reduction(self._h, {"ordered": 0, "allreduce": 1}[mode]))

    def set_force_collectives(self, on: bool = True):
        """Test hook: a one-rank context with a communicator runs every collective
        (the ordered chain's hop as a grouped ncclSend/ncclRecv to itself)."""
        self._check(lib().hmc_set_force_collectives(self._h, int(bool(on))))

    def comm_stats(self) -> dict:
        """Point-to-point hops of the ordered chain issued so far (hmc_comm_stats)."""
        s, r, b = C.c_int64(), C.c_int64(), C.c_uint64()
        self._check(lib().hmc_comm_stats(self._h, C.byref(s), C.byref(r), C.byref(b)))
        return dict(sends=s.value, recvs=r.value, bytes_received=b.value)

    def set_key_probes(self, probes: int):
        """Structure pass: LDS probes of the key table before its HBM tier (results unchanged)."""
        self._check(lib().hmc_set_key_probes(self._h, int(probes)))

    def set_structure_tier(self, key_mult10: int = 0, contrib_mult10: int = 0):
        """Structure pass LDS split (tenths of the frontier states; 0 = default; results unchanged)."""
        self._check(lib().hmc_set_structure_tier(self._h, int(key_mult10), int(contrib_mult10)))

    def set_comm_timeout(self, seconds: float):
        """Bounded waits of an RCCL context (hmc_set_comm_timeout)."""
        self._check(lib().hmc_set_comm_timeout(self._h, float(seconds)))

    def set_estep_mode(self, mode: int):
        """0 = split E-step (structure pass + value pass, default), 1 = fused kernel."""
        self._check(lib().hmc_set_estep_mode(self._h, int(mode)))

    def estep_split_stats(self) -> dict:
        s1, s2, fb, nf = C.c_double(), C.c_double(), C.c_double(), C.c_int()
        self._check(lib().hmc_last_estep_split(self._h, C.byref(s1), C.byref(s2), C.byref(fb), C.byref(nf)))
        ps, pv = C.c_int(), C.c_int()
        self._check(lib().hmc_last_estep_passes(self._h, C.byref(ps), C.byref(pv)))
        no, om = C.c_int(), C.c_double()
        self._check(lib().hmc_last_estep_order(self._h, C.byref(no), C.byref(om)))
        return dict(structure_ms=s1.value, values_ms=s2.value, fallback_ms=fb.value, n_fallback=nf.value,
                    structure_passes=ps.value, value_passes=pv.value, n_order_rerun=no.value, order_ms=om.value)

    def mine_level(self, start, alleles) -> tuple[np.ndarray, int]:
        """PatternManager::checkFrequency for candidates of one length: start[n],
        alleles[n][level] symbols -> (frequencies, items scanned)."""
        start = np.ascontiguousarray(start, np.int32)
        alleles = np.ascontiguousarray(alleles, np.int32).reshape(len(start), -1)
        freq = np.zeros(len(start))
        sc = C.c_uint64()
        self._check(lib().hmc_mine_level(self._h, alleles.shape[1], len(start), _p(start, C.c_int32),
                                         _p(alleles, C.c_int32), _p(freq, C.c_double), C.byref(sc)))
        return freq, sc.value

    def set_shard(self, i0: int, i1: int):
        """One-rank measurement hook (hmc_set_shard): later E- and M-steps cover
        individuals [i0, i1) of the loaded panel with the current model."""
        self._check(lib().hmc_set_shard(self._h, int(i0), int(i1)))
        self.i0, self.i1 = int(i0), int(i1)

    def set_estep_windows(self, mode: str = "auto", window_loci: int = 0):
        """Windowed E-step (hmc_set_estep_windows): "auto",
        "never" or "always"; window_loci = loci per window (0: from the store
        budgets).  Results are identical."""
        self._check(lib().hmc_set_estep_windows(self._h, {"auto": 0, "never": 1, "always": 2}[mode], int(window_loci)))

    def estep_windows(self) -> dict:
        w, wl, g, ms = C.c_int(), C.c_int(), C.c_int(), C.c_double()
        self._check(lib().hmc_last_estep_windows(self._h, C.byref(w), C.byref(wl), C.byref(g), C.byref(ms)))
        rs, sc = C.c_int(), C.c_double()
        self._check(lib().hmc_last_estep_restarts(self._h, C.byref(rs), C.byref(sc)))
        return dict(windows=w.value, window_loci=wl.value, groups=g.value, collection_ms=ms.value,
                    restarts=rs.value, window_scale=sc.value)

    HOST_PHASES = ("estep", "stores", "gmodel", "samples", "accept", "haplocomp", "mstep", "estep_setup")

    def host_phases(self) -> dict:
        """Host wall ms of the last em_iteration's phases (hmc_last_host_phases)."""
        buf = (C.c_double * len(self.HOST_PHASES))()
        n = lib().hmc_last_host_phases(self._h, buf, len(self.HOST_PHASES))
        if n < 0:
            self._check(n)
        return {k: buf[i] for i, k in enumerate(self.HOST_PHASES)}

    def set_value_mode(self, mode: str):
        """Value pass of the split E-step: "fast" (value-only k-best lists, the
        libstdc++ permutations only for individuals with ties), "exact" (the
        permutations for everyone) or "auto" (default: fast on multi-allelic
        panels once the model is smaller than the panel, exact otherwise and
        after an E-step that re-ran more than 35 %).  Results are identical."""
        self._check(lib().hmc_set_value_mode(self._h, {"fast": 0, "exact": 1, "auto": 2}[mode]))

    def set_value_layout(self, mode: int):
        """Phase-B layout of the value pass (hmc_set_value_layout): two links
        per lane for 0 never, 1 heavy groups, 2 every group (default).  Results
        are identical."""
        self._check(lib().hmc_set_value_layout(self._h, mode))

    def set_value_pass(self, mode: str, ring: int = 0):
        """Value-pass schedule (hmc_set_value_pass): "auto", "classic" (locus
        by locus) or "dataflow"; ring = frontiers kept by the dataflow pass
        (3 or 4, 0 = 3).  Results are identical."""
        self._check(lib().hmc_set_value_pass(self._h, {"auto": 0, "classic": 1, "dataflow": 2}[mode], int(ring)))

    def set_end_order(self, on: bool):
        """Structure pass over the pattern table in end-locus order
        (hmc_set_end_order; default on) or in id order.  Results are identical."""
        self._check(lib().hmc_set_end_order(self._h, int(bool(on))))

    def set_dataflow_waves(self, a_waves: int):
        """A waves of the dataflow value pass (hmc_set_dataflow_waves): 1..8,
        0 = by the launch shape.  Results are identical."""
        self._check(lib().hmc_set_dataflow_waves(self._h, int(a_waves)))

    def set_structure_pass(self, version: int):
        """Structure pass (hmc_set_structure_pass): 1 per-chunk ranking, 2 three
        block scans per locus, 0 automatic.  Results are identical."""
        self._check(lib().hmc_set_structure_pass(self._h, int(version)))

    def set_exact_walk(self, items_per_wave: int):
        """Exact M-step trie walk (hmc_set_exact_walk): 1 the depth-first walk,
        one item per wavefront (default); 4 four items per wavefront and 2 the
        breadth-first lane units (variants library)."""
        self._check(lib().hmc_set_exact_walk(self._h, int(items_per_wave)))

    def last_value_pass_dataflow(self) -> bool:
        d = C.c_int()
        self._check(lib().hmc_last_value_pass(self._h, C.byref(d)))
        return bool(d.value)

    # ----------------------------------------------------------------- panel
    def load(self, genos: GenoData):
        a = np.ascontiguousarray(genos.alleles, dtype=np.int32)
        N, _, L = a.shape
        self._check(lib().hmc_load_genotypes(self._h, N, L, _p(a, C.c_int32), genos.types.encode()))
        self._info()

    def load_phase(self, path: str):
        self._check(lib().hmc_load_phase(self._h, path.encode()))
        self._info()

    def load_files(self, fmt: str, paths: list[str]):
        """HaploFile::getHaploFile(format, names)->readGenoData: PHASE, HPM,
        HPM2 (one file), BENCH2 (genotypes, positions), BENCH3 (genotypes,
        positions, children)."""
        arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
        self._check(lib().hmc_load_files(self._h, fmt.encode(), arr, len(paths)))
        self._info()

    def write_files(self, fmt: str, paths: list[str]):
        """writeGenoData of the accepted resolutions in `fmt`."""
        arr = (C.c_char_p * len(paths))(*[p.encode() for p in paths])
        self._check(lib().hmc_write_files(self._h, fmt.encode(), arr, len(paths)))

    def unphased_num(self) -> int:
        n = C.c_int()
        self._check(lib().hmc_unphased_num(self._h, C.byref(n)))
        return n.value

    def _info(self):
        n, l, a = C.c_int(), C.c_int(), C.c_int()
        self._check(lib().hmc_panel_info(self._h, C.byref(n), C.byref(l), C.byref(a)))
        self.N, self.L, self.amax = n.value, l.value, a.value
        i0, i1 = C.c_int(), C.c_int()
        self._check(lib().hmc_shard_range(self._h, C.byref(i0), C.byref(i1)))
        self.i0, self.i1 = i0.value, i1.value

    def allele_table(self):
        num = np.zeros(self.L, np.int32)
        sym = np.zeros((self.L, self.amax), np.int32)
        fr = np.zeros((self.L, self.amax), np.float64)
        self._check(lib().hmc_allele_table(self._h, _p(num, C.c_int32), _p(sym, C.c_int32), _p(fr, C.c_double)))
        return num, sym, fr

    # ---------------------------------------------------------------- M-step
    def find_patterns(self) -> tuple[int, int]:
        """PatternManager::findPatternByFreq + initialize; returns (patterns, R_M)."""
        self._push_params()
        n, rm = C.c_int(), C.c_uint64()
        self._check(lib().hmc_find_patterns(self._h, C.byref(n), C.byref(rm)))
        return n.value, rm.value

    def exact_stats(self) -> dict:
        r, c, ms = C.c_int(), C.c_uint64(), C.c_double()
        self._check(lib().hmc_last_exact_stats(self._h, C.byref(r), C.byref(c), C.byref(ms)))
        u, la, de, pr = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
        self._check(lib().hmc_last_exact_walk(self._h, C.byref(u), C.byref(la), C.byref(de), C.byref(pr)))
        return dict(rounds=r.value, candidates=c.value, walk_ms=ms.value, walk_units=u.value, walk_launches=la.value,
                    walk_deferred=de.value, pruned=pr.value)

    def head_len(self) -> int:
        """PatternManager::head_len of the current model (min pattern length)."""
        P, hl = C.c_int(), C.c_int()
        self._check(lib().hmc_model_info(self._h, C.byref(P), C.byref(hl)))
        return hl.value

    def patterns(self, maxlen: int | None = None) -> dict:
        P, hl = C.c_int(), C.c_int()
        self._check(lib().hmc_model_info(self._h, C.byref(P), C.byref(hl)))
        P = P.value
        A = self.amax
        ml = min(maxlen or self.L, self.L)
        out = dict(start=np.zeros(P, np.int32), len=np.zeros(P, np.int32), freq=np.zeros(P),
                   prefix=np.zeros(P), tp=np.zeros(P), succ=np.zeros((P, A), np.int32),
                   alleles=np.zeros((P, ml), np.int32))
        self._check(lib().hmc_get_patterns(
            self._h, _p(out["start"], C.c_int32), _p(out["len"], C.c_int32), _p(out["freq"], C.c_double),
            _p(out["prefix"], C.c_double), _p(out["tp"], C.c_double), _p(out["succ"], C.c_int32),
            _p(out["alleles"], C.c_int32), ml))
        return out

    def set_patterns(self, start, length, freq, tp, succ, last_symbol):
        self._push_params()
        start = np.ascontiguousarray(start, np.int32)
        length = np.ascontiguousarray(length, np.int32)
        freq = np.ascontiguousarray(freq, np.float64)
        tp = np.ascontiguousarray(tp, np.float64)
        succ = np.ascontiguousarray(succ, np.int32)
        last = np.ascontiguousarray(last_symbol, np.int32)
        self._check(lib().hmc_set_patterns(self._h, len(start), _p(start, C.c_int32), _p(length, C.c_int32),
                                           _p(freq, C.c_double), _p(tp, C.c_double), _p(succ, C.c_int32),
                                           _p(last, C.c_int32)))

    # ---------------------------------------------------------------- E-step
    def resolve_all(self) -> tuple[float, int, int]:
        """HaploModel::resolveAll; returns (log-likelihood, samples, R_E)."""
        self._push_params()
        ll, H, re = C.c_double(), C.c_int(), C.c_uint64()
        self._check(lib().hmc_resolve_all(self._h, C.byref(ll), C.byref(H), C.byref(re)))
        return ll.value, H.value, re.value

    def estep_results(self) -> dict:
        n = self.i1 - self.i0
        S = max(1, self.sample_size)
        out = dict(total=np.zeros(n), ncand=np.zeros(n, np.int32), status=np.zeros(n, np.int32),
                   prior=np.zeros((n, S)), posterior=np.zeros((n, S)), weight=np.zeros((n, S)))
        self._check(lib().hmc_get_estep(self._h, _p(out["total"], C.c_double), _p(out["ncand"], C.c_int32),
                                        _p(out["status"], C.c_int32), _p(out["prior"], C.c_double),
                                        _p(out["posterior"], C.c_double), _p(out["weight"], C.c_double)))
        return out

    def frontier_max(self) -> np.ndarray:
        out = np.zeros(self.i1 - self.i0, np.int32)
        self._check(lib().hmc_get_estep_stats(self._h, _p(out, C.c_int32)))
        return out

    def estep_cost(self) -> np.ndarray:
        """Per-individual E-step time of the last E-step (units of 1024 shader clocks)."""
        out = np.zeros(self.i1 - self.i0, np.int32)
        self._check(lib().hmc_get_estep_cost(self._h, _p(out, C.c_int32)))
        return out

    def samples(self, H: int):
        al = np.zeros((H, self.L), np.int32)
        w = np.zeros(H)
        tw = C.c_double()
        self._check(lib().hmc_get_samples(self._h, _p(al, C.c_int32), _p(w, C.c_double), C.byref(tw)))
        return al, w, tw.value

    def clear_samples(self):
        self._check(lib().hmc_clear_samples(self._h))

    def resolutions(self) -> np.ndarray:
        out = np.zeros((self.i1 - self.i0, 2, self.L), np.int32)
        self._check(lib().hmc_get_resolutions(self._h, _p(out, C.c_int32)))
        return out

    def timings(self) -> dict:
        f, t, m = C.c_double(), C.c_double(), C.c_double()
        self._check(lib().hmc_last_timings(self._h, C.byref(f), C.byref(t), C.byref(m)))
        return dict(estep_forward_ms=f.value, estep_traceback_ms=t.value, mstep_ms=m.value)

    # ------------------------------------------------------------ whole EM
    def run(self, genos: GenoData | None = None) -> np.ndarray:
        """HaploModel::run: M0, then E/M iterations until the LL stops improving."""
        if genos is not None:
            self.load(genos)
        self._push_params()
        cap = max(1, int(self.max_iteration))
        logs = (IterLog * cap)()
        it, tm0, rm0, np0 = C.c_int(), C.c_double(), C.c_uint64(), C.c_int()
        self._check(lib().hmc_run(self._h, int(self.max_iteration), logs, cap, C.byref(it), C.byref(tm0),
                                  C.byref(rm0), C.byref(np0)))
        self.iterations = it.value
        self.m0 = dict(t_s=tm0.value, r_m=rm0.value, n_patterns=np0.value)
        self.log = [dict(ll=l.log_likelihood, t_e=l.t_estep_s, t_m=l.t_mstep_s, r_e=l.r_e, r_m=l.r_m,
                         n_patterns=l.n_patterns, n_samples=l.n_samples,
                         haplocomp=(l.switch_error, l.ihp, l.igp)) for l in logs[:it.value]]
        out = np.zeros((self.i1 - self.i0, 2, self.L), np.int32)
        self._check(lib().hmc_get_best_resolutions(self._h, _p(out, C.c_int32)))
        return out

    def em_iteration(self, iteration: int, old_ll: float, always_mstep: bool = True,
                     max_iteration: int = 1 << 30) -> tuple[dict, float, bool]:
        """One HaploModel::run iteration (HaploModel.cpp:130-144): E-step, accept,
        HaploComp, continue rule, M-step.  Returns (log, new old_ll, go)."""
        self._push_params()
        ol = C.c_double(old_ll)
        rec = IterLog()
        go = C.c_int()
        self._check(lib().hmc_em_iteration(self._h, int(iteration), int(max_iteration), int(bool(always_mstep)),
                                           C.byref(ol), C.byref(rec), C.byref(go)))
        log = {f: getattr(rec, f) for f, _ in IterLog._fields_}
        return log, ol.value, bool(go.value)

    def haplocomp(self):
        """HaploComp (switch error, IHP, IGP) of the input panel against the
        accepted resolutions of the last run (HaploComp.cpp:29-155)."""
        se, ihp, igp = C.c_double(), C.c_double(), C.c_double()
        self._check(lib().hmc_haplocomp(self._h, C.byref(se), C.byref(ihp), C.byref(igp)))
        return se.value, ihp.value, igp.value

    def write_phase(self, path: str):
        self._check(lib().hmc_write_phase(self._h, path.encode()))
