"""ctypes binding of the CPU restatement (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package hmc_amd.
Parity unpinned (see hmc_oracle.cpp header and DESIGN.md §Oracle).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "liboracle.so")
_lib = None


def build() -> str:
    src = os.path.join(_HERE, "hmc_oracle.cpp")
    if not os.path.exists(_LIB) or os.path.getmtime(_LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE, "liboracle.so"])
    return _LIB


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB)
        vp, i, d, u64 = C.c_void_p, C.c_int, C.c_double, C.c_uint64
        P = C.POINTER
        L.ora_create.restype = vp
        L.ora_create.argtypes = [i, i, P(i), C.c_char_p]
        L.ora_create_from_phase.restype = vp
        L.ora_create_from_phase.argtypes = [C.c_char_p]
        L.ora_destroy.argtypes = [vp]
        L.ora_skip_count_range.restype = C.c_uint64
        L.ora_skip_count_range.argtypes = [vp, C.c_int, C.c_int]
        L.ora_set_params.argtypes = [vp, d, i, i, i, i]
        L.ora_dims.argtypes = [vp, P(i), P(i), P(i)]
        L.ora_allele_table.argtypes = [vp, i, P(i), P(i), P(d)]
        L.ora_genotypes.argtypes = [vp, P(i)]
        L.ora_find_patterns.restype = i
        L.ora_find_patterns.argtypes = [vp]
        L.ora_pattern_count.restype = i
        L.ora_pattern_count.argtypes = [vp]
        L.ora_head_len.restype = i
        L.ora_head_len.argtypes = [vp]
        L.ora_patterns.argtypes = [vp, i, i, P(i), P(i), P(d), P(d), P(d), P(i), P(i)]
        L.ora_resolve_all.restype = d
        L.ora_resolve_all.argtypes = [vp]
        L.ora_tie_flags.argtypes = [vp, P(i)]
        L.ora_set_threads.argtypes = [i]
        L.ora_set_unphased.argtypes = [vp, i]
        L.ora_set_exact.argtypes = [vp, i]
        L.ora_set_exact_order.argtypes = [vp, i]
        L.ora_estimate_patterns.restype = i
        L.ora_estimate_patterns.argtypes = [vp, P(u64)]
        L.ora_set_model.argtypes = [vp, i, i]
        L.ora_set_num_patterns.argtypes = [vp, i]
        L.ora_run_comp_log.argtypes = [vp, P(d)]
        L.ora_haplocomp.restype = i
        L.ora_haplocomp.argtypes = [vp, P(i), P(d)]
        L.ora_sample_count.restype = i
        L.ora_sample_count.argtypes = [vp]
        L.ora_total_weight.restype = d
        L.ora_total_weight.argtypes = [vp]
        L.ora_samples.argtypes = [vp, P(i), P(d)]
        L.ora_estep_summary.argtypes = [vp, P(i), P(d)]
        L.ora_candidate.restype = i
        L.ora_candidate.argtypes = [vp, i, i, P(i), P(d), P(d)]
        L.ora_resolutions.argtypes = [vp, P(i)]
        L.ora_counters.argtypes = [vp, P(u64), P(u64)]
        L.ora_reset_counters.argtypes = [vp]
        L.ora_run.restype = i
        L.ora_run.argtypes = [vp]
        L.ora_run_log.argtypes = [vp, P(d), P(u64), P(u64), P(i), P(d), P(d), P(d)]
        L.ora_best_resolutions.argtypes = [vp, P(i)]
        L.ora_std_nth_element.argtypes = [P(d), P(i), i, i]
        L.ora_std_sort.argtypes = [P(d), P(i), i]
        L.ora_set_patterns.restype = i
        L.ora_set_patterns.argtypes = [vp, i, P(i), P(i), P(i), i, P(d), P(d), P(d), P(i), i]
        L.ora_time_resolve_range.restype = d
        L.ora_time_resolve_range.argtypes = [vp, i, i]
        L.ora_set_samples.argtypes = [vp, i, P(i), P(d)]
        L.ora_time_find_patterns.restype = d
        L.ora_time_find_patterns.argtypes = [vp]
        L.ora_time_find_patterns_roots.restype = d
        L.ora_time_find_patterns_roots.argtypes = [vp, i, i]
        L.ora_time_resolve_list.restype = d
        L.ora_time_resolve_list.argtypes = [vp, P(i), i]
        L.ora_time_best_pair_reset.restype = d
        L.ora_time_best_pair_reset.argtypes = [C.c_longlong, i]
        L.ora_time_find_patterns_root_list.restype = d
        L.ora_time_find_patterns_root_list.argtypes = [vp, P(i), i]
        L.ora_resolve_range.restype = d
        L.ora_resolve_range.argtypes = [vp, i, i]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class Oracle:
    """Single-threaded CPU restatement of HaploModel (MV, sampling EM)."""

    def __init__(self, alleles: np.ndarray | None = None, types: str | None = None,
                 phase_path: str | None = None, min_freq_abs=1.5, min_len=1, max_len=30,
                 sample_size=10, max_iter=1):
        L = lib()
        if phase_path is not None:
            self.h = L.ora_create_from_phase(phase_path.encode())
            if not self.h:
                raise IOError(phase_path)
        else:
            a = np.ascontiguousarray(alleles, dtype=np.int32)
            N, _, Lc = a.shape
            self.h = L.ora_create(N, Lc, _p(a, C.c_int), (types or "S" * Lc).encode())
        self.set_params(min_freq_abs, min_len, max_len, sample_size, max_iter)
        n, l, am = C.c_int(), C.c_int(), C.c_int()
        L.ora_dims(self.h, C.byref(n), C.byref(l), C.byref(am))
        self.N, self.L, self.amax = n.value, l.value, am.value

    def __del__(self):
        if getattr(self, "h", None) and _lib is not None:
            _lib.ora_destroy(self.h)
            self.h = None

    def set_params(self, min_freq_abs=1.5, min_len=1, max_len=30, sample_size=10, max_iter=1):
        self.max_len = max_len if max_len > 0 else 0
        lib().ora_set_params(self.h, min_freq_abs, min_len, max_len, sample_size, max_iter)

    def allele_table(self):
        num = np.zeros(self.L, np.int32)
        sym = np.zeros((self.L, self.amax), np.int32)
        fr = np.zeros((self.L, self.amax), np.float64)
        lib().ora_allele_table(self.h, self.amax, _p(num, C.c_int), _p(sym, C.c_int), _p(fr, C.c_double))
        return num, sym, fr

    def genotypes(self):
        out = np.zeros((self.N, 2, self.L), np.int32)
        lib().ora_genotypes(self.h, _p(out, C.c_int))
        return out

    def find_patterns(self) -> int:
        return lib().ora_find_patterns(self.h)

    def head_len(self) -> int:
        return lib().ora_head_len(self.h)

    def patterns(self, maxlen: int | None = None) -> dict:
        P = lib().ora_pattern_count(self.h)
        A = self.amax
        start = np.zeros(P, np.int32)
        ln = np.zeros(P, np.int32)
        fr = np.zeros(P, np.float64)
        pre = np.zeros(P, np.float64)
        tp = np.zeros(P, np.float64)
        succ = np.zeros((P, A), np.int32)
        ml = maxlen or max(1, self.L)
        ml = min(ml, self.L)
        al = np.zeros((P, ml), np.int32)
        lib().ora_patterns(self.h, A, ml, _p(start, C.c_int), _p(ln, C.c_int), _p(fr, C.c_double),
                           _p(pre, C.c_double), _p(tp, C.c_double), _p(succ, C.c_int), _p(al, C.c_int))
        return dict(start=start, len=ln, freq=fr, prefix=pre, tp=tp, succ=succ, alleles=al)

    def set_patterns(self, pt: dict):
        al = np.ascontiguousarray(pt["alleles"], np.int32)
        succ = np.ascontiguousarray(pt["succ"], np.int32)
        P = len(pt["start"])
        a = lambda x, t: np.ascontiguousarray(x, t)
        lib().ora_set_patterns(self.h, P, _p(a(pt["start"], np.int32), C.c_int), _p(a(pt["len"], np.int32), C.c_int),
                               _p(al, C.c_int), al.shape[1], _p(a(pt["freq"], np.float64), C.c_double),
                               _p(a(pt["prefix"], np.float64), C.c_double), _p(a(pt["tp"], np.float64), C.c_double),
                               _p(succ, C.c_int), succ.shape[1])

    def time_resolve_range(self, i0: int, i1: int) -> float:
        return lib().ora_time_resolve_range(self.h, i0, i1)

    def set_samples(self, al: np.ndarray, w: np.ndarray):
        al = np.ascontiguousarray(al, np.int32)
        w = np.ascontiguousarray(w, np.float64)
        lib().ora_set_samples(self.h, al.shape[0], _p(al, C.c_int), _p(w, C.c_double))

    def time_find_patterns(self) -> float:
        return lib().ora_time_find_patterns(self.h)

    def time_find_patterns_roots(self, s0: int, s1: int) -> float:
        """Seconds of searchPattern + initialize over the start loci [s0, s1)."""
        return lib().ora_time_find_patterns_roots(self.h, s0, s1)

    def time_resolve_list(self, ids) -> float:
        """Seconds of HaploBuilder::resolve over the listed individuals."""
        a = np.ascontiguousarray(ids, np.int32)
        return lib().ora_time_resolve_list(self.h, _p(a, C.c_int), len(a))

    @staticmethod
    def time_best_pair_reset(P: int, reps: int = 3) -> float:
        """Seconds of HaploBuilder::initialize's per-individual clear of P
        maps (HaploBuilder.cpp:25-33), which resolve() here does not repeat."""
        return lib().ora_time_best_pair_reset(int(P), int(reps))

    def time_find_patterns_root_list(self, roots) -> float:
        """Seconds of searchPattern + initialize over the listed start loci."""
        a = np.ascontiguousarray(sorted(roots), np.int32)
        return lib().ora_time_find_patterns_root_list(self.h, _p(a, C.c_int), len(a))

    def resolve_range(self, i0: int, i1: int) -> float:
        return lib().ora_resolve_range(self.h, i0, i1)

    def resolve_all(self) -> float:
        return lib().ora_resolve_all(self.h)

    def set_model(self, model: str = "MV", mc_order: int = 1):
        """HaploModel::setModel: MV (default), MC (Markov chain of order
        mc_order: all patterns of length mc_order+1), MA (MV + range checks)."""
        lib().ora_set_model(self.h, {"MV": 0, "MC": 1, "MA": 2}[model], int(mc_order))

    def set_exact(self, on: bool = True):
        """HaploModel::exact_estimate (--exact-estimate): M-steps by estimatePatterns."""
        lib().ora_set_exact(self.h, 1 if on else 0)

    def set_exact_order(self, mode: str):
        """Summation order of the exact M-step: "device" (the walk of
        hmc_amd's exact.hip, bit-exact) or "reference" (HaploBuilder.cpp:334-450's
        list-0/1/2 grouping in double, predecessors in creation order)."""
        lib().ora_set_exact_order(self.h, {"device": 0, "reference": 1}[mode])

    def estimate_patterns(self):
        """One exact M-step (PatternManager::estimatePatterns) after an E-step;
        returns (patterns, match-list entries visited)."""
        rx = C.c_uint64()
        P = lib().ora_estimate_patterns(self.h, C.byref(rx))
        return P, rx.value

    def set_unphased(self, n: int):
        """GenoData::unphased_num: HaploComp covers individuals [0, n) (BENCH3 parents)."""
        lib().ora_set_unphased(self.h, int(n))

    def set_num_patterns(self, n: int):
        """HaploModel::num_patterns: > 0 mines with findPatternByNum."""
        lib().ora_set_num_patterns(self.h, int(n))

    def skip_counts(self) -> np.ndarray:
        """Per individual: pairs extend() skipped because their forward
        likelihood is 0 (HaploBuilder.cpp:237) when resolved with the current
        model (diagnostic of the tests' underflow panels)."""
        return np.array([lib().ora_skip_count_range(self.h, i, i + 1) for i in range(self.N)], np.uint64)

    def tie_flags(self) -> np.ndarray:
        """Per-individual tie diagnostics of the last E-step (Model::tie_flags)."""
        out = np.zeros(self.N, np.int32)
        lib().ora_tie_flags(self.h, _p(out, C.c_int))
        return out

    def samples(self):
        H = lib().ora_sample_count(self.h)
        al = np.zeros((H, self.L), np.int32)
        w = np.zeros(H, np.float64)
        lib().ora_samples(self.h, _p(al, C.c_int), _p(w, C.c_double))
        return al, w, lib().ora_total_weight(self.h)

    def estep_summary(self):
        nc = np.zeros(self.N, np.int32)
        gp = np.zeros(self.N, np.float64)
        lib().ora_estep_summary(self.h, _p(nc, C.c_int), _p(gp, C.c_double))
        return nc, gp

    def candidate(self, i: int, c: int):
        hap = np.zeros((2, self.L), np.int32)
        pr, po = C.c_double(), C.c_double()
        rc = lib().ora_candidate(self.h, i, c, _p(hap, C.c_int), C.byref(pr), C.byref(po))
        if rc:
            raise IndexError((i, c))
        return hap, pr.value, po.value

    def resolutions(self):
        out = np.zeros((self.N, 2, self.L), np.int32)
        lib().ora_resolutions(self.h, _p(out, C.c_int))
        return out

    def counters(self):
        re, rm = C.c_uint64(), C.c_uint64()
        lib().ora_counters(self.h, C.byref(re), C.byref(rm))
        return re.value, rm.value

    def reset_counters(self):
        lib().ora_reset_counters(self.h)

    def run(self) -> dict:
        it = lib().ora_run(self.h)
        ll = np.zeros(it, np.float64)
        re = np.zeros(it, np.uint64)
        rm = np.zeros(it + 1, np.uint64)
        npat = np.zeros(it + 1, np.int32)
        te = np.zeros(it, np.float64)
        tm = np.zeros(it, np.float64)
        tm0 = C.c_double()
        lib().ora_run_log(self.h, _p(ll, C.c_double), _p(re, C.c_uint64), _p(rm, C.c_uint64),
                          _p(npat, C.c_int), _p(te, C.c_double), _p(tm, C.c_double), C.byref(tm0))
        best = np.zeros((self.N, 2, self.L), np.int32)
        lib().ora_best_resolutions(self.h, _p(best, C.c_int))
        comp = np.zeros((it, 3), np.float64)
        lib().ora_run_comp_log(self.h, _p(comp, C.c_double))
        n_m = max(0, it - 1) if len(ll) and np.isfinite(ll).all() else max(0, it - 1)
        return dict(iterations=it, ll=ll, R_E=re, R_M=rm, n_patterns=npat, t_e=te, t_m=tm,
                    t_m0=tm0.value, resolutions=best, n_m=n_m, haplocomp=comp)

    def haplocomp(self, infer: np.ndarray):
        """HaploComp (switch error, IHP, IGP) of the input panel against
        infer[N][2][L] symbols, or None where the reference exits on
        inconsistent genotypes."""
        f = np.ascontiguousarray(infer, np.int32)
        out = np.zeros(3, np.float64)
        rc = lib().ora_haplocomp(self.h, _p(f, C.c_int), _p(out, C.c_double))
        return None if rc else out


def set_threads(n: int):
    """Worker threads of mining, successors and resolveAll (results do not
    depend on it; used by the full-size digest generators)."""
    lib().ora_set_threads(int(n))


def std_nth_element(lik: np.ndarray, tag: np.ndarray, nth: int):
    lik = np.ascontiguousarray(lik, np.float64).copy()
    tag = np.ascontiguousarray(tag, np.int32).copy()
    lib().ora_std_nth_element(_p(lik, C.c_double), _p(tag, C.c_int), len(lik), nth)
    return lik, tag


def std_sort(lik: np.ndarray, tag: np.ndarray):
    lik = np.ascontiguousarray(lik, np.float64).copy()
    tag = np.ascontiguousarray(tag, np.int32).copy()
    lib().ora_std_sort(_p(lik, C.c_double), _p(tag, C.c_int), len(lik))
    return lik, tag
