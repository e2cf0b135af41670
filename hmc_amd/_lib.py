"""ctypes binding of libhmc_amd.so (C-ABI declared in include/hmc_amd.h).

The library is built in-tree by `__graft_entry__.build()` (or `make -C
hmc_amd/csrc`).  There is no fallback: if the shared object is missing or does
not load, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "libhmc_amd.so")
LIB_PATH = os.environ.get("HMC_AMD_LIB") or _DEFAULT_LIB

HMC_OK = 0
ERRORS = {-1: "EARG", -2: "EHIP", -3: "EIO", -4: "EUNSUPPORTED", -5: "ENOPATTERN", -6: "ERCCL", -7: "ENOMEM"}


class HMCError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"hmc_amd error {code} ({ERRORS.get(code, '?')}): {msg}")
        self.code = code


class IterLog(C.Structure):
    _fields_ = [("log_likelihood", C.c_double), ("t_estep_s", C.c_double), ("t_mstep_s", C.c_double),
                ("r_e", C.c_uint64), ("r_m", C.c_uint64), ("n_patterns", C.c_int), ("n_samples", C.c_int),
                ("switch_error", C.c_double), ("ihp", C.c_double), ("igp", C.c_double)]


ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_void_p)

_lib = None

# (name, restype, argtypes)
_P = C.POINTER
_vp, _i, _d, _u64, _cp = C.c_void_p, C.c_int, C.c_double, C.c_uint64, C.c_char_p
_SIGS = [
    ("hmc_version", _cp, []),
    ("hmc_ctx_create", _i, [_i, _P(_vp)]),
    ("hmc_rccl_unique_id", _i, [_vp]),
    ("hmc_ctx_create_dist", _i, [_i, _i, _i, _vp, _P(_vp)]),
    ("hmc_ctx_create_hostcoll", _i, [_i, _i, _i, ALLREDUCE_FN, _vp, _P(_vp)]),
    ("hmc_ctx_create_comm", _i, [_i, _vp, _P(_vp)]),
    ("hmc_rccl_comm_init", _i, [_i, _i, _i, _vp, _P(_vp)]),
    ("hmc_rccl_comm_destroy", _i, [_vp]),
    ("hmc_set_reduction", _i, [_vp, _i]),
    ("hmc_set_force_collectives", _i, [_vp, _i]),
    ("hmc_ctx_destroy", None, [_vp]),
    ("hmc_ctx_error", _cp, [_vp]),
    ("hmc_set_params", _i, [_vp, _d, _d, _i, _i, _i]),
    ("hmc_load_phase", _i, [_vp, _cp]),
    ("hmc_load_genotypes", _i, [_vp, _i, _i, _P(C.c_int32), _cp]),
    ("hmc_panel_info", _i, [_vp, _P(_i), _P(_i), _P(_i)]),
    ("hmc_shard_range", _i, [_vp, _P(_i), _P(_i)]),
    ("hmc_allele_table", _i, [_vp, _P(C.c_int32), _P(C.c_int32), _P(_d)]),
    ("hmc_find_patterns", _i, [_vp, _P(_i), _P(_u64)]),
    ("hmc_model_info", _i, [_vp, _P(_i), _P(_i)]),
    ("hmc_get_patterns", _i, [_vp, _P(C.c_int32), _P(C.c_int32), _P(_d), _P(_d), _P(_d), _P(C.c_int32),
                              _P(C.c_int32), _i]),
    ("hmc_set_patterns", _i, [_vp, _i, _P(C.c_int32), _P(C.c_int32), _P(_d), _P(_d), _P(C.c_int32),
                              _P(C.c_int32)]),
    ("hmc_resolve_all", _i, [_vp, _P(_d), _P(_i), _P(_u64)]),
    ("hmc_get_estep", _i, [_vp, _P(_d), _P(C.c_int32), _P(C.c_int32), _P(_d), _P(_d), _P(_d)]),
    ("hmc_get_estep_stats", _i, [_vp, _P(C.c_int32)]),
    ("hmc_get_estep_cost", _i, [_vp, _P(C.c_int32)]),
    ("hmc_get_stamps", _i, [_vp, _P(C.c_uint64)]),
    ("hmc_set_estep_mode", _i, [_vp, _i]),
    ("hmc_last_estep_split", _i, [_vp, _P(_d), _P(_d), _P(_d), _P(_i)]),
    ("hmc_last_estep_passes", _i, [_vp, _P(_i), _P(_i)]),
    ("hmc_set_value_mode", _i, [_vp, _i]),
    ("hmc_set_value_layout", _i, [_vp, _i]),
    ("hmc_set_value_pass", _i, [_vp, _i, _i]),
    ("hmc_set_structure_pass", _i, [_vp, _i]),
    ("hmc_set_dataflow_waves", _i, [_vp, _i]),
    ("hmc_set_end_order", _i, [_vp, _i]),
    ("hmc_set_exact_walk", _i, [_vp, _i]),
    ("hmc_last_value_pass", _i, [_vp, _P(_i)]),
    ("hmc_mine_level", _i, [_vp, _i, _i, _P(C.c_int32), _P(C.c_int32), _P(_d), _P(_u64)]),
    ("hmc_last_estep_order", _i, [_vp, _P(_i), _P(_d)]),
    ("hmc_get_samples", _i, [_vp, _P(C.c_int32), _P(_d), _P(_d)]),
    ("hmc_get_resolutions", _i, [_vp, _P(C.c_int32)]),
    ("hmc_clear_samples", _i, [_vp]),
    ("hmc_run", _i, [_vp, _i, _P(IterLog), _i, _P(_i), _P(_d), _P(_u64), _P(_i)]),
    ("hmc_em_iteration", _i, [_vp, _i, _i, _i, _P(_d), _P(IterLog), _P(_i)]),
    ("hmc_get_best_resolutions", _i, [_vp, _P(C.c_int32)]),
    ("hmc_haplocomp", _i, [_vp, _P(_d), _P(_d), _P(_d)]),
    ("hmc_set_model", _i, [_vp, _cp, _i]),
    ("hmc_set_num_patterns", _i, [_vp, _i]),
    ("hmc_set_exact_estimate", _i, [_vp, _i]),
    ("hmc_last_exact_stats", _i, [_vp, _P(_i), _P(_u64), _P(_d)]),
    ("hmc_parse_file", _i, [_cp, _cp, _cp, _P(_i), _P(_i), _P(C.c_int32), _cp]),
    ("hmc_load_file", _i, [_vp, _cp, _cp, _cp]),
    ("hmc_write_file", _i, [_vp, _cp, _cp, _cp]),
    ("hmc_parse_files", _i, [_cp, _P(_cp), _i, _P(_i), _P(_i), _P(C.c_int32), _cp, _P(_i)]),
    ("hmc_load_files", _i, [_vp, _cp, _P(_cp), _i]),
    ("hmc_write_files", _i, [_vp, _cp, _P(_cp), _i]),
    ("hmc_unphased_num", _i, [_vp, _P(_i)]),
    ("hmc_write_patterns", _i, [_vp, _cp]),
    ("hmc_write_phase", _i, [_vp, _cp]),
    ("hmc_set_tuning", _i, [_vp, _i, _u64, _i]),
    ("hmc_set_estep_shape", _i, [_vp, _i, _i]),
    ("hmc_set_pass_shapes", _i, [_vp, _i, _i, _i, _i]),
    ("hmc_set_store_budgets", _i, [_vp, _u64, _u64]),
    ("hmc_set_mine_block", _i, [_vp, _i]),
    ("hmc_set_mine_memory", _i, [_vp, C.c_uint64]),
    ("hmc_last_estep_frontier", _i, [_vp, _P(C.c_int), _P(C.c_int)]),
    ("hmc_last_mine_stats", _i, [_vp, _P(_i), _P(C.c_int64), _P(_d)]),
    ("hmc_last_mine_reduction", _i, [_vp, _P(_d), _P(_i)]),
    ("hmc_comm_stats", _i, [_vp, _P(C.c_int64), _P(C.c_int64), _P(C.c_uint64)]),
    ("hmc_set_comm_timeout", _i, [_vp, _d]),
    ("hmc_set_key_probes", _i, [_vp, _i]),
    ("hmc_set_structure_tier", _i, [_vp, _i, _i]),
    ("hmc_debug_stall", _i, [_vp, _d]),
    ("hmc_set_estep_windows", _i, [_vp, _i, _i]),
    ("hmc_set_shard", _i, [_vp, _i, _i]),
    ("hmc_last_exact_walk", _i, [_vp, _P(C.c_int64), _P(C.c_int64), _P(C.c_int64), _P(_i)]),
    ("hmc_last_estep_windows", _i, [_vp, _P(_i), _P(_i), _P(_i), _P(_d)]),
    ("hmc_last_estep_restarts", _i, [_vp, _P(_i), _P(_d)]),
    ("hmc_last_host_phases", _i, [_vp, _P(_d), _i]),
    ("hmc_model_save", _i, [_vp]),
    ("hmc_em_rewind", _i, [_vp]),
    ("hmc_build_info", _cp, []),
    ("hmc_last_timings", _i, [_vp, _P(_d), _P(_d), _P(_d)]),
    ("hmc_test_nth_element", None, [_P(_d), _P(C.c_uint32), _i, _i]),
    ("hmc_test_sort_small", None, [_P(_d), _P(C.c_uint32), _i]),
    ("hmc_test_sort", None, [_P(_d), _P(C.c_uint32), _i]),
    ("hmc_test_nth_element_masks", None, [_P(_d), _P(C.c_uint32), _i, _i]),
    ("hmc_test_coop_nth_element", _i, [_i, _P(_d), _P(C.c_uint32), _P(C.c_int32), _P(C.c_int32), _P(C.c_int32),
                                       _i, _i, _i]),
]

EXPORTED = [s[0] for s in _SIGS]


def lib_identity() -> dict:
    """Which libhmc_amd.so this process loaded: path, SHA-256 prefix of the
    file and the library's own build string."""
    import hashlib

    L = lib()
    with open(LIB_PATH, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    return {"path": os.path.relpath(LIB_PATH, os.path.dirname(_HERE)), "sha256_16": sha,
            "build": L.hmc_build_info().decode()}


def lib():
    """Load libhmc_amd.so; raises if it is absent (no CPU fallback exists)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built; run __graft_entry__.build() or make -C hmc_amd/csrc")
        L = C.CDLL(LIB_PATH)
        # an older build picked with HMC_AMD_LIB (A/B runs) may lack newer
        # entry points; the in-tree product library must export every one
        ab = "HMC_AMD_LIB" in os.environ and os.path.abspath(LIB_PATH) != os.path.abspath(_DEFAULT_LIB)
        for name, res, args in _SIGS:
            try:
                f = getattr(L, name)
            except AttributeError:
                if ab:
                    continue
                raise
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib
