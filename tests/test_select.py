"""The E-step's libstdc++-exact k-best selection (hmc_amd/csrc/select.hpp),
run on the host through the library's test hooks, against the real
std::nth_element / std::sort compiled into the CPU restatement."""
import ctypes as C

import numpy as np
import pytest

import hmc_amd


def _ours(fn, lik, tag, *extra):
    l = np.ascontiguousarray(lik, np.float64).copy()
    t = np.ascontiguousarray(tag, np.uint32).copy()
    fn(l.ctypes.data_as(C.POINTER(C.c_double)), t.ctypes.data_as(C.POINTER(C.c_uint32)), len(l), *extra)
    return l, t.astype(np.int32)


def _cases(rng, n):
    yield rng.random(n)
    yield rng.integers(0, 3, n).astype(np.float64)          # heavy ties
    yield np.zeros(n)                                        # all equal
    yield np.arange(n, dtype=np.float64)                     # ascending
    yield np.arange(n, dtype=np.float64)[::-1].copy()        # descending
    v = np.concatenate([np.arange(n // 2), np.arange(n - n // 2)[::-1]]).astype(np.float64)
    yield v                                                  # organ pipe
    w = rng.integers(0, 4, n).astype(np.float64) * 1e-300
    w[rng.integers(0, n)] = np.nan
    yield w                                                  # denormal-ish ties + NaN


@pytest.mark.parametrize("n", list(range(1, 21)) + [24, 32, 33, 64, 100, 257])
def test_nth_element_matches_libstdcxx(oracle_mod, n):
    L = hmc_amd.lib()
    rng = np.random.default_rng(n)
    for lik in _cases(rng, n):
        for nth in sorted({0, n // 2, n - 1, max(0, n - 2)}):
            tag = np.arange(n, dtype=np.int32)
            l1, t1 = _ours(L.hmc_test_nth_element, lik, tag, nth)
            l2, t2 = oracle_mod.std_nth_element(lik, tag, nth)
            assert np.array_equal(t1, t2), (n, nth, lik)


@pytest.mark.parametrize("n", list(range(1, 33)))
def test_mask_partition_nth_element_matches_libstdcxx(oracle_mod, n):
    """The stop-mask formulation of the Hoare partition (select.hpp,
    partition_pivot_masks) used by the E-step kernel gives the identical
    permutation."""
    L = hmc_amd.lib()
    rng = np.random.default_rng(500 + n)
    for rep in range(40):
        for lik in _cases(rng, n):
            nth = int(rng.integers(0, n))
            tag = np.arange(n, dtype=np.int32)
            _, t1 = _ours(L.hmc_test_nth_element_masks, lik, tag, nth)
            _, t2 = oracle_mod.std_nth_element(lik, tag, nth)
            assert np.array_equal(t1, t2), (n, nth, lik)


@pytest.mark.parametrize("n", range(0, 17))
def test_small_sort_matches_libstdcxx(oracle_mod, n):
    L = hmc_amd.lib()
    rng = np.random.default_rng(100 + n)
    for lik in _cases(rng, max(n, 1)):
        lik = lik[:n]
        tag = np.arange(n, dtype=np.int32)
        _, t1 = _ours(L.hmc_test_sort_small, lik, tag)
        _, t2 = oracle_mod.std_sort(lik, tag)
        assert np.array_equal(t1, t2)


@pytest.mark.parametrize("n", list(range(0, 70)) + [100, 257, 1000])
def test_sort_matches_libstdcxx(oracle_mod, n):
    """std::sort for any n (select.hpp sort_greater: introsort with the
    threshold 16, heap sort at depth 0, final insertion sort) — the final
    candidate order when sample_size > 16."""
    L = hmc_amd.lib()
    rng = np.random.default_rng(300 + n)
    for rep in range(4):
        for ci, lik in enumerate(_cases(rng, max(n, 1))):
            if ci == 6:  # NaN: std::sort's unguarded loops need a strict weak order
                continue
            lik = lik[:n]
            tag = np.arange(n, dtype=np.int32)
            _, t1 = _ours(L.hmc_test_sort, lik, tag)
            _, t2 = oracle_mod.std_sort(lik, tag)
            assert np.array_equal(t1, t2), (n, ci)
