"""The C-ABI library loads on a GPU-less host and exports every entry point
declared in include/hmc_amd.h; without a device it fails loudly."""
import os
import re

import pytest

import hmc_amd
from hmc_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    txt = open(os.path.join(ROOT, "include", "hmc_amd.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(hmc_[a-z0-9_]+)\s*\(", txt)) - {"hmc_allreduce_fn"})


def test_header_symbols_exported():
    L = hmc_amd.lib()
    names = declared_functions()
    assert len(names) >= 25
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing


def test_binding_covers_header():
    assert set(declared_functions()) <= set(_lib.EXPORTED)


def test_version_string():
    assert b"gfx950" in hmc_amd.lib().hmc_version()


def test_no_silent_cpu_fallback():
    import torch

    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(hmc_amd.HMCError) as e:
        hmc_amd.HaploModel()
    assert e.value.code == -2  # HMC_EHIP


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(_lib, "_lib", None)
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "nope.so"))
    with pytest.raises(ImportError):
        _lib.lib()
