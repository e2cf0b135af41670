"""hmc_amd — MI355X-native HaploModel EM (Wu-Lab/HMC hot path) over libhmc_amd.so."""
from ._lib import HMCError, lib, lib_identity  # noqa: F401
from .model import GenoData, HaploModel  # noqa: F401
from . import synth  # noqa: F401

__all__ = ["HaploModel", "GenoData", "HMCError", "lib", "lib_identity", "synth"]
