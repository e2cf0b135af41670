"""hmc_amd — MI355X-native HaploModel EM (Wu-Lab/HMC hot path) over libhmc_amd.so."""
from ._lib import HMCError, lib  # noqa: F401
from .model import GenoData, HaploModel  # noqa: F401
from . import synth  # noqa: F401

__all__ = ["HaploModel", "GenoData", "HMCError", "lib", "synth"]
