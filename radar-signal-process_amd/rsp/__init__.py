"""rsp -- MI355X range-Doppler engine (PC -> MTD -> 0-v -> 2-D CA-CFAR), host side.

The compute lives in lib/librsp.so (HIP kernels for gfx950 behind the C ABI of
include/rsp.h); this package is the Python mirror of the reference's MATLAB interface
(rsp.matlab), parameter presets (rsp.presets), the Engine wrapper (rsp.engine) and the
deterministic synthetic-echo generator (rsp.synth).
"""
from . import _capi, presets, synth  # noqa: F401
from ._capi import RspError, load_library  # noqa: F401
from .engine import Engine, engine_for  # noqa: F401

__version__ = "0.3.0"
