"""ol_dsp_amd -- MI355X-native bulk audio-effect engine (gfx950 HIP kernels behind a C-ABI).

The product is ``libolfx.so`` (ol_dsp_amd/csrc -> ol_dsp_amd/libolfx.so, C-ABI in
include/olfx.h).  This package is the thin Python mirror of that boundary used by tests and
bench.py; it never computes audio on the CPU.
"""
from ._lib import (IO_DEVICE, IO_HOST, KIND_CHAIN, KIND_CHORUS, KIND_DATTORRO, KIND_FXRACK, KIND_PITCHSHIFT,
                   KIND_VOICE, KIND_VOICE_MOOG, LIB_PATH, OlfxError, load)
from .engine import KIND_NAMES, PARAMS, Engine, Polyvoice, control_map, kind_info

__all__ = [
    "Engine", "Polyvoice", "OlfxError", "PARAMS", "KIND_NAMES", "kind_info", "control_map", "load", "LIB_PATH",
    "KIND_DATTORRO", "KIND_CHORUS", "KIND_PITCHSHIFT", "KIND_VOICE", "KIND_CHAIN", "KIND_FXRACK", "KIND_VOICE_MOOG",
    "IO_DEVICE", "IO_HOST",
]
