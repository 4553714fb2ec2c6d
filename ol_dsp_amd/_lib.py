"""ctypes binding of libolfx.so (include/olfx.h).

This is the Python mirror of the C-ABI a maintainer would bind from the reference side
(INTEGRATION.md).  It loads the in-tree ``ol_dsp_amd/libolfx.so`` and fails loudly if it is
missing: there is no CPU fallback anywhere in the product.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# OLFX_LIB may point at an experimental build of the same library (tools/, A/B timing only)
LIB_PATH = os.environ.get("OLFX_LIB") or os.path.join(_HERE, "libolfx.so")

# status codes (olfx.h)
OLFX_OK = 0
OLFX_E_ARG = -1
OLFX_E_NOMEM = -2
OLFX_E_HIP = -3
OLFX_E_NODEVICE = -4
OLFX_E_KIND = -5
OLFX_E_STATE = -6

# kinds
KIND_DATTORRO = 1
KIND_CHORUS = 2
KIND_PITCHSHIFT = 3
KIND_VOICE = 4
KIND_CHAIN = 5
KIND_FXRACK = 6
KIND_VOICE_MOOG = 7

IO_DEVICE = 0
IO_HOST = 1

EV_NOTE_OFF = 0
EV_NOTE_ON = 1


class OlfxError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"olfx error {code}: {msg}")
        self.code = code


class KindInfo(ctypes.Structure):
    _fields_ = [
        ("kind", ctypes.c_int),
        ("n_params", ctypes.c_uint32),
        ("in_channels", ctypes.c_uint32),
        ("out_channels", ctypes.c_uint32),
        ("state_bytes_per_instance", ctypes.c_uint64),
    ]


class Event(ctypes.Structure):
    _fields_ = [
        ("inst", ctypes.c_uint32),
        ("type", ctypes.c_uint8),
        ("note", ctypes.c_uint8),
        ("velocity", ctypes.c_uint8),
        ("pad", ctypes.c_uint8),
    ]


class VoiceEvent(ctypes.Structure):
    _fields_ = [
        ("inst", ctypes.c_uint32),
        ("type", ctypes.c_uint8),
        ("note", ctypes.c_uint8),
        ("velocity", ctypes.c_uint8),
        ("pad", ctypes.c_uint8),
        ("value", ctypes.c_float),
    ]


EV_NOTE_OFF, EV_NOTE_ON, EV_GATE_ON, EV_GATE_OFF, EV_SET_FREQUENCY = 0, 1, 2, 3, 4


class ControlEvent(ctypes.Structure):
    _fields_ = [
        ("inst", ctypes.c_uint32),
        ("control", ctypes.c_uint8),
        ("source", ctypes.c_uint8),
        ("pad", ctypes.c_uint16),
        ("value", ctypes.c_float),
    ]


CTL_MIDI = 0
CTL_HARDWARE = 1
IGNORED = 1
FIELD_UPDATE_ONLY = 0xFFFFFFFF

# every symbol include/olfx.h declares, with (restype, argtypes)
_P = ctypes.c_void_p
_U32 = ctypes.c_uint32
_F = ctypes.c_float
SIGNATURES = {
    "olfx_abi_version": (ctypes.c_int, []),
    "olfx_kind_info_get": (ctypes.c_int, [ctypes.c_int, _F, ctypes.POINTER(KindInfo)]),
    "olfx_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_int, _U32, _F, _U32, ctypes.POINTER(_P)]),
    "olfx_destroy": (ctypes.c_int, [_P]),
    "olfx_reset": (ctypes.c_int, [_P]),
    "olfx_set_params": (ctypes.c_int, [_P, _U32, _U32, _U32, _U32, ctypes.POINTER(_F)]),
    "olfx_set_param": (ctypes.c_int, [_P, _U32, _U32, _F]),
    "olfx_set_member": (ctypes.c_int, [_P, _U32, _U32, _F]),
    "olfx_set_param_list": (ctypes.c_int, [_P, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_F), _U32]),
    "olfx_get_param": (ctypes.c_int, [_P, _U32, _U32, ctypes.POINTER(_F)]),
    "olfx_note_events": (ctypes.c_int, [_P, ctypes.POINTER(Event), _U32]),
    "olfx_voice_events": (ctypes.c_int, [_P, ctypes.POINTER(VoiceEvent), _U32]),
    "olfx_update": (ctypes.c_int, [_P, _U32, _U32]),
    "olfx_control_map": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint8, ctypes.c_int, _F, ctypes.POINTER(_U32),
                                        ctypes.POINTER(_F)]),
    "olfx_control": (ctypes.c_int, [_P, ctypes.POINTER(ControlEvent), _U32]),
    "olfx_process": (ctypes.c_int, [_P, _P, _P, _U32, ctypes.c_int, _P]),
    "olfx_sync": (ctypes.c_int, [_P]),
    "olfx_stream": (_P, [_P]),
    "olfx_num_instances": (_U32, [_P]),
    "olfx_kind": (ctypes.c_int, [_P]),
    "olfx_frames_processed": (ctypes.c_uint64, [_P]),
    "olfx_algorithmic_bytes_per_frame": (ctypes.c_double, [_P]),
    "olfx_algorithmic_read_bytes_per_frame": (ctypes.c_double, [_P]),
    "olfx_kernel_name": (ctypes.c_char_p, [_P]),
    "olfx_last_error": (ctypes.c_char_p, [_P]),
    "olfx_mix_config": (ctypes.c_int, [_P, _U32, ctypes.POINTER(_U32), ctypes.POINTER(_U32)]),
    "olfx_mix": (ctypes.c_int, [_P, _P, _P, _U32, ctypes.c_int, _P]),
    "olfx_num_buses": (_U32, [_P]),
    # include/olfx_sample.h: per-instance, per-sample operators (one block of latency)
    "olfx_sample_pool_config": (ctypes.c_int, [ctypes.c_int, _U32]),
    "olfx_sample_pool_config_depth": (ctypes.c_int, [ctypes.c_int, _U32, _U32]),
    "olfx_sample_create": (ctypes.c_int, [ctypes.c_int, _F, ctypes.POINTER(_P)]),
    "olfx_sample_destroy": (ctypes.c_int, [_P]),
    "olfx_sample_set_param": (ctypes.c_int, [_P, _U32, _F]),
    "olfx_sample_set_member": (ctypes.c_int, [_P, _U32, _F]),
    "olfx_sample_note": (ctypes.c_int, [_P, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8]),
    "olfx_sample_voice_event": (ctypes.c_int, [_P, ctypes.c_uint8, ctypes.c_uint8, ctypes.c_uint8, _F]),
    "olfx_sample_update": (ctypes.c_int, [_P]),
    "olfx_sample_control": (ctypes.c_int, [_P, ctypes.c_uint8, ctypes.c_int, _F]),
    "olfx_sample_process": (ctypes.c_int, [_P, ctypes.POINTER(_F), ctypes.POINTER(_F)]),
    "olfx_sample_latency": (_U32, [_P]),
    "olfx_sample_generation_size": (_U32, [_P]),
    "olfx_sample_index": (_U32, [_P]),
    # include/olfx_dattorro.h: pool control of the verb.h-compatible names
    "olfx_dattorro_pool_config": (ctypes.c_int, [ctypes.c_int, _U32]),
    "olfx_dattorro_pool_config_depth": (ctypes.c_int, [ctypes.c_int, _U32, _U32]),
    "olfx_dattorro_latency": (_U32, [_P]),
    "olfx_dattorro_generation_size": (_U32, [_P]),
    "olfx_dattorro_index": (_U32, [_P]),
}

# include/olfx_dattorro.h: libs/dattorro-verb/verb.h:5-26 by name (C linkage; libolfx.so also
# exports the C++-mangled twins the reference's own callers link to)
DATTORRO_SIGNATURES = {
    "DattorroVerb_create": (_P, []),
    "DattorroVerb_delete": (None, [_P]),
    "DattorroVerb_setPreDelay": (None, [_P, _F]),
    "DattorroVerb_setPreFilter": (None, [_P, _F]),
    "DattorroVerb_setInputDiffusion1": (None, [_P, _F]),
    "DattorroVerb_setInputDiffusion2": (None, [_P, _F]),
    "DattorroVerb_setDecayDiffusion": (None, [_P, _F]),
    "DattorroVerb_setDecay": (None, [_P, _F]),
    "DattorroVerb_setDamping": (None, [_P, _F]),
    "DattorroVerb_process": (None, [_P, _F]),
    "DattorroVerb_getLeft": (_F, [_P]),
    "DattorroVerb_getRight": (_F, [_P]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libolfx.so (once).  Raises if the HIP library has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(make -C ol_dsp_amd/csrc).  There is no CPU fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in list(SIGNATURES.items()) + list(DATTORRO_SIGNATURES.items()):
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, handle=None) -> None:
    if rc != OLFX_OK:
        lib = load()
        msg = lib.olfx_last_error(handle)
        raise OlfxError(rc, msg.decode() if msg else "")
