"""ctypes access to the CPU oracle (TEST INFRASTRUCTURE ONLY).

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the
product package.  Two libraries:
  oracle/liboracle.so        the C restatements (dattorro bit-exact; chorus/pitch/voice spec oracles)
  oracle/_ref/libverb_ref.so the REAL reference reverb compiled from /root/reference (dev container;
                             travels to the GPU box as a prebuilt .so, never rebuilt there)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
LIB_O0 = os.path.join(HERE, "liboracle_O0.so")      # the same sources at -O0 (reference CMake default)
REF_LIB = os.path.join(HERE, "_ref", "libverb_ref.so")
REF_LIB_O0 = os.path.join(HERE, "_ref", "libverb_ref_O0.so")

DT_FIELDS = ["pre_delay", "pre_filter", "input_diffusion1", "input_diffusion2",
             "decay_diffusion", "decay", "damping"]
CH_FIELDS = ["pitch", "mix", "q", "cutoff", "phase", "depth", "rate", "window"]
FR_FIELDS = ["delay_time", "delay_feedback", "delay_balance", "delay_cutoff", "delay_resonance",
             "reverb_balance", "filter_cutoff", "filter_resonance", "filter_drive", "filter_type",
             "master_volume", "topology"]
VC_FIELDS = ["filter_cutoff", "filter_resonance", "filter_drive", "filter_env_amount",
             "filter_attack", "filter_attack_shape", "filter_decay", "filter_sustain",
             "filter_release", "amp_env_amount", "amp_attack", "amp_attack_shape",
             "amp_decay", "amp_sustain", "amp_release", "portamento"]
VOICE_DEFAULTS = [0.0, 0.0, 0.0, 1.0, 0.0, 1.0, 0.2, 0.0, 0.0, 0.8, 0.01, 1.0, 0.0, 1.0, 0.01, 0.0]

_F = ctypes.c_float
_PF = ctypes.POINTER(ctypes.c_float)
_libs = {}
_ref = {}


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib(o0: bool = False) -> ctypes.CDLL:
    path = LIB_O0 if o0 else LIB
    if path not in _libs:
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_dattorro_create.restype = ctypes.c_void_p
        L.oracle_dattorro_create.argtypes = [ctypes.c_int]
        L.oracle_dattorro_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_dattorro_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _F]
        L.oracle_dattorro_process.argtypes = [ctypes.c_void_p, _PF, ctypes.c_int, _PF, ctypes.c_int, ctypes.c_int]
        L.oracle_dattorro_state_floats.restype = ctypes.c_size_t
        L.oracle_xorshift_noise.restype = ctypes.c_uint32
        L.oracle_xorshift_noise.argtypes = [ctypes.c_uint32, _PF, ctypes.c_long, ctypes.c_long]
        L.oracle_fnv1a64_lr.restype = ctypes.c_uint64
        L.oracle_fnv1a64_lr.argtypes = [_PF, _PF, ctypes.c_long, ctypes.c_long]
        L.oracle_cos2pi.restype = _F
        L.oracle_cos2pi.argtypes = [_F]
        L.oracle_win_gains.restype = None
        L.oracle_win_gains.argtypes = [_F, ctypes.POINTER(_F), ctypes.POINTER(_F)]
        L.oracle_chorus_create.restype = ctypes.c_void_p
        L.oracle_chorus_create.argtypes = [ctypes.c_int, _F, ctypes.c_int]
        L.oracle_chorus_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_chorus_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _F]
        L.oracle_chorus_process.argtypes = [ctypes.c_void_p, _PF, _PF, ctypes.c_int, ctypes.c_int]
        L.oracle_voice_create.restype = ctypes.c_void_p
        L.oracle_voice_create.argtypes = [ctypes.c_int, _F]
        L.oracle_voice_create_model.restype = ctypes.c_void_p
        L.oracle_voice_create_model.argtypes = [ctypes.c_int, _F, ctypes.c_int]
        L.oracle_voice_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_voice_config.argtypes = [ctypes.c_void_p, ctypes.c_int, _PF]
        L.oracle_voice_init_members.argtypes = [ctypes.c_void_p, ctypes.c_int, _PF]
        L.oracle_chorus64_create.restype = ctypes.c_void_p
        L.oracle_chorus64_create.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int]
        L.oracle_chorus64_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_chorus64_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.oracle_chorus64_process.argtypes = [ctypes.c_void_p, _PF, ctypes.POINTER(ctypes.c_double), ctypes.c_int]
        L.oracle_voice_note.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.oracle_voice_event.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, _F]
        L.oracle_voice_process.argtypes = [ctypes.c_void_p, _PF, ctypes.c_int, ctypes.c_int]
        L.oracle_voice_set_arith.argtypes = [ctypes.c_void_p, ctypes.c_int]
        L.oracle_rcp_table_set.argtypes = [ctypes.c_void_p]
        L.oracle_rcp_model.restype = _F
        L.oracle_rcp_model.argtypes = [_F]
        L.oracle_fxrack_defaults.argtypes = [_PF]
        L.oracle_fxrack_create.restype = ctypes.c_void_p
        L.oracle_fxrack_create.argtypes = [ctypes.c_int, _F]
        L.oracle_fxrack_destroy.argtypes = [ctypes.c_void_p]
        L.oracle_fxrack_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _F]
        L.oracle_fxrack_process.argtypes = [ctypes.c_void_p, _PF, _PF, ctypes.c_int, ctypes.c_int]
        L.oracle_chorus_c1.restype = ctypes.c_long
        L.oracle_chorus_c1.argtypes = [_F, _PF, ctypes.c_long, ctypes.c_int, ctypes.POINTER(ctypes.c_double)]
        _libs[path] = L
    return _libs[path]


def ref_available(o0: bool = False) -> bool:
    return os.path.exists(REF_LIB_O0 if o0 else REF_LIB)


def ref_lib(o0: bool = False) -> ctypes.CDLL:
    path = REF_LIB_O0 if o0 else REF_LIB
    if path not in _ref:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (needs /root/reference at build time)")
        L = ctypes.CDLL(path)
        L.ref_verb_create.restype = ctypes.c_void_p
        L.ref_verb_create.argtypes = [ctypes.c_int]
        L.ref_verb_destroy.argtypes = [ctypes.c_void_p]
        L.ref_verb_set.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, _F]
        L.ref_verb_process.argtypes = [ctypes.c_void_p, _PF, ctypes.c_int, _PF, ctypes.c_int, ctypes.c_int]
        _ref[path] = L
    return _ref[path]


def _pf(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_PF)


def xorshift_noise(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, dtype=np.float32)
    lib().oracle_xorshift_noise(seed & 0xFFFFFFFF, _pf(out), n, 1)
    return out


def fnv1a64_lr(l: np.ndarray, r: np.ndarray) -> int:
    l = np.ascontiguousarray(l, dtype=np.float32)
    r = np.ascontiguousarray(r, dtype=np.float32)
    return int(lib().oracle_fnv1a64_lr(_pf(l), _pf(r), len(l), 1))


def instance_seed(i: int, c: int) -> int:
    """SURVEY.md section 8d per-(instance, channel) seed."""
    return ((0x9E3779B9 ^ (((2 * i + c + 1) * 0x85EBCA6B) & 0xFFFFFFFF)) | 1) & 0xFFFFFFFF


class _Bank:
    """Common shape: process(in [ch][frames][n]) -> out [och][frames][n]."""

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Dattorro(_Bank):
    """The C restatement (ref=False) or the real reference (ref=True) for n instances."""

    def __init__(self, n: int, ref: bool = False, o0: bool = False):
        self.n = n
        self.ref = ref
        if ref:
            self.L = ref_lib(o0)
            self.h = self.L.ref_verb_create(n)
        else:
            self.L = lib(o0)
            self.h = self.L.oracle_dattorro_create(n)
        assert self.h

    def close(self):
        if getattr(self, "h", None):
            (self.L.ref_verb_destroy if self.ref else self.L.oracle_dattorro_destroy)(self.h)
            self.h = None

    def set(self, inst: int, field, value: float) -> None:
        f = DT_FIELDS.index(field) if isinstance(field, str) else int(field)
        rc = (self.L.ref_verb_set if self.ref else self.L.oracle_dattorro_set)(self.h, inst, f, value)
        assert rc == 0

    def process(self, x: np.ndarray, threads: int = 1) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        ch, frames, n = x.shape
        assert n == self.n and ch in (1, 2)
        out = np.empty((2, frames, n), dtype=np.float32)
        fn = self.L.ref_verb_process if self.ref else self.L.oracle_dattorro_process
        assert fn(self.h, _pf(x), ch, _pf(out), frames, threads) == 0
        return out


class Chorus(_Bank):
    """mode 0 = stereo chorus, 1 = pitch-shift stage (fields 'pitch' = shift Hz, 'window')."""

    def __init__(self, n: int, sample_rate: float = 48000.0, mode: int = 0, o0: bool = False):
        self.n = n
        self.L = lib(o0)
        self.h = self.L.oracle_chorus_create(n, sample_rate, mode)
        assert self.h

    def close(self):
        if getattr(self, "h", None):
            self.L.oracle_chorus_destroy(self.h)
            self.h = None

    def set(self, inst: int, field, value: float) -> None:
        f = CH_FIELDS.index(field) if isinstance(field, str) else int(field)
        assert self.L.oracle_chorus_set(self.h, inst, f, value) == 0

    def process(self, x: np.ndarray, threads: int = 1) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        ch, frames, n = x.shape
        assert ch == 2 and n == self.n
        out = np.empty_like(x)
        assert self.L.oracle_chorus_process(self.h, _pf(x), _pf(out), frames, threads) == 0
        return out


class Chorus64(_Bank):
    """The chorus / pitch-shift in double precision with double phasors (gen~ / RNBO arithmetic,
    oracle/chorus_ref_f64.c): the yardstick for the fp32 spec's arithmetic deviation."""

    def __init__(self, n: int, sample_rate: float = 48000.0, mode: int = 0):
        self.n = n
        self.L = lib()
        self.h = self.L.oracle_chorus64_create(n, sample_rate, mode)
        assert self.h

    def close(self):
        if getattr(self, "h", None):
            self.L.oracle_chorus64_destroy(self.h)
            self.h = None

    def set(self, inst: int, field, value: float) -> None:
        f = CH_FIELDS.index(field) if isinstance(field, str) else int(field)
        assert self.L.oracle_chorus64_set(self.h, inst, f, float(value)) == 0

    def process(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        ch, frames, n = x.shape
        assert ch == 2 and n == self.n
        out = np.empty(x.shape, np.float64)
        assert self.L.oracle_chorus64_process(
            self.h, _pf(x), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), frames) == 0
        return out


class Voice(_Bank):
    """SynthVoice bank.  moog=False: SvfFilter voice (SynthVoice default); moog=True: MoogFilter
    voice (daisysp::LadderFilter, the Daisy synth firmware's voice, main.cpp:49-52)."""

    def __init__(self, n: int, sample_rate: float = 48000.0, moog: bool = False, o0: bool = False,
                 kernel_arith: bool = False):
        self.n = n
        self.L = lib(o0)
        self.h = self.L.oracle_voice_create_model(n, sample_rate, int(bool(moog)))
        assert self.h
        if kernel_arith:
            assert self.L.oracle_voice_set_arith(self.h, 1) == 0

    def close(self):
        if getattr(self, "h", None):
            self.L.oracle_voice_destroy(self.h)
            self.h = None

    def config(self, inst: int, values) -> None:
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float32))
        assert v.shape == (len(VC_FIELDS),)
        assert self.L.oracle_voice_config(self.h, inst, _pf(v)) == 0

    def init_members(self, inst: int, values) -> None:
        """Member values set before Init, then Init (no Update): voice_ref.c oracle_voice_init_members."""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float32))
        assert v.shape == (len(VC_FIELDS),)
        assert self.L.oracle_voice_init_members(self.h, inst, _pf(v)) == 0

    def note(self, inst: int, on: bool, note: int = 60) -> None:
        assert self.L.oracle_voice_note(self.h, inst, int(bool(on)), int(note)) == 0

    def event(self, inst: int, type_: int, note: int = 0, value: float = 0.0) -> None:
        """Voice.h:33-57: 0 NoteOff, 1 NoteOn, 2 GateOn, 3 GateOff, 4 SetFrequency(value)."""
        assert self.L.oracle_voice_event(self.h, inst, int(type_), int(note), float(value)) == 0

    def process(self, frames: int, threads: int = 1) -> np.ndarray:
        out = np.empty((1, frames, self.n), dtype=np.float32)
        assert self.L.oracle_voice_process(self.h, _pf(out), frames, threads) == 0
        return out


def set_rcp_table(tab) -> None:
    """The v_rcp_f32 model of the voice's kernel arithmetic (voice_ref.c): `tab` = the instruction's
    2^23 results (uint32 bits) over the mantissas of [1, 2), as read from the device; None = the
    correctly rounded reciprocal."""
    L = lib()
    if tab is None:
        assert L.oracle_rcp_table_set(None) == 0
        return
    t = np.ascontiguousarray(tab, dtype=np.uint32)
    assert t.shape == (1 << 23,)
    assert L.oracle_rcp_table_set(t.ctypes.data) == 0


def chorus_c1(params, n_frames: int, block: int = 256, sample_rate: float = 48000.0, o0: bool = False):
    """BASELINE configs[0]: one chorus instance on one core, per-frame calls in fx_test.cpp:45-54's
    loop shape (oracle_chorus_c1).  Returns (nan_count, sum |y|)."""
    p = np.ascontiguousarray(np.asarray(params, dtype=np.float32))
    assert p.shape == (len(CH_FIELDS),)
    acc = ctypes.c_double()
    nans = lib(o0).oracle_chorus_c1(sample_rate, _pf(p), int(n_frames), int(block), ctypes.byref(acc))
    assert nans >= 0
    return int(nans), acc.value


def fxrack_defaults() -> np.ndarray:
    p = np.zeros(len(FR_FIELDS), np.float32)
    lib().oracle_fxrack_defaults(_pf(p))
    return p


class FxRack(_Bank):
    """ol::fx::FxRack<2>: stereo in -> delay -> reverb (ReverbSc stub) -> filter (ch 0) -> master."""

    def __init__(self, n: int, sample_rate: float = 48000.0, o0: bool = False):
        self.n = n
        self.L = lib(o0)
        self.h = self.L.oracle_fxrack_create(n, sample_rate)
        assert self.h

    def close(self):
        if getattr(self, "h", None):
            self.L.oracle_fxrack_destroy(self.h)
            self.h = None

    def set(self, inst: int, field, value: float) -> None:
        f = FR_FIELDS.index(field) if isinstance(field, str) else int(field)
        assert self.L.oracle_fxrack_set(self.h, inst, f, value) == 0

    def process(self, x: np.ndarray, threads: int = 1) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float32)
        ch, frames, n = x.shape
        assert ch == 2 and n == self.n
        out = np.empty_like(x)
        assert self.L.oracle_fxrack_process(self.h, _pf(x), _pf(out), frames, threads) == 0
        return out


def mix_ref(voice_out: np.ndarray, buses, bus_init=None) -> np.ndarray:
    """Polyvoice::Process (modules/synthlib/Polyvoice.h:28-33) / VoiceMap::Process (VoiceMap.h:64-73):
    per frame, `*frame_out += frame_buffer` voice by voice, in list order -- float32 adds, one
    rounding each, vectorised over frames only.  voice_out [1][F][n] or [F][n] -> [F][len(buses)]."""
    v = np.asarray(voice_out, np.float32)
    v = v.reshape(v.shape[-2], v.shape[-1])
    out = (np.zeros((v.shape[0], len(buses)), np.float32) if bus_init is None
           else np.array(bus_init, dtype=np.float32, copy=True))
    for b, voices in enumerate(buses):
        acc = out[:, b].copy()
        for i in voices:
            acc = acc + v[:, int(i)]
        out[:, b] = acc
    return out
