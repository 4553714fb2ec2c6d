"""Host-side Python mirror of the batch engine C-ABI (include/olfx.h).

``Engine`` owns one libolfx engine: one effect kind x N independent instances on one GPU.
Audio crosses the boundary as ``[channels][frames][instances]`` float32 buffers, either torch
CUDA tensors (device pointers, the fast path; torch is only plumbing for device memory and
streams) or numpy arrays (host pointers, staged through pinned memory inside the library).

Reference surfaces this mirrors (per instance, batched here):
  DattorroVerb_create/set*/process/getLeft/getRight   libs/dattorro-verb/verb.h:5-26
  ChorusEffect init/setDepth/setRate/process           README.md:114-128 (+ RNBO params)
  SynthVoice Init/UpdateConfig/NoteOn/NoteOff/Process  modules/synthlib/SynthVoice.h:31-256
  Polyvoice NoteOn/NoteOff/Process (voice buses)       modules/synthlib/Polyvoice.h:11-86
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check, load

KIND_NAMES = {
    "dattorro": _lib.KIND_DATTORRO,
    "chorus": _lib.KIND_CHORUS,
    "pitchshift": _lib.KIND_PITCHSHIFT,
    "voice": _lib.KIND_VOICE,
    "chain": _lib.KIND_CHAIN,
    "fxrack": _lib.KIND_FXRACK,
    "voice_moog": _lib.KIND_VOICE_MOOG,
}

# parameter field names, in C-ABI order
PARAMS = {
    _lib.KIND_DATTORRO: ["pre_delay", "pre_filter", "input_diffusion1", "input_diffusion2",
                         "decay_diffusion", "decay", "damping"],
    _lib.KIND_CHORUS: ["pitch", "mix", "q", "cutoff", "phase", "depth", "rate", "window"],
    _lib.KIND_PITCHSHIFT: ["shift", "window"],
    _lib.KIND_VOICE: ["filter_cutoff", "filter_resonance", "filter_drive", "filter_env_amount",
                      "filter_attack", "filter_attack_shape", "filter_decay", "filter_sustain",
                      "filter_release", "amp_env_amount", "amp_attack", "amp_attack_shape",
                      "amp_decay", "amp_sustain", "amp_release", "portamento"],
    _lib.KIND_FXRACK: ["delay_time", "delay_feedback", "delay_balance", "delay_cutoff", "delay_resonance",
                       "reverb_balance", "filter_cutoff", "filter_resonance", "filter_drive", "filter_type",
                       "master_volume", "topology"],
}
PARAMS[_lib.KIND_VOICE_MOOG] = PARAMS[_lib.KIND_VOICE]
PARAMS[_lib.KIND_CHAIN] = (["chorus_" + p for p in PARAMS[_lib.KIND_CHORUS]]
                           + ["pitch_" + p for p in PARAMS[_lib.KIND_PITCHSHIFT]]
                           + ["verb_" + p for p in PARAMS[_lib.KIND_DATTORRO]])


def kind_info(kind: int, sample_rate: float = 48000.0) -> _lib.KindInfo:
    info = _lib.KindInfo()
    check(load().olfx_kind_info_get(int(kind), float(sample_rate), ctypes.byref(info)))
    return info


def _is_torch(x) -> bool:
    return type(x).__module__.startswith("torch")


class Engine:
    """N instances of one effect kind on one GPU (see module docstring)."""

    def __init__(self, kind, n_inst: int, sample_rate: float = 48000.0, block: int = 256,
                 device: int = 0):
        self.lib = load()
        self.kind = KIND_NAMES[kind] if isinstance(kind, str) else int(kind)
        self.n = int(n_inst)
        self.sample_rate = float(sample_rate)
        self.block = int(block)
        self.device = int(device)
        self.info = kind_info(self.kind, sample_rate)
        h = ctypes.c_void_p()
        check(self.lib.olfx_create(self.kind, self.device, self.n, self.sample_rate, self.block,
                                   ctypes.byref(h)))
        self._h = h

    # ---- lifetime ----
    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.olfx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def reset(self) -> None:
        check(self.lib.olfx_reset(self._h), self._h)

    # ---- parameters ----
    def field(self, name_or_index) -> int:
        if isinstance(name_or_index, str):
            return PARAMS[self.kind].index(name_or_index)
        return int(name_or_index)

    def set_param(self, inst: int, field, value: float) -> None:
        check(self.lib.olfx_set_param(self._h, int(inst), self.field(field), float(value)), self._h)

    def get_param(self, inst: int, field) -> float:
        v = ctypes.c_float()
        check(self.lib.olfx_get_param(self._h, int(inst), self.field(field), ctypes.byref(v)), self._h)
        return v.value

    def set_params(self, field0, values, first: int = 0) -> None:
        """values: array [n_fields][count] (field-major) for fields field0.. and instances first.."""
        arr = np.ascontiguousarray(np.asarray(values, dtype=np.float32))
        if arr.ndim == 1:
            arr = arr[None, :]
        nf, cnt = arr.shape
        check(self.lib.olfx_set_params(self._h, int(first), int(cnt), self.field(field0), int(nf),
                                       arr.ctypes.data_as(ctypes.POINTER(ctypes.c_float))), self._h)

    def set_param_list(self, field, inst, values) -> None:
        """One field of scattered instances: inst[k] <- values[k] (olfx_set_param_list)."""
        ii = np.ascontiguousarray(np.asarray(inst, dtype=np.uint32).ravel())
        vv = np.ascontiguousarray(np.asarray(values, dtype=np.float32).ravel())
        assert ii.shape == vv.shape
        check(self.lib.olfx_set_param_list(self._h, self.field(field), ii.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                           vv.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), len(ii)), self._h)

    @staticmethod
    def make_events(inst, type_, note, velocity=100):
        """A prebuilt event array (numpy-vectorised) for note_events: inst / note arrays (or
        scalars broadcast against them), type 1 = NoteOn, 0 = NoteOff."""
        inst = np.asarray(inst, np.uint32).ravel()
        rec = np.zeros(len(inst), dtype=[("inst", "<u4"), ("type", "u1"), ("note", "u1"), ("velocity", "u1"),
                                         ("pad", "u1")])
        rec["inst"] = inst
        rec["type"] = type_
        rec["note"] = note
        rec["velocity"] = velocity
        assert ctypes.sizeof(_lib.Event) == rec.dtype.itemsize
        return rec

    def note_events(self, events) -> None:
        """events: iterable of (inst, type, note[, velocity]) (type 1 = NoteOn, 0 = NoteOff), or an
        array from make_events()."""
        if isinstance(events, np.ndarray):
            if len(events):
                check(self.lib.olfx_note_events(self._h, events.ctypes.data_as(ctypes.POINTER(_lib.Event)),
                                                len(events)), self._h)
            return
        evs = list(events)
        if not evs:
            return
        arr = (_lib.Event * len(evs))()
        for k, e in enumerate(evs):
            arr[k].inst = int(e[0])
            arr[k].type = int(e[1])
            arr[k].note = int(e[2])
            arr[k].velocity = int(e[3]) if len(e) > 3 else 100
        check(self.lib.olfx_note_events(self._h, arr, len(evs)), self._h)

    def voice_events(self, events: Iterable[Sequence]) -> None:
        """Voice events in order: iterable of (inst, type[, note[, value]]) with type one of
        _lib.EV_* (NoteOn/NoteOff/GateOn/GateOff/SetFrequency, Voice.h:33-57); value = Hz for
        SetFrequency."""
        evs = list(events)
        if not evs:
            return
        arr = (_lib.VoiceEvent * len(evs))()
        for k, e in enumerate(evs):
            arr[k].inst = int(e[0])
            arr[k].type = int(e[1])
            arr[k].note = int(e[2]) if len(e) > 2 else 0
            arr[k].velocity = 100
            arr[k].value = float(e[3]) if len(e) > 3 else 0.0
        check(self.lib.olfx_voice_events(self._h, arr, len(evs)), self._h)

    def update(self, first: int = 0, count: int = -1) -> None:
        """Update() of instances first..first+count with their current parameters."""
        count = self.n - first if count < 0 else count
        check(self.lib.olfx_update(self._h, int(first), int(count)), self._h)

    def control(self, events: Iterable[Sequence]) -> None:
        """Control changes, applied in order: iterable of (inst, cc, value[, source]); source
        "midi" (value 0..127, the default) or "hw" (UpdateHardwareControl value)."""
        evs = list(events)
        if not evs:
            return
        arr = (_lib.ControlEvent * len(evs))()
        for k, e in enumerate(evs):
            arr[k].inst = int(e[0])
            arr[k].control = int(e[1])
            arr[k].value = float(e[2])
            arr[k].source = _lib.CTL_HARDWARE if len(e) > 3 and e[3] in ("hw", _lib.CTL_HARDWARE) else _lib.CTL_MIDI
        check(self.lib.olfx_control(self._h, arr, len(evs)), self._h)

    # ---- processing ----
    def process(self, x, out=None, n_frames: Optional[int] = None, stream=None):
        """Process one block for all instances.

        x: [in_ch][frames][n] torch CUDA tensor or numpy array (None for voices).
        out: optional preallocated output of the same kind; returned.
        stream: hipStream_t as int (torch.cuda.Stream.cuda_stream; 0 = the null stream) or
        None = torch's current stream for tensors, the engine's own stream for numpy.
        """
        ich, och = self.info.in_channels, self.info.out_channels
        ref = x if x is not None else out
        if n_frames is None:
            if x is not None:
                n_frames = int(x.shape[1])
            elif out is not None:
                n_frames = int(out.shape[1])
            else:
                raise ValueError("n_frames required")
        if ref is not None and _is_torch(ref):
            import torch
            if x is not None:
                assert x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()
                assert tuple(x.shape) == (ich, n_frames, self.n), (tuple(x.shape), (ich, n_frames, self.n))
            if out is None:
                out = torch.empty((och, n_frames, self.n), dtype=torch.float32, device=ref.device)
            assert out.is_contiguous() and tuple(out.shape) == (och, n_frames, self.n)
            if stream is None:
                stream = torch.cuda.current_stream(ref.device).cuda_stream
            check(self.lib.olfx_process(self._h, ctypes.c_void_p(x.data_ptr() if x is not None else 0),
                                        ctypes.c_void_p(out.data_ptr()), int(n_frames), _lib.IO_DEVICE,
                                        ctypes.c_void_p(stream)), self._h)
            return out
        # host path
        xin = None
        if x is not None:
            xin = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
            assert xin.shape == (ich, n_frames, self.n), (xin.shape, (ich, n_frames, self.n))
        if out is None:
            out = np.empty((och, n_frames, self.n), dtype=np.float32)
        if stream is None:
            stream = self.lib.olfx_stream(self._h)
        check(self.lib.olfx_process(self._h, ctypes.c_void_p(xin.ctypes.data if xin is not None else 0),
                                    ctypes.c_void_p(out.ctypes.data), int(n_frames), _lib.IO_HOST,
                                    ctypes.c_void_p(stream)), self._h)
        return out

    # ---- voice buses: the Polyvoice / VoiceMap sums (Polyvoice.h:28-33, VoiceMap.h:64-73) ----
    def mix_config(self, buses: Sequence[Sequence[int]]) -> None:
        """Bus b adds the voices buses[b] in list order, one float add per voice (the reference's
        `*frame_out += frame_buffer`); each voice at most once over all buses; [] removes them."""
        lists = [np.asarray(b, dtype=np.uint32).ravel() for b in buses]
        off = np.zeros(len(lists) + 1, np.uint32)
        if lists:
            off[1:] = np.cumsum([len(b) for b in lists])
        order = np.ascontiguousarray(np.concatenate(lists) if off[-1] else np.zeros(1, np.uint32))
        u32 = ctypes.POINTER(ctypes.c_uint32)
        check(self.lib.olfx_mix_config(self._h, len(lists), off.ctypes.data_as(u32), order.ctypes.data_as(u32)),
              self._h)

    @property
    def n_buses(self) -> int:
        return int(self.lib.olfx_num_buses(self._h))

    def mix(self, voice_out, bus_out=None, stream=None):
        """bus_out [frames][n_buses] += each bus's voices of voice_out ([1][frames][n] or
        [frames][n]), added in bus order.  Torch CUDA tensors (device path) or numpy arrays (host
        path); bus_out defaults to zeros."""
        nb = self.n_buses
        frames = int(voice_out.shape[-2])
        assert tuple(voice_out.shape[-2:]) == (frames, self.n), (tuple(voice_out.shape), self.n)
        if _is_torch(voice_out):
            import torch
            assert voice_out.is_cuda and voice_out.dtype == torch.float32 and voice_out.is_contiguous()
            if bus_out is None:
                bus_out = torch.zeros((frames, nb), dtype=torch.float32, device=voice_out.device)
            assert bus_out.is_contiguous() and tuple(bus_out.shape) == (frames, nb)
            if stream is None:
                stream = torch.cuda.current_stream(voice_out.device).cuda_stream
            check(self.lib.olfx_mix(self._h, ctypes.c_void_p(voice_out.data_ptr()), ctypes.c_void_p(bus_out.data_ptr()),
                                    frames, _lib.IO_DEVICE, ctypes.c_void_p(stream)), self._h)
            return bus_out
        v = np.ascontiguousarray(np.asarray(voice_out, dtype=np.float32))
        if bus_out is None:
            bus_out = np.zeros((frames, nb), np.float32)
        assert bus_out.dtype == np.float32 and bus_out.flags.c_contiguous and bus_out.shape == (frames, nb)
        if stream is None:
            stream = self.lib.olfx_stream(self._h)
        check(self.lib.olfx_mix(self._h, ctypes.c_void_p(v.ctypes.data), ctypes.c_void_p(bus_out.ctypes.data),
                                frames, _lib.IO_HOST, ctypes.c_void_p(stream)), self._h)
        return bus_out

    def sync(self) -> None:
        check(self.lib.olfx_sync(self._h), self._h)

    # ---- facts ----
    @property
    def frames_processed(self) -> int:
        return int(self.lib.olfx_frames_processed(self._h))

    @property
    def algorithmic_bytes_per_frame(self) -> float:
        return float(self.lib.olfx_algorithmic_bytes_per_frame(self._h))

    @property
    def algorithmic_read_bytes_per_frame(self) -> float:
        return float(self.lib.olfx_algorithmic_read_bytes_per_frame(self._h))

    @property
    def kernel_name(self) -> str:
        return self.lib.olfx_kernel_name(self._h).decode()


def control_map(kind, control: int, value: float, source: str = "midi"):
    """The reference's UpdateMidiControl / UpdateHardwareControl mapping for one control change
    (host-only, no device): (field name or "update_only", mapped value), or None if the
    reference ignores the control for this kind."""
    k = KIND_NAMES[kind] if isinstance(kind, str) else int(kind)
    lib = load()
    field = ctypes.c_uint32()
    val = ctypes.c_float()
    src = _lib.CTL_HARDWARE if source in ("hw", _lib.CTL_HARDWARE) else _lib.CTL_MIDI
    rc = lib.olfx_control_map(k, int(control), src, float(value), ctypes.byref(field), ctypes.byref(val))
    if rc == _lib.IGNORED:
        return None
    check(rc, None)
    if field.value == _lib.FIELD_UPDATE_ONLY:
        return "update_only", val.value
    return PARAMS[k][field.value], val.value



class Polyvoice:
    """ol::synth::Polyvoice (modules/synthlib/Polyvoice.h:11-86), batched: each group of voices of a
    voice Engine is one Polyvoice and one bus.  note_on takes the group's first voice not Playing(),
    note_off its first voice Playing() that note (Polyvoice.h:35-51; SynthVoice::Playing() is the
    last NoteOn's note and 0 after NoteOff, SynthVoice.h:245-260, tracked here on the host).
    process() runs the voice block, then adds each group's voices into its bus in group order
    (olfx_mix): bit-identical to Polyvoice::Process over the same voice samples."""

    def __init__(self, engine: Engine, groups: Sequence[Sequence[int]]):
        self.engine = engine
        self.groups = [[int(v) for v in g] for g in groups]
        self.playing = np.zeros(engine.n, np.int64)
        engine.mix_config(self.groups)

    def note_on(self, group: int, note: int, velocity: int = 100) -> None:
        for v in self.groups[group]:
            if not self.playing[v]:
                self.engine.note_events([(v, 1, note, velocity)])
                self.playing[v] = note
                return

    def note_off(self, group: int, note: int, velocity: int = 0) -> None:
        for v in self.groups[group]:
            if self.playing[v] == note:
                self.engine.note_events([(v, 0, note, velocity)])
                self.playing[v] = 0
                return

    def process(self, voice_out, bus_out=None, stream=None):
        """One block: voice_out [1][frames][n] is written, the buses [frames][groups] are added into
        (zeros if None) and returned."""
        self.engine.process(None, out=voice_out, stream=stream)
        return self.engine.mix(voice_out, bus_out, stream=stream)
