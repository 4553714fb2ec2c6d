"""Control-change plumbing: the reference's UpdateMidiControl /
UpdateHardwareControl handlers mapped onto parameter fields by olfx_control_map -- a host-only
C-ABI function, so this runs without a GPU.  Expected values restate ol::core::scale
(corelib/ol_corelib.h:31-44) in float32 for each handler:
  voice : SynthVoice.h:100-229         fx rack: Fx.h:116-163 (FilterFx), 218-267 (DelayFx),
                                                 313-391 (ReverbFx), 451-489 (FxRack)
"""
import numpy as np
import pytest

import ol_dsp_amd as ofx

f32 = np.float32


def close(got, want, power):
    """Exact for power 1 (no pow); within 2 ulp otherwise (powf here vs the host libm's powf)."""
    return got == want if power == 1 else abs(got - want) <= 2.5e-7 * max(abs(want), 1e-30)


def scale(x, inlow, inhigh, outlow, outhigh, power):
    """ol::core::scale with t_sample = float (powf for the curve)."""
    x, inlow, inhigh, outlow, outhigh, power = map(f32, (x, inlow, inhigh, outlow, outhigh, power))
    denom = f32(inhigh - inlow)
    inscale = f32(0) if denom == 0 else f32(f32(1) / denom)
    v = f32(f32(x - inlow) * inscale)
    if v > 0:
        v = f32(np.power(v, power, dtype=np.float32))
    elif v < 0:
        v = f32(-np.power(-v, power, dtype=np.float32))
    return float(f32(f32(v * f32(outhigh - outlow)) + outlow))


@pytest.mark.parametrize("cc,field,midi_scale,hw_scale", [
    (7, "amp_env_amount", (1, 1), None),
    (5, "portamento", (1, 4), (1, 4)),
    (41, "filter_cutoff", (20000, 2.5), (20000, 2.5)),
    (42, "filter_resonance", (1, 1), None),
    (44, "filter_drive", (1, 1), None),
    (73, "filter_env_amount", (1, 1), None),
    (74, "filter_attack", (1, 1), None),
    (75, "filter_decay", (1, 3), (1, 3)),
    (76, "filter_sustain", (1, 1), None),
    (77, "filter_release", (1, 1), None),
    (108, "amp_attack", (1, 1), None),
    (109, "amp_decay", (1, 1), None),
    (110, "amp_sustain", (1, 1), None),
    (111, "amp_release", (1, 1), None),
])
def test_voice_controls(cc, field, midi_scale, hw_scale):
    for v in (0, 1, 64, 100, 127):
        got = ofx.control_map("voice", cc, v)
        assert got[0] == field and close(got[1], scale(v, 0, 127, 0, *midi_scale), midi_scale[1]), (cc, v, got)
    for v in (0.0, 0.25, 0.7, 1.0):
        got = ofx.control_map("voice", cc, v, "hw")
        want = scale(v, 0, 1, 0, *hw_scale) if hw_scale else float(f32(v))
        assert got[0] == field and close(got[1], want, hw_scale[1] if hw_scale else 1), (cc, v, got)


def test_voice_osc_mix_is_update_only_and_unknown_ignored():
    assert ofx.control_map("voice", 114, 90)[0] == "update_only"      # osc_1_mix: Update() only
    for cc in (0, 1, 34, 45, 70, 127):
        assert ofx.control_map("voice", cc, 64) is None


@pytest.mark.parametrize("cc,field,midi_scale,hw", [
    (45, "filter_cutoff", (20000, 1), (20000, 1.02)),   # FilterFx::UpdateHardwareControl: power 1.02
    (46, "filter_resonance", (1, 1), "raw"),
    (48, "filter_drive", (1, 1), "raw"),
    (35, "delay_time", (1, 1), "raw"),
    (36, "delay_feedback", (1, 1), "raw"),
    (39, "delay_balance", (1, 1), "raw"),
    (34, "reverb_balance", (1, 1), "raw"),
    (7, "master_volume", (1, 1), "raw"),
    (37, "delay_cutoff", (20000, 1), None),              # DelayFx: MIDI only
    (38, "delay_resonance", (1, 1), None),
])
def test_fxrack_controls(cc, field, midi_scale, hw):
    for v in (0, 13, 64, 127):
        got = ofx.control_map("fxrack", cc, v)
        assert got[0] == field and close(got[1], scale(v, 0, 127, 0, *midi_scale), midi_scale[1]), (cc, v, got)
    for v in (0.0, 0.3, 1.0):
        got = ofx.control_map("fxrack", cc, v, "hw")
        if hw is None:
            assert got is None
        else:
            want = float(f32(v)) if hw == "raw" else scale(v, 0, 1, 0, *hw)
            assert got[0] == field and close(got[1], want, 1 if hw == "raw" else hw[1]), (cc, v, got)


def test_fxrack_filter_type_truncates_and_stub_reverb_ccs_ignored():
    # FilterType(scale(value, 0, 127, 0, 5, 1)): float -> enum truncation; 127 -> 5 (out of range:
    # FilterFx::Process falls to its LowPass default)
    assert [ofx.control_map("fxrack", 47, v)[1] for v in (0, 25, 26, 64, 127)] == [0, 0, 1, 2, 5]
    for cc in (32, 33, 50, 52, 53, 54, 55, 56, 41, 60):
        assert ofx.control_map("fxrack", cc, 64) is None


def test_kinds_without_control_handlers():
    assert ofx.control_map("chorus", 41, 64) is None
    assert ofx.control_map("dattorro", 33, 64) is None
    with pytest.raises(ofx.OlfxError):
        ofx.control_map(99, 41, 64)
