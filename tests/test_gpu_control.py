"""GPU tests of the asynchronous control path (round 3) and of frame tiling.

Parameters, control changes and note events reach the device at the block boundary -- the JUCE
host's pattern, modules/juce/host/host.cpp:646-653 -- without a host round trip: the engine
re-derives the coefficients of the changed instances only and ships them (and the block's folded
note events) with the block (olfx_engine.cpp submit_control, control.hip, voice.hip voice_event).

Bars: the chain and the rack are BIT-EXACT against the oracle with the same changes applied at
the same block boundaries; the voice is within the parity tolerance of the oracle applying every
event in order (VOICE_TOL, as tests/test_gpu_parity.py), and BIT-IDENTICAL to a second engine given
only the folded (last-wins) equivalent of each block's events.
"""
import numpy as np
import pytest

import oracle as O
from helpers import bits_equal, chorus_params, dt_params, fast_noise, first_mismatch, fxrack_params, rel_err, voice_configs
from test_gpu_parity import VOICE_TOL, _chain_oracle, _voice_run, engine, run_gpu

pytestmark = pytest.mark.gpu


def test_chain_param_list_every_block_vs_oracle(cuda):
    """A control change at every block boundary on 10 % of the chains, scattered (olfx_set_param_list:
    one CC fanned out to many objects), rotating over chorus, pitch and reverb fields (the pre-delay
    too): bit-exact against the composed oracle given the same values at the same boundaries."""
    from ol_dsp_amd.engine import PARAMS
    n, blocks = 100, 16
    rng = np.random.default_rng(301)
    pc, pp, pd = chorus_params(rng, n), chorus_params(rng, n)[[0, 7]], dt_params(rng, n, 0.05)
    e = engine("chain", n)
    e.set_params(0, np.concatenate([pc, pp, pd], 0))
    c1, c2, d = _chain_oracle(n, pc, pp, pd)
    names = PARAMS[e.kind]
    ranges = {"chorus_depth": (.08, 1), "chorus_mix": (0, 1), "chorus_rate": (.01, 1), "chorus_pitch": (0, 3),
              "pitch_shift": (0, 3), "verb_decay": (.25, .95), "verb_damping": (.05, .95), "verb_pre_delay": (0, 1)}
    x = fast_noise(n, 256 * blocks, seed=301)
    ys, yrs = [], []
    for b in range(blocks):
        if b:
            fname = list(ranges)[b % len(ranges)]
            lo, hi = ranges[fname]
            sel = np.flatnonzero(rng.random(n) < 0.1).astype(np.uint32)
            vals = rng.uniform(lo, hi, len(sel)).astype(np.float32)
            e.set_param_list(fname, sel, vals)
            f = names.index(fname)
            for i, v in zip(sel, vals):
                if f < 8:
                    c1.set(int(i), f, float(v))
                elif f < 10:
                    c2.set(int(i), ("pitch", "window")[f - 8], float(v))
                else:
                    d.set(int(i), f - 10, float(v))
        xb = x[:, 256 * b:256 * (b + 1)]
        ys.append(run_gpu(e, xb, [256], cuda))
        yrs.append(d.process(c2.process(c1.process(xb))))
    y, yr = np.concatenate(ys, 1), np.concatenate(yrs, 1)
    assert bits_equal(y, yr), first_mismatch(y, yr)


def test_param_list_rejects_bad_values_atomically(cuda):
    """olfx_set_param_list validates the whole list first: an out-of-range instance or an illegal
    value anywhere leaves every parameter unchanged."""
    from ol_dsp_amd._lib import OlfxError
    e = engine("dattorro", 8)
    with pytest.raises(OlfxError):
        e.set_param_list("decay", [1, 2, 99], [0.3, 0.4, 0.5])
    with pytest.raises(OlfxError):
        e.set_param_list("pre_delay", [1, 2], [0.5, 20.0])       # 20 x 4800 leaves uint16
    assert e.get_param(1, "decay") == np.float32(0.75) and e.get_param(1, "pre_delay") == np.float32(0.1)


def test_fxrack_controls_every_block_and_firmware_routing(cuda):
    """MIDI / hardware CCs at every block boundary on a rack engine holding every topology: FxRack<2>
    (0), the Daisy firmware's chain (1) and its objects alone (2 DelayFx, 3 ReverbFx, 4 FilterFx).
    The firmware has no FxRack: every CC reaches delay_fx, reverb_fx and filter_fx directly
    (ol_daisy/app/synth/main.cpp:201-207), so CCs 41-44 drive a FilterFx (Fx.h:116-139) and 45-48 / 7
    do nothing; a component alone takes only its own CCs; topology-0 instances keep FxRack's routing
    (Fx.h:451-470).  Bit-exact against the oracle given the mapped values at the same boundaries."""
    import ol_dsp_amd as ofx
    n, blocks = 50, 12
    rng = np.random.default_rng(302)
    p = np.concatenate([fxrack_params(rng, n), np.zeros((1, n), np.float32)], 0)
    p[11] = np.arange(n) % 5                              # every topology: racks, firmware chain, components
    e = engine("fxrack", n)
    e.set_params(0, p)
    ref = O.FxRack(n)
    for i in range(n):
        for f in range(p.shape[0]):
            ref.set(i, f, float(p[f, i]))
    x = fast_noise(n, 256 * blocks, seed=302)
    ccs = [7, 34, 35, 36, 37, 38, 39, 41, 42, 43, 44, 45, 46, 47, 48]
    ys, yrs = [], []
    for b in range(blocks):
        if b:
            evs = []
            for i in np.flatnonzero(rng.random(n) < (0.5, 0.03, 0.1)[b % 3]):
                cc = int(rng.choice(ccs))
                if rng.random() < 0.8:
                    evs.append((int(i), cc, int(rng.integers(0, 128))))
                else:
                    evs.append((int(i), cc, float(rng.random()), "hw"))
            e.control(evs)
            for ev in evs:
                i, cc = ev[0], ev[1]
                src = ev[3] if len(ev) > 3 else "midi"
                topo = int(p[11, i])
                filt, dly = 41 <= cc <= 44, 35 <= cc <= 39
                if topo == 0 and filt:                    # FxRack: the voice-filter CCs reach no rack member
                    continue
                if topo:                                  # no FxRack: each object's own handler
                    takes = {1: filt or dly or cc == 34, 2: dly, 3: cc == 34, 4: filt}[topo]
                    if not takes:
                        continue
                    if filt:
                        cc += 4
                m = ofx.control_map("fxrack", cc, ev[2], src)
                if m is not None:
                    ref.set(i, m[0], m[1])
        xb = x[:, 256 * b:256 * (b + 1)]
        ys.append(run_gpu(e, xb, [256], cuda))
        yrs.append(ref.process(xb, threads=8))
    y, yr = np.concatenate(ys, 1), np.concatenate(yrs, 1)
    assert bits_equal(y, yr), first_mismatch(y, yr)
    # the routing itself, read back: topology 1 takes CC 41 as its post-filter cutoff, ignores 45
    e2 = engine("fxrack", 2)
    e2.set_param(1, "topology", 1.0)
    e2.control([(0, 41, 100), (1, 41, 100), (0, 45, 10), (1, 45, 10)])
    assert e2.get_param(0, "filter_cutoff") == ofx.control_map("fxrack", 45, 10)[1]
    assert e2.get_param(1, "filter_cutoff") == ofx.control_map("fxrack", 45, 100)[1]


def test_fxrack_component_topologies_vs_oracle(cuda):
    """DelayFx<2>, ReverbFx<2> and FilterFx<2> alone (OLFX_FR_TOPOLOGY 2 / 3 / 4, the firmware's
    objects, main.cpp:82-85) mixed with racks (0, 1) in one engine -- the kernel's COMP variant --
    through ragged blocks, short delays, every filter type, and a topology change mid-run (a
    component becomes a rack and back: filter1's state is kept only where it runs): bit-exact
    against the rack oracle.  Channel 1 of a FilterFx is its input (frame_out[1] in place)."""
    n = 75
    rng = np.random.default_rng(310)
    p = np.concatenate([fxrack_params(rng, n), np.zeros((1, n), np.float32)], 0)
    p[11] = (np.arange(n) * 3) % 5
    e = engine("fxrack", n)
    e.set_params(0, p)
    ref = O.FxRack(n)
    for i in range(n):
        for f in range(p.shape[0]):
            ref.set(i, f, float(p[f, i]))
    x = fast_noise(n, 4000, seed=310)
    y1 = run_gpu(e, x[:, :2000], [256, 4, 12, 240, 1488], cuda)
    yr1 = ref.process(x[:, :2000], threads=8)
    assert bits_equal(y1, yr1), first_mismatch(y1, yr1)
    flt = p[11] == 4
    assert np.array_equal(y1[1][:, flt], x[1, :2000][:, flt])
    topo2 = ((np.arange(n) * 3 + 1) % 5).astype(np.float32)
    e.set_params("topology", topo2[None, :])
    for i in range(n):
        ref.set(i, 11, float(topo2[i]))
    y2 = run_gpu(e, x[:, 2000:], [1024, 976], cuda)
    yr2 = ref.process(x[:, 2000:], threads=8)
    assert bits_equal(y2, yr2), first_mismatch(y2, yr2)
    # all components gone: the rack-only kernel again, state carried
    e.set_params("topology", np.zeros((1, n), np.float32))
    for i in range(n):
        ref.set(i, 11, 0.0)
    x3 = fast_noise(n, 512, seed=311)
    y3, yr3 = run_gpu(e, x3, [512], cuda), ref.process(x3, threads=8)
    assert bits_equal(y3, yr3), first_mismatch(y3, yr3)


def _fold(seq):
    """The last-wins equivalent of one voice's event sequence (SynthVoice.h:231-268): NoteOn of the
    last NoteOn's note if any, then SetFrequency if a SetFrequency came after it, then the final gate
    call (GateOn / GateOff) if any gate-changing call came after that NoteOn."""
    out = []
    last_on = max((k for k, ev in enumerate(seq) if ev[0] == 1), default=None)
    if last_on is not None:
        out.append(seq[last_on])
    last_freq = max((k for k, ev in enumerate(seq) if ev[0] in (1, 4)), default=None)
    if last_freq is not None and seq[last_freq][0] == 4:
        out.append(seq[last_freq])
    last_gate = max((k for k, ev in enumerate(seq) if ev[0] in (0, 1, 2, 3)), default=None)
    if last_gate is not None and last_gate != last_on:
        out.append((2, 0, 0.0) if seq[last_gate][0] == 2 else (3, 0, 0.0))
    return out


@pytest.mark.parametrize("kind", ["voice", "voice_moog"])
def test_voice_events_fused_fold(cuda, kind):
    """Several voice calls per voice per block (NoteOn, NoteOff, GateOn, GateOff, SetFrequency in
    random order), every block, for a random 50 %, 3 % or 10 % of the voices (workgroups of 64 voices
    above, below and on both sides of the kernel's kVevCap = 4 fixed event slots: the overflow
    list, the fixed slots, and both in one block): (1) within the parity tolerance of
    the oracle applying every call in order; (2) bit-identical to a second engine that gets only
    each block's last-wins equivalent -- the device applies the host's per-voice fold exactly as the
    calls would compose one by one."""
    from ol_dsp_amd import _lib
    n, blocks = 200, 24
    rng = np.random.default_rng(303)
    cfg = voice_configs(rng, n)
    cfg[15, :] = rng.uniform(0.0, 0.01, n).astype(np.float32)
    ea, eb = engine(kind, n), engine(kind, n)
    ref = O.Voice(n, moog=kind == "voice_moog")
    for e in (ea, eb):
        e.set_params(0, cfg)
    for i in range(n):
        ref.config(i, cfg[:, i])
    ya, yb, yr = [], [], []
    for b in range(blocks):
        evs_a, evs_b = [], []
        for i in np.flatnonzero(rng.random(n) < (0.5, 0.03, 0.1)[b % 3]):
            seq = []
            for _ in range(int(rng.integers(1, 5))):
                t = int(rng.integers(0, 5))
                seq.append((t, int(rng.integers(36, 97)), float(rng.uniform(50, 2000))))
            for t, note, hz in seq:
                evs_a.append((int(i), t, note, hz))
                ref.event(int(i), t, note, hz)
            for t, note, hz in _fold(seq):
                evs_b.append((int(i), t, note, hz))
        ea.voice_events(evs_a)
        eb.voice_events(evs_b)
        ya.append(_voice_run(ea, 256, cuda))
        yb.append(_voice_run(eb, 256, cuda))
        yr.append(ref.process(256))
    a, b_, r = np.concatenate(ya, 1), np.concatenate(yb, 1), np.concatenate(yr, 1)
    assert bits_equal(a, b_), first_mismatch(a, b_)
    assert np.all(np.isfinite(a))
    assert rel_err(a[0].T, r[0].T) <= VOICE_TOL
    assert _lib.EV_SET_FREQUENCY == 4


def test_voice_events_dead_lanes_and_ragged_groups(cuda):
    """Events on the last voice of a ragged engine (the dead lanes of its workgroup mirror it) and
    on group edges (voices 63, 64, 127): within tolerance of the oracle, and the engine's output of
    the last voice equals a 1-voice engine given the same calls (bit-identical)."""
    n = 130
    rng = np.random.default_rng(304)
    cfg = voice_configs(rng, n)
    e, one = engine("voice", n), engine("voice", 1)
    ref = O.Voice(n)
    e.set_params(0, cfg)
    one.set_params(0, cfg[:, n - 1:n])
    for i in range(n):
        ref.config(i, cfg[:, i])
    ys, y1, yr = [], [], []
    for b in range(12):
        who = [63, 64, 127, 128, n - 1]
        t = (1, 0, 2, 3, 4, 1)[b % 6]
        note = 40 + 3 * b
        e.voice_events([(i, t, note, 220.0 + b) for i in who])
        one.voice_events([(0, t, note, 220.0 + b)])
        for i in who:
            ref.event(i, t, note, 220.0 + b)
        ys.append(_voice_run(e, 256, cuda))
        y1.append(_voice_run(one, 256, cuda))
        yr.append(ref.process(256))
    y, a1, r = np.concatenate(ys, 1), np.concatenate(y1, 1), np.concatenate(yr, 1)
    assert bits_equal(y[:, :, n - 1:], a1), first_mismatch(y[:, :, n - 1:], a1)
    assert rel_err(y[0].T, r[0].T) <= VOICE_TOL


def test_tiled_frames_equal_short_calls(cuda):
    """olfx_process over planes the kernels' 32-bit offsets cannot span in one launch: 65,536
    chains x 8,192 frames (2 GiB per plane: frame tiles at the caller's plane distance) and 32,768
    choruses x 32,768 frames (4 GiB per plane: tiles staged through a compact buffer) are
    bit-identical to the same input given in 4,096-frame calls."""
    import torch
    for kind, n, frames in (("chain", 65536, 8192), ("chorus", 32768, 32768)):
        g = torch.Generator(device=cuda)
        g.manual_seed(305)
        x = torch.rand((2, frames, n), device=cuda, generator=g) - 0.5
        p = chorus_params(np.random.default_rng(305), n)
        big, small = engine(kind, n), engine(kind, n)
        if kind == "chain":
            rng = np.random.default_rng(306)
            p = np.concatenate([p, chorus_params(rng, n)[[0, 7]], dt_params(rng, n, 0.1)], 0)
        for e in (big, small):
            e.set_params(0, p)
        y = big.process(x)
        torch.cuda.synchronize()
        ok = True
        for f0 in range(0, frames, 4096):
            ys = small.process(x[:, f0:f0 + 4096].contiguous())
            ok = ok and torch.equal(ys.view(torch.int32), y[:, f0:f0 + 4096].view(torch.int32))
            del ys
        torch.cuda.synchronize()
        assert ok, kind
        assert big.frames_processed == small.frames_processed == frames
        del x, y, big, small
        torch.cuda.empty_cache()


@pytest.mark.parametrize("copy_bytes", [None, "0"])
def test_chain_controls_slot_reuse_across_streams(cuda, monkeypatch, copy_bytes):
    """40 blocks queued without a host wait, a parameter-list change before every block, the
    caller's stream alternating every block (each new stream ordered after the previous one, as a
    caller switching streams must): the 16 small zero-copy slots are reused (their group markers,
    flush_markers on each stream switch).  With OLFX_COPY_BYTES=0 every packet is copied through the
    two big slots: 40 large packets reuse them.  Bit-exact against the oracle given the same values
    at the same block boundaries."""
    import torch

    from ol_dsp_amd.engine import PARAMS
    if copy_bytes is not None:
        monkeypatch.setenv("OLFX_COPY_BYTES", copy_bytes)
    n, blocks = 96, 40
    rng = np.random.default_rng(320)
    pc, pp, pd = chorus_params(rng, n), chorus_params(rng, n)[[0, 7]], dt_params(rng, n, 0.05)
    e = engine("chain", n)
    e.set_params(0, np.concatenate([pc, pp, pd], 0))
    c1, c2, d = _chain_oracle(n, pc, pp, pd)
    names = PARAMS[e.kind]
    fields = [("chorus_depth", .08, 1), ("verb_decay", .25, .95), ("pitch_shift", 0, 3), ("chorus_rate", .01, 1)]
    x = fast_noise(n, 256 * blocks, seed=320)
    xd = torch.from_numpy(x).to(cuda)
    out = torch.empty((2, 256 * blocks, n), device=cuda)
    streams = [torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)]
    torch.cuda.synchronize()
    prev = torch.cuda.current_stream(cuda)
    yrs = []
    for b in range(blocks):
        fname, lo, hi = fields[b % len(fields)]
        sel = np.flatnonzero(rng.random(n) < 0.2).astype(np.uint32)
        vals = rng.uniform(lo, hi, len(sel)).astype(np.float32)
        e.set_param_list(fname, sel, vals)
        f = names.index(fname)
        for i, v in zip(sel, vals):
            if f < 8:
                c1.set(int(i), f, float(v))
            elif f < 10:
                c2.set(int(i), ("pitch", "window")[f - 8], float(v))
            else:
                d.set(int(i), f - 10, float(v))
        s = streams[b & 1]
        s.wait_stream(prev)
        xb = xd[:, 256 * b:256 * (b + 1)].contiguous()
        ob = out[:, 256 * b:256 * (b + 1)]
        with torch.cuda.stream(s):
            yb = e.process(xb, stream=s.cuda_stream)
            ob.copy_(yb)
        prev = s
        yrs.append(d.process(c2.process(c1.process(x[:, 256 * b:256 * (b + 1)]))))
    torch.cuda.synchronize()
    y, yr = out.cpu().numpy(), np.concatenate(yrs, 1)
    assert bits_equal(y, yr), first_mismatch(y, yr)


def test_stream_switch_is_ordered_by_the_engine(cuda):
    """Blocks alternating between two caller streams with NO ordering from the caller (no
    wait_stream, no event): the engine orders each block after the previous one at the switch
    (olfx.h, olfx_reset's note), so the state carries exactly -- bit-exact against the reference
    reverb's restatement over 12 blocks of 8,192 instances (a block takes ~0.1 ms, long enough for
    an unordered successor to overtake it)."""
    import torch
    n, blocks = 8192, 12
    rng = np.random.default_rng(322)
    p = dt_params(rng, n, 0.02)
    e = engine("dattorro", n)
    e.set_params(0, p)
    ref = O.Dattorro(n)
    for i in range(n):
        for f in range(7):
            ref.set(i, f, float(p[f, i]))
    x = fast_noise(n, 256 * blocks, seed=322)
    xd = torch.from_numpy(x).to(cuda)
    streams = [torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)]
    torch.cuda.synchronize()
    outs = []
    for b in range(blocks):
        s = streams[b & 1]
        with torch.cuda.stream(s):
            outs.append(e.process(xd[:, 256 * b:256 * (b + 1)].contiguous(), stream=s.cuda_stream))
    torch.cuda.synchronize()
    y = torch.cat(outs, 1).cpu().numpy()
    yr = ref.process(x)
    assert bits_equal(y, yr), first_mismatch(y, yr)


def test_stream_switch_through_the_mix_is_ordered(cuda):
    """olfx_process on one stream, olfx_mix on a second, the next olfx_process on a third, with no
    ordering from the caller: the mix is ordered after the block it sums, and the next
    block after the mix, hence after the previous block.  Voices and buses bit-identical to the
    same calls on one stream."""
    import torch
    n, blocks = 32768, 9
    cfg = voice_configs(np.random.default_rng(323), n)
    notes = [36 + (i % 60) for i in range(n)]
    buses = [list(range(g, g + 8)) for g in range(0, n, 8)]
    res = []
    for rotate in (False, True):
        e = engine("voice", n)
        e.set_params(0, cfg)
        e.note_events([(i, 1, notes[i]) for i in range(n)])
        e.mix_config(buses)
        streams = [torch.cuda.Stream(cuda) for _ in range(3)]
        outs = [torch.empty((1, 256, n), device=cuda) for _ in range(blocks)]
        bus = [torch.zeros((256, len(buses)), device=cuda) for _ in range(blocks)]
        torch.cuda.synchronize()
        for b in range(blocks):
            sp, sm = (streams[(2 * b) % 3], streams[(2 * b + 1) % 3]) if rotate else (streams[0], streams[0])
            e.process(None, out=outs[b], stream=sp.cuda_stream)
            e.mix(outs[b], bus[b], stream=sm.cuda_stream)
        torch.cuda.synchronize()
        res.append((torch.cat(outs, 1).cpu().numpy(), torch.cat(bus, 0).cpu().numpy()))
        e.close()
    assert bits_equal(res[1][0], res[0][0]), first_mismatch(res[1][0], res[0][0])
    assert bits_equal(res[1][1], res[0][1]), first_mismatch(res[1][1], res[0][1])
    assert np.any(res[0][1] != 0)


def test_reset_waits_for_the_engines_own_stream(cuda):
    """olfx_reset waits engine-scoped (the stream of its latest block, not the device): blocks
    queued on a caller stream without a host wait, then reset, then a block on the same stream --
    bit-identical to a freshly created engine's first block."""
    import torch
    n = 128
    rng = np.random.default_rng(321)
    p = dt_params(rng, n, 0.02)
    a, fresh = engine("dattorro", n), engine("dattorro", n)
    for e in (a, fresh):
        e.set_params(0, p)
    s = torch.cuda.Stream(cuda)
    x = torch.from_numpy(fast_noise(n, 256 * 8, seed=321)).to(cuda)
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        for b in range(6):
            a.process(x[:, 256 * b:256 * (b + 1)].contiguous(), stream=s.cuda_stream)
    a.reset()
    a.set_params(0, p)
    with torch.cuda.stream(s):
        ya = a.process(x[:, :256].contiguous(), stream=s.cuda_stream)
    yf = fresh.process(x[:, :256].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(ya.view(torch.int32), yf.view(torch.int32))


def test_set_member_after_update_is_refused(cuda):
    """olfx_set_member is the member write BEFORE Init/Update (the firmware's setup order); once a
    voice has been Update()d, members that feed the components only through Update() (resonance,
    drive, envelope times, portamento) are refused (OLFX_E_STATE) instead of acting like an Update()
    the reference would not run; the members SynthVoice::Process reads itself every sample
    (filter_cutoff, filter_env_amount, amp_env_amount, SynthVoice.h:42-52) are accepted at any time
    and take effect at the next block (test_voice_bit_exact_kernel_arith checks the audio)."""
    from ol_dsp_amd import _lib
    e = engine("voice", 4)
    lib, h = e.lib, e.handle
    assert lib.olfx_set_member(h, 1, 1, 0.5) == 0                 # before Update: accepted
    e.update(1, 1)
    assert lib.olfx_set_member(h, 1, 1, 0.9) == _lib.OLFX_E_STATE    # after: refused, unchanged
    assert e.get_param(1, "filter_resonance") == np.float32(0.5)
    for f in ("filter_attack", "portamento", "amp_sustain"):
        assert lib.olfx_set_member(h, 1, e.field(f), 0.3) == _lib.OLFX_E_STATE
    assert lib.olfx_set_member(h, 2, 1, 0.9) == 0                 # other voices untouched
    for f, v in (("filter_cutoff", 900.0), ("filter_env_amount", 0.25), ("amp_env_amount", 0.5)):
        assert lib.olfx_set_member(h, 1, e.field(f), v) == 0      # Process reads these: accepted
        assert e.get_param(1, f) == np.float32(v)
