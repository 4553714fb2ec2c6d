/*
 * include/olfx_fx.hpp -- C++ operator surface over the olfx C-ABI (header-only).
 *
 * These classes give reference callers the method names and argument meanings of the reference
 * effect operators. Each object holds N instances and processes whole blocks on the GPU:
 *
 *   olfx::ReverbBank  <- ol::fx::Reverb (modules/fxlib/Reverb.h:43-66) backed by DattorroVerb
 *                        (libs/dattorro-verb/verb.h:5-26). The stereo -> (l+r)/2 -> L/R glue
 *                        follows ReverbFx.cpp:11-27.
 *   olfx::ChorusBank  <- ChorusEffect (README.md:114-128: init / setDepth / setRate / process),
 *                        which wraps the RNBO stereo chorus. Its params follow
 *                        modules/rnbo/patcher/mono-chorus.rnbopat.
 *   olfx::PitchShiftBank <- gen~ pitchshift (modules/rnbo/patcher/pitchshift.gendsp)
 *   olfx::VoiceBank   <- ol::synth::SynthVoice (modules/synthlib/SynthVoice.h:31-98, :245-256):
 *                        Init / UpdateConfig / NoteOn / NoteOff / Process.
 *
 * and, one object per reference object (include/olfx_sample.h: per-sample calls batched into one
 * GPU block per generation; D blocks of latency and any call order within D blocks, D = the pool
 * depth, 1 by default: frame-major calls):
 *   olfx::ChorusEffect <- ChorusEffect (README.md:114-128): init / setDepth / setRate / process(float)
 *   olfx::SynthVoice   <- ol::synth::SynthVoice (SynthVoice.h:31-256): Init / UpdateConfig / NoteOn /
 *                         NoteOff / UpdateMidiControl / UpdateHardwareControl / Process(frame_out)
 *   olfx::FxRack       <- ol::fx::FxRack<2> (Fx.h:398-492): Init / Process(frame_in, frame_out) /
 *                         UpdateMidiControl / UpdateHardwareControl
 *   olfx::Polyvoice    <- ol::synth::Polyvoice (Polyvoice.h:11-86): the NoteOn / NoteOff allocation
 *                         and the in-order sum of its SynthVoices
 *   olfx::VoiceMap<CH> <- ol::synth::VoiceMap<CH> (VoiceMap.h:14-84)
 *   (the reverb: DattorroVerb_* by name, include/olfx_dattorro.h)
 *
 * Each per-instance setter takes the same value as the reference setter and applies it at the
 * next Process call (block-boundary parameter updates, modules/juce/host/host.cpp:646-653).
 *
 * Error behaviour: the reference's setters and Process return void, and DattorroVerb_create
 * returns NULL on failure (verb.cpp:227). Here every failing C-ABI call throws olfx::Error,
 * carrying the OLFX_E_* code and olfx_last_error()'s text. Nothing fails silently, and there is
 * no CPU fallback: without a GPU, construction throws OLFX_E_NODEVICE.
 *
 * Audio buffers are [channel][frame][instance] float32. They are host pointers by default
 * (OLFX_IO_HOST: staged through pinned memory, PCIe-inclusive) or device pointers
 * (OLFX_IO_DEVICE: asynchronous on `stream`, the fast path).
 */
#ifndef OLFX_FX_HPP
#define OLFX_FX_HPP

#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "olfx.h"
#include "olfx_sample.h"

namespace olfx {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string &what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }
private:
    int code_;
};

inline void check(int rc, const olfx_engine *e, const char *call) {
    if (rc != OLFX_OK) {
        const char *msg = olfx_last_error(e);
        throw Error(rc, std::string(call) + ": " + (msg ? msg : "") + " (code " + std::to_string(rc) + ")");
    }
}

/* RAII owner of one engine: one effect kind x N instances on one GPU. */
class Engine {
public:
    Engine(int kind, uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0) {
        check(olfx_create(kind, device, n_inst, sample_rate, block, &e_), nullptr, "olfx_create");
    }
    ~Engine() { if (e_) olfx_destroy(e_); }
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    Engine(Engine &&o) noexcept : e_(std::exchange(o.e_, nullptr)) {}
    Engine &operator=(Engine &&o) noexcept {
        if (this != &o) { if (e_) olfx_destroy(e_); e_ = std::exchange(o.e_, nullptr); }
        return *this;
    }

    olfx_engine *handle() const { return e_; }
    uint32_t size() const { return olfx_num_instances(e_); }
    uint64_t frames_processed() const { return olfx_frames_processed(e_); }
    const char *kernel_name() const { return olfx_kernel_name(e_); }

    void set(uint32_t inst, uint32_t field, float v) {
        check(olfx_set_param(e_, inst, field, v), e_, "olfx_set_param");
    }
    float get(uint32_t inst, uint32_t field) const {
        float v = 0.f;
        check(olfx_get_param(e_, inst, field, &v), e_, "olfx_get_param");
        return v;
    }
    /* values: field-major [n_fields][count] for instances [first, first+count). */
    void set_block(uint32_t first, uint32_t count, uint32_t field0, uint32_t n_fields, const float *values) {
        check(olfx_set_params(e_, first, count, field0, n_fields, values), e_, "olfx_set_params");
    }
    /* One field, the same value for every instance. */
    void set_all(uint32_t field, float v) {
        std::vector<float> vals(size(), v);
        set_block(0, size(), field, 1, vals.data());
    }
    void process(const float *in, float *out, uint32_t n_frames, int io = OLFX_IO_HOST, void *stream = nullptr) {
        check(olfx_process(e_, in, out, n_frames, io, stream), e_, "olfx_process");
    }
    void sync() { check(olfx_sync(e_), e_, "olfx_sync"); }
    /* UpdateMidiControl / UpdateHardwareControl of the reference operator (SynthVoice.h:100-229,
       Fx.h:451-489): applied at the next process; controls the reference ignores are skipped. */
    void UpdateMidiControl(uint32_t i, uint8_t control, uint8_t value) { ctl(i, control, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint32_t i, uint8_t control, float value) { ctl(i, control, OLFX_CTL_HARDWARE, value); }
    void reset() { check(olfx_reset(e_), e_, "olfx_reset"); }

protected:
    void ctl(uint32_t i, uint8_t control, int source, float value) {
        olfx_control_event ev{};
        ev.inst = i; ev.control = control; ev.source = (uint8_t)source; ev.value = value;
        check(olfx_control(e_, &ev, 1), e_, "olfx_control");
    }
    olfx_engine *e_ = nullptr;
};

/* ol::fx::Reverb over N Dattorro plates (Reverb.h:43-66; setters verb.cpp:137-170). */
class ReverbBank : public Engine {
public:
    ReverbBank(uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0)
        : Engine(OLFX_KIND_DATTORRO, n_inst, sample_rate, block, device) {}
    /* Per instance, [0,1] x 4800 samples (verb.cpp:137-139); instances of one wave sharing a value
       keep the pre-delay tap's loads coalesced. */
    void SetPredelay(uint32_t i, float v) { set(i, OLFX_DT_PREDELAY, v); }
    void SetPredelay(float v) { set_all(OLFX_DT_PREDELAY, v); }
    void SetPrefilter(uint32_t i, float v) { set(i, OLFX_DT_PREFILTER, v); }
    void SetInputDiffusion1(uint32_t i, float v) { set(i, OLFX_DT_INPUT_DIFFUSION1, v); }
    void SetInputDiffusion2(uint32_t i, float v) { set(i, OLFX_DT_INPUT_DIFFUSION2, v); }
    void SetDecayDiffusion(uint32_t i, float v) { set(i, OLFX_DT_DECAY_DIFFUSION, v); }
    void SetDecay(uint32_t i, float v) { set(i, OLFX_DT_DECAY, v); }
    void SetDamping(uint32_t i, float v) { set(i, OLFX_DT_DAMPING, v); }
    /* frame_in [2][F][N] -> frame_out [2][F][N]; in = (l+r)/2 like ReverbFx::dattorro_process. */
    void Process(const float *frame_in, float *frame_out, uint32_t n_frames,
                 int io = OLFX_IO_HOST, void *stream = nullptr) {
        process(frame_in, frame_out, n_frames, io, stream);
    }
};

/* ChorusEffect (README.md:114-128) over N stereo RNBO choruses. Values are RNBO param values,
   clamped to @min/@max like RNBO (include/olfx.h OLFX_CH_*). */
class ChorusBank : public Engine {
public:
    ChorusBank(uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0)
        : Engine(OLFX_KIND_CHORUS, n_inst, sample_rate, block, device) {}
    void setDepth(uint32_t i, float v) { set(i, OLFX_CH_DEPTH, v); }
    void setRate(uint32_t i, float v) { set(i, OLFX_CH_RATE, v); }
    void setMix(uint32_t i, float v) { set(i, OLFX_CH_MIX, v); }
    void setCutoff(uint32_t i, float v) { set(i, OLFX_CH_CUTOFF, v); }
    void setQ(uint32_t i, float v) { set(i, OLFX_CH_Q, v); }
    void setPitch(uint32_t i, float v) { set(i, OLFX_CH_PITCH, v); }
    void setPhase(uint32_t i, float v) { set(i, OLFX_CH_PHASE, v); }
    void setWindow(uint32_t i, float v) { set(i, OLFX_CH_WINDOW, v); }
    /* [2][F][N] stereo in -> [2][F][N] stereo out */
    void process(const float *in, float *out, uint32_t n_frames, int io = OLFX_IO_HOST, void *stream = nullptr) {
        Engine::process(in, out, n_frames, io, stream);
    }
};

/* gen~ pitchshift (pitchshift.gendsp), stereo. */
class PitchShiftBank : public Engine {
public:
    PitchShiftBank(uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0)
        : Engine(OLFX_KIND_PITCHSHIFT, n_inst, sample_rate, block, device) {}
    void SetShift(uint32_t i, float hz) { set(i, OLFX_PS_SHIFT, hz); }
    void SetWindow(uint32_t i, float ms) { set(i, OLFX_PS_WINDOW, ms); }
};

/* ol::fx::FxRack<2> over N racks (modules/fxlib/Fx.h:398-492): DelayFx -> ReverbFx (over the
   in-tree ReverbSc stub) -> FilterFx -> master volume; stereo in, [2][F][N] out (channel 1 is 0,
   as in the reference: FilterFx writes only channel 0 of the rack's zeroed output buffer). */
class FxRackBank : public Engine {
public:
    FxRackBank(uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0)
        : Engine(OLFX_KIND_FXRACK, n_inst, sample_rate, block, device) {}
    void Process(const float *frame_in, float *frame_out, uint32_t n_frames,
                 int io = OLFX_IO_HOST, void *stream = nullptr) {
        process(frame_in, frame_out, n_frames, io, stream);
    }
    /* OLFX_FR_TOPOLOGY: FxRack<2>::Process (Fx.h:432-440), or the Daisy synth firmware's callback
       chain (ol_daisy/app/synth/main.cpp:78-86: mono in channel 0, delay, stereo copy, reverb,
       filter in place, no master) */
    enum class Topology { Rack = 0, DaisyFirmware = 1 };
    void SetTopology(uint32_t i, Topology t) { set(i, OLFX_FR_TOPOLOGY, static_cast<float>(t)); }
};

/* ol::synth::SynthVoice over N voices (SynthVoice.h). The config array is in Voice::Config field
   order (modules/synthlib/Voice.h:14-31 == OLFX_VC_*). Note events queue up and take effect at
   the next Process, in call order. */
class VoiceBank : public Engine {
public:
    /* filter: the SynthVoice's Filter (SynthVoice.h:22-29) -- SvfFilter (default, OLFX_KIND_VOICE)
     * or MoogFilter (OLFX_KIND_VOICE_MOOG, the Daisy synth firmware's voices, main.cpp:49-52) */
    enum class Filter { Svf, Moog };
    VoiceBank(uint32_t n_inst, float sample_rate, uint32_t block = 256, int device = 0, Filter filter = Filter::Svf)
        : Engine(filter == Filter::Moog ? OLFX_KIND_VOICE_MOOG : OLFX_KIND_VOICE, n_inst, sample_rate, block,
                 device) {}
    /* SynthVoice::UpdateConfig + Update (SynthVoice.h:55-98) */
    void UpdateConfig(uint32_t i, const float config[OLFX_VC_NPARAMS]) {
        set_block(i, 1, 0, OLFX_VC_NPARAMS, config);   /* [16][1] field-major == the config array */
    }
    void NoteOn(uint32_t i, uint8_t midi_note, uint8_t velocity) { push(i, OLFX_EV_NOTE_ON, midi_note, velocity); }
    void NoteOff(uint32_t i, uint8_t midi_note, uint8_t velocity) { push(i, OLFX_EV_NOTE_OFF, midi_note, velocity); }
    /* frame_out [1][F][N] */
    void Process(float *frame_out, uint32_t n_frames, int io = OLFX_IO_HOST, void *stream = nullptr) {
        process(nullptr, frame_out, n_frames, io, stream);
    }
    /* Buses: the Polyvoice / VoiceMap sums (Polyvoice.h:28-33, VoiceMap.h:64-73).  buses[b] lists the
       voices bus b adds, in order; each voice at most once (olfx_mix_config). */
    void SetBuses(const std::vector<std::vector<uint32_t>> &buses) {
        std::vector<uint32_t> off(1, 0), order;
        for (const auto &b : buses) {
            order.insert(order.end(), b.begin(), b.end());
            off.push_back((uint32_t)order.size());
        }
        check(olfx_mix_config(e_, (uint32_t)buses.size(), off.data(), order.data()), e_, "olfx_mix_config");
    }
    /* bus_out [F][n_buses] += each bus's voices of voice_out [1][F][N], added in bus order */
    void Mix(const float *voice_out, float *bus_out, uint32_t n_frames, int io = OLFX_IO_HOST, void *stream = nullptr) {
        check(olfx_mix(e_, voice_out, bus_out, n_frames, io, stream), e_, "olfx_mix");
    }

private:
    /* the engine queues note events itself and applies them, in call order, at the next process
       (olfx_note_events), so Engine::process (BlockAdapter) sees them too */
    void push(uint32_t i, uint8_t type, uint8_t note, uint8_t vel) {
        olfx_event ev{};
        ev.inst = i; ev.type = type; ev.note = note; ev.velocity = vel;
        check(olfx_note_events(e_, &ev, 1), e_, "olfx_note_events");
    }
};

/* ------------------------------------------------------------------------------------------
 * Per-instance, per-sample operators: the reference's objects one for one.  The k-th Process /
 * process call returns the reference's output of frame k - latency() (zeros before); setters,
 * notes and controls land at the next block boundary.  No instance of a generation may run the
 * pool depth D (1 by default: frame-major calls) blocks ahead of the slowest one
 * (include/olfx_sample.h); a violation throws OLFX_E_STATE.
 * ------------------------------------------------------------------------------------------ */
class SampleOperator {
public:
    SampleOperator() = default;
    SampleOperator(const SampleOperator &) = delete;
    SampleOperator &operator=(const SampleOperator &) = delete;
    ~SampleOperator() { release(); }
    uint32_t latency() const { return s_ ? olfx_sample_latency(s_) : 0; }
    void set(uint32_t field, float value) { check(olfx_sample_set_param(need(), field, value), nullptr, "olfx_sample_set_param"); }

protected:
    void create(int kind, float sample_rate) {
        release();
        check(olfx_sample_create(kind, sample_rate, &s_), nullptr, "olfx_sample_create");
    }
    void frame(const float *in, float *out) { check(olfx_sample_process(need(), in, out), nullptr, "olfx_sample_process"); }
    void note(uint8_t type, uint8_t midi_note, uint8_t velocity) {
        check(olfx_sample_note(need(), type, midi_note, velocity), nullptr, "olfx_sample_note");
    }
    void control(uint8_t cc, int source, float value) {
        check(olfx_sample_control(need(), cc, source, value), nullptr, "olfx_sample_control");
    }
    void voice_event(uint8_t type, uint8_t midi_note, uint8_t velocity, float value) {
        check(olfx_sample_voice_event(need(), type, midi_note, velocity, value), nullptr, "olfx_sample_voice_event");
    }
    void update() { check(olfx_sample_update(need()), nullptr, "olfx_sample_update"); }
    void set_member(uint32_t field, float value) {
        check(olfx_sample_set_member(need(), field, value), nullptr, "olfx_sample_set_member");
    }
    bool live() const { return s_ != nullptr; }

private:
    olfx_sample *need() const {
        if (!s_) throw Error(OLFX_E_STATE, "operator used before init()/Init()");
        return s_;
    }
    void release() {
        if (s_) olfx_sample_destroy(s_);
        s_ = nullptr;
    }
    olfx_sample *s_ = nullptr;
};

/* README.md:114-128's ChorusEffect: mono in, mono out.  The mono sample drives both channels of
   the stereo RNBO chorus, whose L and R are then identical (one LFO, stereo-chorus.rnbopat:546,
   1196); process returns L.  Values are RNBO param values, clamped to @min/@max. */
class ChorusEffect : public SampleOperator {
public:
    void init(float sample_rate) { create(OLFX_KIND_CHORUS, sample_rate); }
    void setDepth(float v) { set(OLFX_CH_DEPTH, v); }
    void setRate(float v) { set(OLFX_CH_RATE, v); }
    void setMix(float v) { set(OLFX_CH_MIX, v); }
    void setCutoff(float v) { set(OLFX_CH_CUTOFF, v); }
    void setQ(float v) { set(OLFX_CH_Q, v); }
    void setPitch(float v) { set(OLFX_CH_PITCH, v); }
    void setPhase(float v) { set(OLFX_CH_PHASE, v); }
    void setWindow(float v) { set(OLFX_CH_WINDOW, v); }
    float process(float in) {
        const float x[2] = {in, in};
        float y[2];
        frame(x, y);
        return y[0];
    }
};

/* ol::synth::SynthVoice (SynthVoice.h:31-256) with its SvfFilter or the Daisy firmware's
   MoogFilter (ol_daisy/app/synth/main.cpp:49-52). */
class SynthVoice : public SampleOperator {
public:
    enum class Filter { Svf, Moog };
    explicit SynthVoice(Filter filter = Filter::Svf) : kind_(filter == Filter::Moog ? OLFX_KIND_VOICE_MOOG : OLFX_KIND_VOICE) {}
    void Init(float sample_rate) { create(kind_, sample_rate); }
    /* Voice::Config in field order (Voice.h:14-31 == OLFX_VC_*), then Update() */
    void UpdateConfig(const float config[OLFX_VC_NPARAMS]) {
        for (uint32_t f = 0; f < OLFX_VC_NPARAMS; ++f) set(f, config[f]);
    }
    /* NoteOn / NoteOff also set Playing() and Gate() as SynthVoice.h:231-260 does (host side, at the
       call; the engine applies the note at the next block boundary) */
    void NoteOn(uint8_t midi_note, uint8_t velocity) {
        note(OLFX_EV_NOTE_ON, midi_note, velocity);
        gate_ = true;
        playing_ = midi_note;
    }
    void NoteOff(uint8_t midi_note, uint8_t velocity) {
        note(OLFX_EV_NOTE_OFF, midi_note, velocity);
        gate_ = false;
        playing_ = 0;
    }
    uint8_t Playing() const { return playing_; }
    bool Gate() const { return gate_; }
    void UpdateMidiControl(uint8_t control_, uint8_t value) { control(control_, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control_, float value) { control(control_, OLFX_CTL_HARDWARE, value); }
    /* frame_out[0] = this voice's sample (SynthVoice.h:41-53) */
    void Process(float *frame_out) { frame(nullptr, frame_out); }

private:
    int kind_;
    uint8_t playing_ = 0;
    bool gate_ = false;
};

/* ol::synth::Polyvoice (modules/synthlib/Polyvoice.h:11-86) over per-sample SynthVoices: NoteOn goes
   to the first voice not Playing(), NoteOff to the first voice Playing() that note, and Process
   adds each voice's sample into *frame_out in vector order (the caller zeroes it, as in the
   reference).  The batch form of the same sum is VoiceBank::SetBuses / Mix (olfx_mix). */
class Polyvoice {
public:
    explicit Polyvoice(std::vector<SynthVoice *> &voices) : voices_(voices) {}
    void Init(float sample_rate) { for (SynthVoice *v : voices_) v->Init(sample_rate); }
    void Process(float *frame_out) {
        for (SynthVoice *v : voices_) {
            v->Process(&frame_buffer_);
            *frame_out += frame_buffer_;
        }
    }
    void NoteOn(uint8_t note, uint8_t velocity) {
        for (SynthVoice *v : voices_)
            if (!v->Playing()) { v->NoteOn(note, velocity); break; }
    }
    void NoteOff(uint8_t note, uint8_t velocity) {
        for (SynthVoice *v : voices_)
            if (v->Playing() == note) { v->NoteOff(note, velocity); break; }
    }
    void UpdateMidiControl(uint8_t control, uint8_t value) { for (SynthVoice *v : voices_) v->UpdateMidiControl(control, value); }
    void UpdateHardwareControl(uint8_t control, float value) { for (SynthVoice *v : voices_) v->UpdateHardwareControl(control, value); }
    void UpdateConfig(const float config[OLFX_VC_NPARAMS]) { for (SynthVoice *v : voices_) v->UpdateConfig(config); }
    uint8_t Playing() const { return 0; }      /* Polyvoice.h:79-81 */
    bool Gate() const { return false; }        /* Polyvoice.h:83-85 */

private:
    std::vector<SynthVoice *> &voices_;
    float frame_buffer_ = 0.f;
};

/* ol::synth::VoiceMap<CHANNEL_COUNT> (modules/synthlib/VoiceMap.h:14-84): note -> voice slots.
   Process runs the voices of slots 0..127 in note order and adds frame_buffer[0..CH) into
   frame_out (SynthVoice writes channel 0 only, so the other channels add the buffer's zeros). */
template <int CHANNEL_COUNT>
class VoiceMap {
public:
    void NoteOn(uint8_t note, uint8_t velocity) {
        if (note < 128 && note2voice_[note].voice) note2voice_[note].voice->NoteOn(note, velocity);
    }
    void NoteOff(uint8_t note, uint8_t velocity) {
        if (note < 128 && note2voice_[note].voice) note2voice_[note].voice->NoteOff(note, velocity);
    }
    void SetVoice(uint8_t channel, uint8_t note, SynthVoice *voice) {
        if (note < 128 && channel < 16) {
            note2voice_[note] = Slot{voice, channel, note};
            channel2voice_[channel] = Slot{voice, channel, note};
        }
    }
    void Init(float sample_rate) {
        for (Slot &s : note2voice_)
            if (s.voice) s.voice->Init(sample_rate);
    }
    void Process(float *frame_out) {
        for (Slot &s : note2voice_) {
            if (!s.voice) continue;
            s.voice->Process(frame_buffer_);
            for (int i = 0; i < CHANNEL_COUNT; ++i) frame_out[i] += frame_buffer_[i];
        }
    }
    void UpdateMidiControl(uint8_t channel, uint8_t control, uint8_t value) {
        if (channel < 16 && channel2voice_[channel].voice) channel2voice_[channel].voice->UpdateMidiControl(control, value);
    }

private:
    struct Slot {
        SynthVoice *voice = nullptr;
        uint8_t channel = 0, note = 0;
    };
    Slot note2voice_[128] = {};
    Slot channel2voice_[16] = {};
    float frame_buffer_[CHANNEL_COUNT] = {};
};

/* ol::fx::FxRack<2> (Fx.h:398-492): delay -> reverb (ReverbSc stub) -> filter -> master volume.
   Members are the OLFX_FR_* fields (set(field, value)). */
class FxRack : public SampleOperator {
public:
    void Init(float sample_rate) { create(OLFX_KIND_FXRACK, sample_rate); }
    void Process(const float *frame_in, float *frame_out) { frame(frame_in, frame_out); }
    void UpdateMidiControl(uint8_t control_, uint8_t value) { control(control_, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control_, float value) { control(control_, OLFX_CTL_HARDWARE, value); }
};

}  // namespace olfx
#endif  // OLFX_FX_HPP
