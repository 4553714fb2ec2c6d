/*
 * include/olfx_ref.hpp -- the reference's own C++ types over the GPU engine (header-only).
 *
 * A reference caller keeps its source: it includes this header in place of
 * modules/synthlib/SynthVoice.h and modules/fxlib/Fx.h and links libolfx.so.  Every class here has
 * the reference's namespace, name, base class, constructor and methods:
 *
 *   ol::synth::Voice          modules/synthlib/Voice.h:12-57 (restated; include guard OL_SYNTH_VOICE,
 *                             so the reference's own Voice.h and this one are interchangeable)
 *   ol::synth::SoundSource<N> modules/synthlib/SoundSource.h:8-27 (restated; guard OL_DSP_SOUNDSOURCE_H)
 *   ol::synth::SynthVoice     modules/synthlib/SynthVoice.h:15-317: SynthVoice(SoundSource<1>*, Filter*,
 *                             Adsr*, Adsr*, Portamento*) : Voice -- Init / Update / UpdateConfig(Config&) /
 *                             Process / GateOn / GateOff / Gate / SetFrequency / NoteOn / NoteOff /
 *                             Playing / UpdateMidiControl / UpdateHardwareControl
 *   ol::synth::OscillatorSoundSource, SvfFilter, MoogFilter, DaisyAdsr, DaisyPortamento
 *                             the components SynthVoice is built from (OscillatorSoundSource.h, Filter.h,
 *                             Adsr.h, Portamento.h).  Here they are configuration tags: the voice
 *                             kernel runs them.  MoogFilter selects OLFX_KIND_VOICE_MOOG.
 *   ol::fx::FilterFx<CH>, DelayFx<CH>, DaisyVerb<CH>, ReverbFx<CH>
 *                             modules/fxlib/Fx.h:65-393, Reverb.h:67-124: the rack's components,
 *                             constructed as the reference constructs them (DelayFx(delay_lines),
 *                             DaisyVerb(verb), ReverbFx(daisy_verb), FilterFx())
 *   ol::fx::FxRack<2>         Fx.h:398-492: FxRack(DelayFx&, ReverbFx&, FilterFx&) -- Init / Process /
 *                             Update / UpdateMidiControl / UpdateHardwareControl
 *   ol::fx::ChorusFx<CH>      SURVEY 8b's duck-typed chorus (the fxlib surface, Fx.h:27-62, over the
 *                             RNBO stereo chorus): Init / Process / Update / UpdateMidiControl /
 *                             UpdateHardwareControl, plus the README ChorusEffect setters
 *
 * Compiling the reference's unmodified modules/synthlib/Polyvoice.h and VoiceMap.h against these
 * classes is tested (tests/cpp/test_ref_surface.cpp, recipe in tests/cpp/Makefile).
 *
 * Semantics: one object = one instance of the per-sample pool (include/olfx_sample.h): output is
 * the reference's output one block (olfx_sample_latency, default 256 frames) late; setters, notes,
 * gates and controls land at the first block boundary at or after the call; calls are frame-major
 * across the instances of a generation.  Errors throw olfx::Error (the reference returns void).
 * Gate() and Playing() are host-side and change at the call, as SynthVoice.h:231-262 does.
 *
 * FxRack's components: inside an FxRack<2>, FxRack::Init binds them to the rack's GPU instance and
 * their controls (before or after Init) reach it.  On their own -- the Daisy synth firmware's
 * delay_fx -> stereo copy -> reverb_fx -> filter_fx callback (ol_daisy/app/synth/main.cpp:78-88) --
 * Init gives each a GPU rack instance whose topology is the component alone (OLFX_FR_TOPOLOGY
 * 2 DelayFx, 3 ReverbFx, 4 FilterFx), so that callback compiles and runs unchanged; a chain of k
 * such objects is k blocks late (each object one block).
 */
#ifndef OLFX_REF_HPP
#define OLFX_REF_HPP

#include <cstdint>
#include <memory>
#include <vector>

#include "olfx_fx.hpp"

typedef float t_sample;   /* corelib/ol_corelib.h:23 */

#ifndef OL_SYNTH_VOICE
#define OL_SYNTH_VOICE
namespace ol::synth {
/* modules/synthlib/Voice.h:12-57, member for member */
class Voice {
public:
    struct Config {
        t_sample filter_cutoff;
        t_sample filter_resonance;
        t_sample filter_drive;
        t_sample filter_env_amount;
        t_sample filter_attack;
        t_sample filter_attack_shape;
        t_sample filter_decay;
        t_sample filter_sustain;
        t_sample filter_release;
        t_sample amp_env_amount;
        t_sample amp_attack;
        t_sample amp_attack_shape;
        t_sample amp_decay;
        t_sample amp_sustain;
        t_sample amp_release;
        t_sample portamento;
    };
    virtual void Init(t_sample sample_rate) = 0;
    virtual void Update() = 0;
    virtual void Process(t_sample *frame_out) = 0;
    virtual void UpdateMidiControl(uint8_t control, uint8_t value) = 0;
    virtual void UpdateHardwareControl(uint8_t control, t_sample value) = 0;
    virtual void UpdateConfig(Config &config) = 0;
    virtual void GateOn() = 0;
    virtual void GateOff() = 0;
    virtual bool Gate() = 0;
    virtual void SetFrequency(t_sample) = 0;
    virtual void NoteOn(uint8_t midi_note, uint8_t velocity) = 0;
    virtual void NoteOff(uint8_t midi_note, uint8_t velocity) = 0;
    virtual uint8_t Playing() = 0;
};
}  // namespace ol::synth
#endif  // OL_SYNTH_VOICE

#ifndef OL_DSP_SOUNDSOURCE_H
#define OL_DSP_SOUNDSOURCE_H
namespace ol::synth {
/* modules/synthlib/SoundSource.h:8-27 */
enum InitStatus { Ok, Error };
template <int SOUND_SOURCE>
class SoundSource {
public:
    virtual InitStatus Init(t_sample sample_rate) = 0;
    virtual void Process(t_sample *frame) = 0;
    virtual void GateOn() = 0;
    virtual void GateOff() = 0;
    virtual void SetFreq(t_sample freq) = 0;
};
}  // namespace ol::synth
#endif  // OL_DSP_SOUNDSOURCE_H

namespace ol::synth {

/* Voice components (SynthVoice.h:20-29 takes them by pointer).  Tags: the GPU voice kernel is the
   implementation; the objects carry only which component was chosen. */
class OscillatorSoundSource : public SoundSource<1> {   /* OscillatorSoundSource.h:12-38 (POLYBLEP_SAW) */
public:
    InitStatus Init(t_sample) override { return Ok; }
    void Process(t_sample *) override {}
    void GateOn() override {}
    void GateOff() override {}
    void SetFreq(t_sample) override {}
};
class Filter {                                          /* Filter.h:12-33 */
public:
    virtual ~Filter() = default;
};
class SvfFilter : public Filter {};                     /* Filter.h:65-108 (daisysp::Svf, Low()) */
class MoogFilter : public Filter {};                    /* Filter.h:35-63 (daisysp::LadderFilter) */
class Adsr {                                            /* Adsr.h:12-33 */
public:
    virtual ~Adsr() = default;
};
class DaisyAdsr : public Adsr {};                       /* Adsr.h:35-76 */
class Portamento {                                      /* Portamento.h:46-55 */
public:
    virtual ~Portamento() = default;
};
class DaisyPortamento : public Portamento {};           /* Portamento.h:57-76 */

/* ol::synth::SynthVoice (SynthVoice.h:15-317) on the GPU voice kernel. */
class SynthVoice : public Voice, private olfx::SampleOperator {
public:
    /* The reference's defaults are `new OscillatorSoundSource()`, `new SvfFilter()`, ... (SynthVoice.h:
       20-24); nullptr means the same default here.  The components are not owned (the reference
       never frees them either). */
    explicit SynthVoice(SoundSource<1> *sound_source = nullptr, Filter *filter = nullptr,
                        Adsr *filter_envelope = nullptr, Adsr *amp_envelope = nullptr,
                        Portamento *portamento = nullptr)
        : kind_(pick_kind(sound_source, filter, filter_envelope, amp_envelope, portamento)) {}

    /* SynthVoice::Init (SynthVoice.h:31-39).  Members set before it (the Daisy firmware's order,
       ol_daisy/app/synth/main.cpp:114-128 then :149) keep their values; the components start at
       DaisySP's defaults, as Init leaves them (olfx_set_member). */
    void Init(t_sample sample_rate) override {
        create(kind_, sample_rate);
        for (uint32_t f = 0; f < OLFX_VC_NPARAMS; ++f)
            if (pre_set_[f]) set_member(f, pre_[f]);
        playing_ = 0;
        gate_ = false;
    }
    void Update() override {
        if (live()) update();   /* before Init: Init resets the components anyway */
    }
    void Process(t_sample *frame_out) override { frame(nullptr, frame_out); }
    void UpdateMidiControl(uint8_t control_, uint8_t value) override { ctl(control_, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control_, t_sample value) override { ctl(control_, OLFX_CTL_HARDWARE, value); }
    /* copies the 16 members, then Update() (SynthVoice.h:55-76) */
    void UpdateConfig(Config &config) override {
        static constexpr t_sample Config::*kFields[OLFX_VC_NPARAMS] = {
            &Config::filter_cutoff, &Config::filter_resonance, &Config::filter_drive, &Config::filter_env_amount,
            &Config::filter_attack, &Config::filter_attack_shape, &Config::filter_decay, &Config::filter_sustain,
            &Config::filter_release, &Config::amp_env_amount, &Config::amp_attack, &Config::amp_attack_shape,
            &Config::amp_decay, &Config::amp_sustain, &Config::amp_release, &Config::portamento};
        if (!live()) {
            for (uint32_t f = 0; f < OLFX_VC_NPARAMS; ++f) { pre_[f] = config.*kFields[f]; pre_set_[f] = true; }
            return;
        }
        for (uint32_t f = 0; f < OLFX_VC_NPARAMS; ++f) set(f, config.*kFields[f]);
        update();
    }
    void GateOn() override {                           /* SynthVoice.h:231-234 */
        voice_event(OLFX_EV_GATE_ON, 0, 0, 0.f);
        gate_ = true;
    }
    void GateOff() override {                          /* :236-239 */
        voice_event(OLFX_EV_GATE_OFF, 0, 0, 0.f);
        gate_ = false;
    }
    bool Gate() override { return gate_; }
    void SetFrequency(t_sample freq) override { voice_event(OLFX_EV_SET_FREQUENCY, 0, 0, freq); }   /* :264-267 */
    void NoteOn(uint8_t midi_note, uint8_t velocity) override {                                     /* :245-251 */
        voice_event(OLFX_EV_NOTE_ON, midi_note, velocity, 0.f);
        gate_ = true;
        playing_ = midi_note;
    }
    void NoteOff(uint8_t midi_note, uint8_t velocity) override {                                    /* :253-256 */
        voice_event(OLFX_EV_NOTE_OFF, midi_note, velocity, 0.f);
        gate_ = false;
        playing_ = 0;
    }
    uint8_t Playing() override { return playing_; }

    using olfx::SampleOperator::latency;
    bool moog() const { return kind_ == OLFX_KIND_VOICE_MOOG; }

private:
    static int pick_kind(SoundSource<1> *src, Filter *filter, Adsr *fenv, Adsr *aenv, Portamento *port) {
        if (src && !dynamic_cast<OscillatorSoundSource *>(src))
            throw olfx::Error(OLFX_E_KIND, "SynthVoice: only OscillatorSoundSource runs on the GPU voice kernel");
        if ((fenv && !dynamic_cast<DaisyAdsr *>(fenv)) || (aenv && !dynamic_cast<DaisyAdsr *>(aenv)) ||
            (port && !dynamic_cast<DaisyPortamento *>(port)))
            throw olfx::Error(OLFX_E_KIND, "SynthVoice: only DaisyAdsr / DaisyPortamento run on the GPU voice kernel");
        if (!filter || dynamic_cast<SvfFilter *>(filter)) return OLFX_KIND_VOICE;
        if (dynamic_cast<MoogFilter *>(filter)) return OLFX_KIND_VOICE_MOOG;
        throw olfx::Error(OLFX_E_KIND, "SynthVoice: only SvfFilter / MoogFilter run on the GPU voice kernel");
    }
    /* a control before Init: the member it sets (SynthVoice::UpdateMidiControl's mapping,
       olfx_control_map), applied at Init without Update() */
    void ctl(uint8_t control_, int source, float value) {
        if (live()) return control(control_, source, value);
        uint32_t field;
        float v;
        const int rc = olfx_control_map(kind_, control_, source, value, &field, &v);
        if (rc == OLFX_IGNORED || (rc == OLFX_OK && field == OLFX_FIELD_UPDATE_ONLY)) return;
        if (rc != OLFX_OK) throw olfx::Error(rc, "SynthVoice control before Init");
        pre_[field] = v;
        pre_set_[field] = true;
    }
    int kind_;
    uint8_t playing_ = 0;
    bool gate_ = false;
    float pre_[OLFX_VC_NPARAMS] = {};
    bool pre_set_[OLFX_VC_NPARAMS] = {};
};

}  // namespace ol::synth

namespace ol::fx {

namespace detail {
/* One GPU rack instance (OLFX_KIND_FXRACK) with the per-sample calls public. */
class RackInstance : public olfx::SampleOperator {
public:
    void Init(float sample_rate) { create(OLFX_KIND_FXRACK, sample_rate); }
    void Process(const float *in, float *out) { frame(in, out); }
    void Control(uint8_t cc, int source, float value) { control(cc, source, value); }
};

/* A rack component.  Inside an FxRack<2> (FxRack::Init binds it) its controls go to the rack's
   instance; on its own -- the Daisy synth firmware's delay_fx / reverb_fx / filter_fx
   (ol_daisy/app/synth/main.cpp:55-67, 82-85) -- Init gives it a GPU rack instance of its own whose
   topology is the component alone (OLFX_FR_TOPOLOGY 2 / 3 / 4).  Controls given before either
   exists are kept and replayed, in order, when it does; a component that an FxRack binds after
   its own Init hands its instance over (the rack gets every control so far). */
class RackComponent {
public:
    explicit RackComponent(int topology) : topology_(topology) {}
    RackComponent(const RackComponent &) = delete;
    RackComponent &operator=(const RackComponent &) = delete;
    virtual ~RackComponent() = default;

    void bind(RackInstance *rack) {
        own_.reset();                               /* a rack member has no instance of its own */
        rack_ = rack;
        for (const Ctl &c : history_) deliver(c);   /* every control so far, in order */
        history_.clear();
    }
    void unbind(RackInstance *rack) { if (rack_ == rack) rack_ = nullptr; }

protected:
    /* Init outside a rack: the component's own instance (a rack member keeps the rack's) */
    void init_alone(float sample_rate) {
        if (rack_) return;
        own_.reset(new RackInstance());
        own_->Init(sample_rate);
        own_->set(OLFX_FR_TOPOLOGY, (float)topology_);
        for (const Ctl &c : history_) deliver(c);
    }
    /* one frame of the component alone: [2] in, [2] out, one block late */
    void process_alone(const float in[2], float out[2]) {
        if (rack_) throw olfx::Error(OLFX_E_STATE, "component of an FxRack: FxRack::Process runs it");
        if (!own_) throw olfx::Error(OLFX_E_STATE, "component used before Init");
        if (!processed_) history_.clear();          /* it runs alone from now on: no replay needed */
        processed_ = true;
        own_->Process(in, out);
    }
    void send(uint8_t cc, int source, float value) {
        const Ctl c{cc, source, value};
        if (rack_ || own_) deliver(c);
        /* kept for an FxRack that may bind it later (until it has run alone) */
        if (!rack_ && !processed_) history_.push_back(c);
    }
    /* the control's number at the rack's own map (FxRack forwards CC_FX_FILTER_* to its filter1 as
       CC_FILTER_*, Fx.h:451-470); 0 = no rack member takes it.  A component alone keeps its own
       numbers (the engine routes them by topology, olfx_control). */
    virtual uint8_t rack_cc(uint8_t cc) const { return cc; }

private:
    struct Ctl { uint8_t cc; int source; float value; };
    void deliver(const Ctl &c) {
        if (rack_) {
            if (const uint8_t rc = rack_cc(c.cc)) rack_->Control(rc, c.source, c.value);
        } else {
            own_->Control(c.cc, c.source, c.value);
        }
    }
    int topology_;
    bool processed_ = false;
    RackInstance *rack_ = nullptr;
    std::unique_ptr<RackInstance> own_;
    std::vector<Ctl> history_;
};

/* cc_map.h numbers (modules/corelib/cc_map.h:8-67) */
enum : uint8_t {
    kCtlVolume = 7, kReverbTime = 32, kReverbCutoff = 33, kReverbBalance = 34,
    kDelayTime = 35, kDelayFeedback = 36, kDelayCutoff = 37, kDelayResonance = 38, kDelayBalance = 39,
    kFilterCutoff = 41, kFilterResonance = 42, kFilterType = 43, kFilterDrive = 44,
    kFxFilterCutoff = 45, kFxFilterResonance = 46, kFxFilterType = 47, kFxFilterDrive = 48,
    kEarlyPredelay = 50, kReverbPredelay = 52, kReverbPrefilter = 53, kReverbInputDiffusion1 = 54,
    kReverbInputDiffusion2 = 55, kReverbDecayDiffusion = 56,
};

/* frame_in / frame_out of a CHANNEL_COUNT-channel component on the stereo instance */
template <int CH>
inline void to_stereo(const t_sample *in, float x[2], bool dup) { x[0] = in[0]; x[1] = CH > 1 ? in[1] : (dup ? in[0] : 0.f); }
}  // namespace detail

/* Fx.h:65-165: the Svf on channel 0 with the selected output (FilterFx::Process, Fx.h:88-108).  In an
   FxRack<2> it is filter1: CC_FILTER_* map to the rack's CC_FX_FILTER_* (Fx.h:451-462).  Alone
   (OLFX_FR_TOPOLOGY 4), channel 1 of frame_out is channel 1 of frame_in one block late: the reference
   leaves frame_out[1] unwritten, which in place -- the firmware's call -- keeps channel 1 of the input. */
template <int CHANNEL_COUNT>
class FilterFx : public detail::RackComponent {
public:
    FilterFx() : RackComponent(4) {}
    void Init(t_sample sample_rate) { init_alone(sample_rate); }
    void Update() {}
    void Process(const t_sample *frame_in, t_sample *frame_out) {
        float x[2], y[2];
        detail::to_stereo<CHANNEL_COUNT>(frame_in, x, false);
        process_alone(x, y);
        for (int c = 0; c < CHANNEL_COUNT; ++c) frame_out[c] = y[c];
    }
    void UpdateMidiControl(uint8_t control, uint8_t value) { route(control, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control, t_sample value) { route(control, OLFX_CTL_HARDWARE, value); }

private:
    void route(uint8_t control, int source, float value) {
        if (control >= detail::kFilterCutoff && control <= detail::kFilterDrive) send(control, source, value);
        /* anything else: ignored (Fx.h:131-133) */
    }
    uint8_t rack_cc(uint8_t cc) const override { return (uint8_t)(cc - detail::kFilterCutoff + detail::kFxFilterCutoff); }
};

/* Fx.h:168-268.  The delay lines are the GPU instance's ([n][48000][2] rings): the constructor takes
   the reference's `std::vector<daisysp::DelayLine<t_sample, MAX_DELAY> *> &` (any type) and ignores
   it.  Alone (OLFX_FR_TOPOLOGY 2) it is DelayFx<2>: channel 0 through its filter_, channel 1 not;
   DelayFx<1> is channel 0 of it. */
template <int CHANNEL_COUNT>
class DelayFx : public detail::RackComponent {
public:
    DelayFx() : RackComponent(2) {}
    template <class DelayLines>
    explicit DelayFx(DelayLines &) : RackComponent(2) {}
    /* DelayFx::Init (Fx.h:183-192): its filter_ at UpdateMidiControl(CC_FILTER_CUTOFF, 64) and
       (CC_FILTER_RESONANCE, 24) -- the rack's delay cutoff / resonance fields -- after any earlier
       control.  (Called again after processing started, it re-applies those settings; the delay
       lines keep their contents.) */
    void Init(t_sample sample_rate) {
        init_alone(sample_rate);
        send(detail::kDelayCutoff, OLFX_CTL_MIDI, 64.f);
        send(detail::kDelayResonance, OLFX_CTL_MIDI, 24.f);
    }
    void Update() {}
    void Process(const t_sample *frame_in, t_sample *frame_out) {
        float x[2], y[2];
        detail::to_stereo<CHANNEL_COUNT>(frame_in, x, false);
        process_alone(x, y);
        for (int c = 0; c < CHANNEL_COUNT; ++c) frame_out[c] = y[c];
    }
    void UpdateHardwareControl(uint8_t control, t_sample value) {   /* time / feedback / balance (Fx.h:220-240) */
        using namespace detail;
        if (control == kDelayTime || control == kDelayFeedback || control == kDelayBalance)
            send(control, OLFX_CTL_HARDWARE, value);
    }
    void UpdateMidiControl(uint8_t control, uint8_t value) {        /* + its filter's cutoff / resonance (:242-266) */
        using namespace detail;
        if (control >= kDelayTime && control <= kDelayBalance) send(control, OLFX_CTL_MIDI, value);
    }
};

/* Reverb.h:67-124 (over the in-tree daisysp::ReverbSc stub, Reverb.h:12-40): constructed from the
   caller's ReverbSc (any type, ignored: the stub's 0.8 gain runs in the rack kernel). */
template <int CHANNEL_COUNT>
class DaisyVerb {
public:
    template <class ReverbSc>
    explicit DaisyVerb(ReverbSc &) {}
};

/* Fx.h:270-393.  Of its members only `balance` reaches the output through the ReverbSc stub; the
   others are accepted and have no audible effect, as in the reference.  Alone (OLFX_FR_TOPOLOGY 3):
   per channel 0.8 in balance + in (1 - balance); ReverbFx<1> (DaisyVerb<1> feeds the one channel to
   both stub inputs, Reverb.h:82-91) is channel 0 of it. */
template <int CHANNEL_COUNT>
class ReverbFx : public detail::RackComponent {
public:
    explicit ReverbFx(DaisyVerb<CHANNEL_COUNT> &) : RackComponent(3) {}
    void Init(t_sample sample_rate) { init_alone(sample_rate); }
    void Update() {}
    void Process(const t_sample *frame_in, t_sample *frame_out) {
        float x[2], y[2];
        detail::to_stereo<CHANNEL_COUNT>(frame_in, x, true);
        process_alone(x, y);
        for (int c = 0; c < CHANNEL_COUNT; ++c) frame_out[c] = y[c];
    }
    void UpdateMidiControl(uint8_t control, uint8_t value) { route(control, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control, t_sample value) { route(control, OLFX_CTL_HARDWARE, value); }

private:
    void route(uint8_t control, int source, float value) {
        using namespace detail;
        switch (control) {
        case kReverbDecayDiffusion: case kReverbInputDiffusion1: case kReverbInputDiffusion2:
        case kReverbCutoff: case kReverbBalance: case kReverbPredelay: case kEarlyPredelay:
        case kReverbPrefilter: case kReverbTime:
            send(control, source, value);
            break;
        default: break;
        }
    }
};

/* Fx.h:396-490: delay -> reverb -> filter1 -> master volume, one GPU rack instance. */
template <int CHANNEL_COUNT>
class FxRack {
    static_assert(CHANNEL_COUNT == 2, "the GPU rack kernel is FxRack<2> (stereo)");

public:
    FxRack(DelayFx<CHANNEL_COUNT> &delay, ReverbFx<CHANNEL_COUNT> &reverb, FilterFx<CHANNEL_COUNT> &filter)
        : delay_(delay), reverb_(reverb), filter1_(filter) {}
    FxRack(const FxRack &) = delete;
    FxRack &operator=(const FxRack &) = delete;
    ~FxRack() {
        delay_.unbind(&rack_);
        reverb_.unbind(&rack_);
        filter1_.unbind(&rack_);
    }

    /* Fx.h:408-416: a fresh rack instance; the components' controls so far are replayed, then
       DelayFx::Init's own filter settings (UpdateMidiControl(CC_FILTER_CUTOFF, 64), (.., 24),
       Fx.h:186-190) are applied last, as the reference's Init does. */
    void Init(t_sample sample_rate) {
        rack_.Init(sample_rate);
        delay_.bind(&rack_);
        reverb_.bind(&rack_);
        filter1_.bind(&rack_);
        rack_.Control(detail::kDelayCutoff, OLFX_CTL_MIDI, 64.f);
        rack_.Control(detail::kDelayResonance, OLFX_CTL_MIDI, 24.f);
    }
    void Process(const t_sample *frame_in, t_sample *frame_out) { rack_.Process(frame_in, frame_out); }
    void Update() {}
    void UpdateMidiControl(uint8_t control, uint8_t value) { rack_.Control(control, OLFX_CTL_MIDI, value); }
    void UpdateHardwareControl(uint8_t control, t_sample value) { rack_.Control(control, OLFX_CTL_HARDWARE, value); }
    uint32_t latency() const { return rack_.latency(); }

private:
    DelayFx<CHANNEL_COUNT> &delay_;
    ReverbFx<CHANNEL_COUNT> &reverb_;
    FilterFx<CHANNEL_COUNT> &filter1_;
    detail::RackInstance rack_;
};

/* The chorus with the fxlib operator surface (Fx.h:27-62's shape) and the README ChorusEffect
   setters (README.md:114-128), over the RNBO stereo chorus.  CHANNEL_COUNT 1: the mono sample feeds
   both channels and frame_out[0] = L; 2: stereo.  No cc_map.h control addresses the chorus, so
   UpdateMidiControl / UpdateHardwareControl change nothing (as the reference's Update-only fx). */
template <int CHANNEL_COUNT>
class ChorusFx : private olfx::SampleOperator {
    static_assert(CHANNEL_COUNT == 1 || CHANNEL_COUNT == 2, "ChorusFx<1> or ChorusFx<2>");

public:
    void Init(t_sample sample_rate) { create(OLFX_KIND_CHORUS, sample_rate); }
    void Process(const t_sample *frame_in, t_sample *frame_out) {
        const float x[2] = {frame_in[0], frame_in[CHANNEL_COUNT - 1]};
        float y[2];
        frame(x, y);
        for (int c = 0; c < CHANNEL_COUNT; ++c) frame_out[c] = y[c];
    }
    void Update() {}
    void UpdateMidiControl(uint8_t, uint8_t) {}
    void UpdateHardwareControl(uint8_t, t_sample) {}
    void setDepth(t_sample v) { set(OLFX_CH_DEPTH, v); }
    void setRate(t_sample v) { set(OLFX_CH_RATE, v); }
    void setMix(t_sample v) { set(OLFX_CH_MIX, v); }
    void setCutoff(t_sample v) { set(OLFX_CH_CUTOFF, v); }
    void setQ(t_sample v) { set(OLFX_CH_Q, v); }
    void setPitch(t_sample v) { set(OLFX_CH_PITCH, v); }
    void setPhase(t_sample v) { set(OLFX_CH_PHASE, v); }
    void setWindow(t_sample v) { set(OLFX_CH_WINDOW, v); }
    using olfx::SampleOperator::latency;
};

}  // namespace ol::fx

#endif  // OLFX_REF_HPP
