/*
 * tests/cpp/test_ref_surface.cpp -- the reference's own types over the GPU (include/olfx_ref.hpp),
 * driven by the reference's own, unmodified headers (TEST INFRASTRUCTURE).
 *
 * Compiled by tests/cpp/Makefile's `test_ref_surface` recipe against
 *   /root/reference/modules/corelib/ol_corelib.h, cc_map.h          (ol::core::scale, the CC numbers)
 *   /root/reference/modules/synthlib/Voice.h, SoundSource.h           (the abstract Voice)
 *   /root/reference/modules/synthlib/Polyvoice.h, VoiceMap.h          (the voice containers)
 * exactly as they lie in the reference tree (include path only, nothing copied or stubbed).  The
 * binary is git-ignored and travels to the GPU box prebuilt, like oracle/_ref.
 *
 * Each case compares with the CPU oracle (oracle/liboracle.so) delayed by one block (the
 * per-sample pool's latency): bit-exact for the rack and the chorus, within 1e-5 of
 * max(|ref|, rms(ref)) for voices (the tolerance of tests/test_gpu_parity.py).
 */
#include <cstdint>  /* the reference headers use uint8_t and std::vector without including them */
#include <cstdio>
#include <vector>

#include "corelib/ol_corelib.h"
#include "synthlib/Polyvoice.h"
#include "synthlib/VoiceMap.h"

#include "olfx_ref.hpp"
#include "harness.h"

namespace {

constexpr uint32_t B = 256;

ol::synth::Voice::Config test_config(float cutoff) {
    ol::synth::Voice::Config c{};
    c.filter_cutoff = cutoff; c.filter_resonance = 0.3f; c.filter_drive = 0.1f; c.filter_env_amount = 0.5f;
    c.filter_attack = 0.01f; c.filter_attack_shape = 0.f; c.filter_decay = 0.2f; c.filter_sustain = 0.5f;
    c.filter_release = 0.1f; c.amp_env_amount = 1.f; c.amp_attack = 0.005f; c.amp_attack_shape = 0.f;
    c.amp_decay = 0.1f; c.amp_sustain = 0.7f; c.amp_release = 0.05f; c.portamento = 0.f;
    return c;
}

void config_values(const ol::synth::Voice::Config &c, float *v) {
    const float vals[OVC_NPARAMS] = {c.filter_cutoff, c.filter_resonance, c.filter_drive, c.filter_env_amount,
                                     c.filter_attack, c.filter_attack_shape, c.filter_decay, c.filter_sustain,
                                     c.filter_release, c.amp_env_amount, c.amp_attack, c.amp_attack_shape,
                                     c.amp_decay, c.amp_sustain, c.amp_release, c.portamento};
    std::memcpy(v, vals, sizeof vals);
}

/* |y(t) - ref(t - B)| <= 1e-5 * max(|ref|, rms(ref)) over t in [B, F), zeros before B */
bool close_delayed(const std::vector<float> &y, const std::vector<float> &ref, uint32_t F, const char *what) {
    double ss = 0, mx = 0, err = 0;
    for (uint32_t t = B; t < F; ++t) {
        const double a = ref[t - B];
        ss += a * a; mx = std::max(mx, std::fabs(a));
        err = std::max(err, std::fabs((double)y[t] - a));
    }
    for (uint32_t t = 0; t < B; ++t)
        if (y[t] != 0.f) { std::printf("  %s: nonzero output inside the latency\n", what); return false; }
    const double scale = std::max(mx, std::sqrt(ss / (F - B)));
    const bool ok = std::isfinite(err) && err <= 1e-5 * std::max(scale, 1e-30) && mx > 0;
    std::printf("  %s: max |err| %.3g, scale %.3g\n", what, err, scale);
    return ok;
}

/* one oracle voice per reference voice, events applied at block boundaries */
struct OracleVoices {
    oracle_voice *svf, *moog;
    std::vector<int> model;   /* per voice: 0 svf, 1 moog */
    std::vector<int> slot;    /* its index in that oracle */
    explicit OracleVoices(const std::vector<int> &models) : model(models) {
        int ns = 0, nm = 0;
        for (int m : models) slot.push_back(m ? nm++ : ns++);
        svf = oracle_voice_create_model(std::max(ns, 1), 48000.f, 0);
        moog = oracle_voice_create_model(std::max(nm, 1), 48000.f, 1);
    }
    ~OracleVoices() { oracle_voice_destroy(svf); oracle_voice_destroy(moog); }
    oracle_voice *of(size_t v) { return model[v] ? moog : svf; }
    void config(size_t v, const ol::synth::Voice::Config &c) {
        float vals[OVC_NPARAMS];
        config_values(c, vals);
        oracle_voice_config(of(v), slot[v], vals);
    }
    void event(size_t v, int type, int note, float value = 0.f) { oracle_voice_event(of(v), slot[v], type, note, value); }
    /* one frame of every voice (in voice order) */
    std::vector<float> frame() {
        std::vector<float> out(model.size());
        float ys[64], ym[64];
        oracle_voice_process(svf, ys, 1, 1);
        oracle_voice_process(moog, ym, 1, 1);
        for (size_t v = 0; v < model.size(); ++v) out[v] = model[v] ? ym[slot[v]] : ys[slot[v]];
        return out;
    }
};

}  // namespace

/* The reference's Polyvoice (Polyvoice.h:11-86, unmodified) over four GPU SynthVoices built the
   way the Daisy firmware builds them (ol_daisy/app/synth/main.cpp:48-53), two MoogFilter and two
   default (SvfFilter) voices; NoteOn takes the first voice not Playing(), NoteOff the one playing
   that note, Process sums with += in vector order. */
TEST(RefPolyvoice, SumsGpuVoicesInOrder) {
    const uint32_t F = 4 * B;
    ol::synth::SynthVoice v1(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v2(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v3;
    ol::synth::SynthVoice v4(new ol::synth::OscillatorSoundSource(), new ol::synth::SvfFilter(),
                             new ol::synth::DaisyAdsr(), new ol::synth::DaisyAdsr(), new ol::synth::DaisyPortamento());
    std::vector<ol::synth::Voice *> voices{&v1, &v2, &v3, &v4};
    ol::synth::Polyvoice poly(voices);
    EXPECT_TRUE(v1.moog() && v2.moog() && !v3.moog() && !v4.moog());
    poly.Init(48000.f);
    ol::synth::Voice::Config cfg = test_config(2500.f);
    poly.UpdateConfig(cfg);
    poly.NoteOn(60, 100);
    poly.NoteOn(64, 100);
    poly.NoteOn(67, 100);
    EXPECT_TRUE(v1.Playing() == 60 && v2.Playing() == 64 && v3.Playing() == 67 && v4.Playing() == 0);
    EXPECT_TRUE(v1.Gate() && !v4.Gate() && poly.Playing() == 0 && !poly.Gate());

    OracleVoices ref({1, 1, 0, 0});
    for (size_t v = 0; v < 4; ++v) ref.config(v, cfg);
    ref.event(0, 1, 60); ref.event(1, 1, 64); ref.event(2, 1, 67);

    std::vector<float> y(F), yr(F);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 9) poly.NoteOff(64, 0);          /* lands at frame 2B */
        if (t == 2 * B + 3) poly.NoteOn(72, 90);      /* the first free voice is v2 again; lands at 3B */
        float out = 0.f;                               /* the caller zeroes the frame */
        poly.Process(&out);
        y[t] = out;
    }
    EXPECT_TRUE(v2.Playing() == 72 && v4.Playing() == 0);
    for (uint32_t t = 0; t < F - B; ++t) {
        if (t == 2 * B) ref.event(1, 0, 64);
        if (t == 3 * B) ref.event(1, 1, 72);
        const std::vector<float> f = ref.frame();
        float out = 0.f;
        for (float s : f) out += s;                   /* Polyvoice.h:31 */
        yr[t] = out;
    }
    EXPECT_TRUE(close_delayed(y, yr, F, "Polyvoice sum"));
}

/* The reference's VoiceMap<1> (VoiceMap.h:14-84, unmodified): notes routed to voices by SetVoice,
   Process adds the mapped voices in note order; per-channel controls reach the channel's voice. */
TEST(RefVoiceMap, RoutesNotesAndSumsInNoteOrder) {
    const uint32_t F = 3 * B;
    ol::synth::SynthVoice a, b, c;
    ol::synth::VoiceMap<1> map;
    map.SetVoice(0, 36, &a);
    map.SetVoice(1, 38, &b);
    map.SetVoice(2, 42, &c);
    map.Init(48000.f);
    ol::synth::Voice::Config cfg = test_config(1800.f);
    a.UpdateConfig(cfg); b.UpdateConfig(cfg); c.UpdateConfig(cfg);
    map.NoteOn(36, 100);
    map.NoteOn(42, 100);
    map.NoteOn(50, 100);                              /* unmapped: nothing */
    map.UpdateMidiControl(2, CC_FILTER_CUTOFF, 90);   /* channel 2 -> c */

    OracleVoices ref({0, 0, 0});
    for (size_t v = 0; v < 3; ++v) ref.config(v, cfg);
    /* SynthVoice::UpdateMidiControl(CC_FILTER_CUTOFF, v): scale(v, 0,127, 0,20000, 2.5) (SynthVoice.h:171) */
    ol::synth::Voice::Config cc = cfg;
    cc.filter_cutoff = ol::core::scale(90, 0, 127, 0, 20000, 2.5);
    ref.config(2, cc);
    ref.event(0, 1, 36); ref.event(2, 1, 42);

    std::vector<float> y(F), yr(F);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 100) map.NoteOff(36, 0);
        float out[1] = {0.f};
        map.Process(out);
        y[t] = out[0];
    }
    for (uint32_t t = 0; t < F - B; ++t) {
        if (t == 2 * B) ref.event(0, 0, 36);
        const std::vector<float> f = ref.frame();
        float out = 0.f;
        for (float s : f) out += s;                   /* slots 36 < 38 < 42: voice order */
        yr[t] = out;
    }
    EXPECT_TRUE(close_delayed(y, yr, F, "VoiceMap sum"));
}

/* Voice.h's gate / pitch calls through the abstract interface: GateOff / GateOn (no retrigger) and
   SetFrequency (the oscillator follows the portamento'd frequency from the next boundary); an
   Update() without UpdateConfig ends SynthVoice::Init's component defaults with the members'
   defaults (SynthVoice.h:285-311). */
TEST(RefVoice, GateAndFrequencyThroughTheInterface) {
    const uint32_t F = 5 * B;
    ol::synth::SynthVoice sv, dv;
    ol::synth::Voice &v = sv, &d = dv;
    v.Init(48000.f);
    d.Init(48000.f);
    ol::synth::Voice::Config cfg = test_config(3000.f);
    cfg.portamento = 0.002f;
    v.UpdateConfig(cfg);
    d.Update();                                        /* member defaults into the components */
    v.NoteOn(57, 100);
    d.NoteOn(45, 100);

    OracleVoices ref({0, 0});
    ref.config(0, cfg);
    ol::synth::Voice::Config defaults{};
    defaults.filter_cutoff = 0.f; defaults.filter_resonance = 0.f; defaults.filter_drive = 0.f;
    defaults.filter_env_amount = 1.f; defaults.filter_attack = 0.f; defaults.filter_attack_shape = 1.f;
    defaults.filter_decay = 0.2f; defaults.filter_sustain = 0.f; defaults.filter_release = 0.f;
    defaults.amp_env_amount = 0.8f; defaults.amp_attack = 0.01f; defaults.amp_attack_shape = 1.f;
    defaults.amp_decay = 0.f; defaults.amp_sustain = 1.f; defaults.amp_release = 0.01f; defaults.portamento = 0.f;
    ref.config(1, defaults);
    ref.event(0, 1, 57);
    ref.event(1, 1, 45);

    std::vector<float> y(F), yd(F), yr(F), yrd(F);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 1) v.SetFrequency(523.25f);       /* lands at 2B */
        if (t == 2 * B + 2) v.GateOff();               /* lands at 3B */
        if (t == 3 * B + 3) { v.GateOn(); d.GateOff(); }   /* lands at 4B */
        v.Process(&y[t]);
        d.Process(&yd[t]);
    }
    EXPECT_TRUE(v.Gate() && v.Playing() == 57 && !d.Gate());
    for (uint32_t t = 0; t < F - B; ++t) {
        if (t == 2 * B) ref.event(0, 4, 0, 523.25f);
        if (t == 3 * B) ref.event(0, 3, 0);
        if (t == 4 * B) { ref.event(0, 2, 0); ref.event(1, 3, 0); }
        const std::vector<float> f = ref.frame();
        yr[t] = f[0];
        yrd[t] = f[1];
    }
    EXPECT_TRUE(close_delayed(y, yr, F, "SetFrequency / GateOff / GateOn"));
    EXPECT_TRUE(close_delayed(yd, yrd, F, "Update() with member defaults"));
}

/* ol::fx::FxRack<2>(DelayFx&, ReverbFx&, FilterFx&) built as the reference builds its components
   (ol_daisy/app/synth/main.cpp:55-67), controls on the components before Init and on the rack and
   components after it: bit-exact against the rack oracle with the reference's own mapping
   (ol::core::scale from the reference's ol_corelib.h), one block late. */
TEST(RefFxRack, ComponentsAndRackControlsBitExact) {
    const uint32_t n = 2, F = 4 * B;
    struct Lines { int dummy; };                       /* stands for the caller's DelayLine vector */
    std::vector<Lines *> delay_lines_a, delay_lines_b;
    struct Sc { int dummy; } verb_a, verb_b;           /* stands for the caller's daisysp::ReverbSc */
    ol::fx::DelayFx<2> delay_a(delay_lines_a), delay_b(delay_lines_b);
    ol::fx::DaisyVerb<2> dv_a(verb_a), dv_b(verb_b);
    ol::fx::ReverbFx<2> reverb_a(dv_a), reverb_b(dv_b);
    ol::fx::FilterFx<2> filter_a, filter_b;
    ol::fx::FxRack<2> rack_a(delay_a, reverb_a, filter_a), rack_b(delay_b, reverb_b, filter_b);
    ol::fx::FxRack<2> *racks[n] = {&rack_a, &rack_b};

    oracle_fxrack *ref = oracle_fxrack_create((int)n, 48000.f);
    /* before Init: a short delay on both, a band-pass filter1 on rack b, a delay cutoff that
       DelayFx::Init overrides (Fx.h:186-190) */
    delay_a.UpdateMidiControl(CC_DELAY_TIME, 2);
    delay_b.UpdateHardwareControl(CC_DELAY_TIME, 0.004f);
    delay_b.UpdateMidiControl(CC_DELAY_CUTOFF, 10);
    filter_b.UpdateMidiControl(CC_FILTER_TYPE, 30);
    filter_b.UpdateMidiControl(CC_FILTER_CUTOFF, 70);
    rack_a.Init(48000.f);
    rack_b.Init(48000.f);
    oracle_fxrack_set(ref, 0, OFR_DELAY_TIME, ol::core::scale(2, 0, 127, 0, 1, 1));
    oracle_fxrack_set(ref, 1, OFR_DELAY_TIME, 0.004f);
    oracle_fxrack_set(ref, 1, OFR_FILTER_TYPE, (float)(int)ol::core::scale(30, 0, 127, 0, 5, 1));
    oracle_fxrack_set(ref, 1, OFR_FILTER_CUTOFF, ol::core::scale(70, 0, 127, 0, 20000, 1));

    std::vector<float> x = noise(2, F, n, 77), y(2 * (size_t)F * n);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 5) {                              /* land at 2B */
            rack_a.UpdateMidiControl(CC_CTL_VOLUME, 100);
            reverb_b.UpdateHardwareControl(CC_REVERB_BALANCE, 0.5f);
            delay_a.UpdateMidiControl(CC_DELAY_FEEDBACK, 90);
            filter_a.UpdateHardwareControl(CC_FILTER_RESONANCE, 0.4f);
            reverb_a.UpdateMidiControl(CC_REVERB_TIME, 99);   /* reaches only the ReverbSc stub */
        }
        for (uint32_t i = 0; i < n; ++i) {
            const float in[2] = {x[(size_t)t * n + i], x[((size_t)F + t) * n + i]};
            float out[2];
            racks[i]->Process(in, out);
            y[(size_t)t * n + i] = out[0];
            y[((size_t)F + t) * n + i] = out[1];
        }
    }
    std::vector<float> yr(y.size());
    uint32_t done = 0;
    yr = run_blocks([&](const float *xi, float *yo, uint32_t b) {
        if (done == 2 * B) {
            oracle_fxrack_set(ref, 0, OFR_MASTER_VOLUME, ol::core::scale(100, 0, 127, 0, 1, 1));
            oracle_fxrack_set(ref, 1, OFR_REVERB_BALANCE, 0.5f);
            oracle_fxrack_set(ref, 0, OFR_DELAY_FEEDBACK, ol::core::scale(90, 0, 127, 0, 1, 1));
            oracle_fxrack_set(ref, 0, OFR_FILTER_RESONANCE, 0.4f);
        }
        oracle_fxrack_process(ref, xi, yo, (int)b, 1);
        done += b;
    }, x, 2, 2, F, n, B);
    bool ok = true;
    for (uint32_t c = 0; c < 2 && ok; ++c)
        for (uint32_t t = 0; t < F && ok; ++t)
            for (uint32_t i = 0; i < n && ok; ++i) {
                const float want = t < B ? 0.f : yr[((size_t)c * F + t - B) * n + i];
                ok = std::memcmp(&y[((size_t)c * F + t) * n + i], &want, 4) == 0;
                if (!ok) std::printf("  first mismatch c=%u t=%u i=%u: %.9g vs %.9g\n", c, t, i,
                                     y[((size_t)c * F + t) * n + i], want);
            }
    EXPECT_TRUE(ok);
    oracle_fxrack_destroy(ref);

    int code = 0;                                      /* a rack's component is run by its rack */
    float in2[2] = {0.f, 0.f}, out2[2];
    try { filter_a.Process(in2, out2); } catch (const olfx::Error &e) { code = e.code(); }
    EXPECT_EQ(code, OLFX_E_STATE);
    code = 0;
    ol::fx::FilterFx<2> lone;                          /* ... and a lone one needs its Init */
    try { lone.Process(in2, out2); } catch (const olfx::Error &e) { code = e.code(); }
    EXPECT_EQ(code, OLFX_E_STATE);
}

/* The Daisy synth firmware, ol_daisy/app/synth/main.cpp: its objects built as it builds them
   (:48-67), its voice set-up before Init (:114-128, 149-152), MIDI control changes fanned out to all
   four objects as handleMidi does (:201-207), and the body of audio_callback (:78-88) run verbatim
   over an interleaved AUDIO_BLOCK_SIZE buffer.  The objects are the GPU's (olfx_ref.hpp): the four
   MoogFilter voices one generation, delay_fx / reverb_fx / filter_fx standalone rack instances
   (OLFX_FR_TOPOLOGY 2 / 3 / 4), each object one block late.
   Checks: (1) the fx chain is bit-exact against oracle/fxrack_ref.c topology 1 (the firmware's
   chain as one instance) fed the voices' GPU output, 3 blocks late (delay, reverb, filter);
   (2) that voice output is within the voice tolerance of the oracle voices (4 MoogFilter
   SynthVoices, members set before Init), 1 block late. */
TEST(RefFirmware, SynthCallbackVerbatim) {
    const uint32_t kBlocks = 10, F = kBlocks * B;
    struct DelayLine { int dummy; } delay_line1;        /* stands for daisysp::DelayLine<t_sample, 48000> */
    struct ReverbSc { int dummy; } verb;                /* stands for daisysp::ReverbSc */
    /* ---- main.cpp:48-67, verbatim but for the two stand-in types ---- */
    ol::synth::SynthVoice v1(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v2(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v3(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice v4(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    std::vector<ol::synth::Voice *> voices{&v1, &v2, &v3, &v4};
    ol::synth::Polyvoice voice(voices);
    std::vector<DelayLine *> delay_lines{&delay_line1};
    ol::fx::DelayFx<1> delay_fx(delay_lines);
    ol::fx::DaisyVerb<2> daisy_verb(verb);
    ol::fx::ReverbFx<2> reverb_fx(daisy_verb);
    ol::fx::FilterFx<2> filter_fx;
    t_sample mono = 0;
    t_sample stereo[]{0, 0};
    auto audio_callback = [&](const float *in, float *out, size_t size) {
        (void)in;
        /* ---- main.cpp:78-88, the loop body verbatim ---- */
        for (size_t i = 0; i < size; i += 2) {
            mono = 0;
            voice.Process(&mono);

            delay_fx.Process(&mono, &mono);
            stereo[0] = stereo[1] = mono;
            reverb_fx.Process(stereo, stereo);
            filter_fx.Process(stereo, stereo);
            out[i] = stereo[0];
            out[i + 1] = stereo[1];
        }
    };
    /* ---- main.cpp:114-128, 149-152 ---- */
    voice.UpdateMidiControl(CC_CTL_PORTAMENTO, 48);
    voice.UpdateMidiControl(CC_FILTER_CUTOFF, 0);
    voice.UpdateMidiControl(CC_FILTER_RESONANCE, 0);
    voice.UpdateMidiControl(CC_ENV_FILT_A, 0);
    voice.UpdateMidiControl(CC_ENV_FILT_D, 100);
    voice.UpdateMidiControl(CC_ENV_FILT_S, 0);
    voice.UpdateMidiControl(CC_ENV_FILT_R, 24);
    voice.UpdateMidiControl(CC_ENV_FILT_AMT, 127);
    voice.UpdateMidiControl(CC_ENV_AMP_A, 0);
    voice.UpdateMidiControl(CC_ENV_AMP_D, 127);
    voice.UpdateMidiControl(CC_ENV_AMP_S, 127);
    voice.UpdateMidiControl(CC_ENV_AMP_R, 100);
    voice.UpdateMidiControl(CC_OSC_1_VOLUME, 100);
    voice.UpdateMidiControl(CC_CTL_VOLUME, 80);
    const float sample_rate = 48000.f;
    voice.Init(sample_rate);
    delay_fx.Init(sample_rate);
    reverb_fx.Init(sample_rate);
    filter_fx.Init(sample_rate);
    /* handleMidi (main.cpp:190-207): notes to the Polyvoice, every CC to all four objects */
    auto cc = [&](uint8_t c, uint8_t v) {
        voice.UpdateMidiControl(c, v);
        delay_fx.UpdateMidiControl(c, v);
        reverb_fx.UpdateMidiControl(c, v);
        filter_fx.UpdateMidiControl(c, v);
    };
    std::vector<float> out(2 * (size_t)F);
    const size_t size = 2 * 128;                        /* AUDIO_BLOCK_SIZE 128, interleaved (main.cpp:22) */
    for (uint32_t f0 = 0; f0 < F; f0 += 128) {
        if (f0 == 0) { voice.NoteOn(48, 100); voice.NoteOn(55, 90); }
        if (f0 == 2 * B) { cc(CC_DELAY_TIME, 3); cc(CC_DELAY_FEEDBACK, 80); cc(CC_REVERB_BALANCE, 70); }
        if (f0 == 3 * B + 128) { cc(CC_FILTER_CUTOFF, 50); cc(CC_FILTER_RESONANCE, 40); voice.NoteOn(60, 100); }
        if (f0 == 5 * B) { cc(CC_FILTER_TYPE, 60); cc(CC_DELAY_BALANCE, 100); voice.NoteOff(48, 0); }
        audio_callback(nullptr, out.data() + 2 * (size_t)f0, size);
    }

    /* (1) the voices' GPU output: the same objects, configured and driven the same way, alone */
    ol::synth::SynthVoice w1(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice w2(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice w3(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    ol::synth::SynthVoice w4(new ol::synth::OscillatorSoundSource(), new ol::synth::MoogFilter());
    std::vector<ol::synth::Voice *> wv{&w1, &w2, &w3, &w4};
    ol::synth::Polyvoice wpoly(wv);
    const uint8_t setup[][2] = {{CC_CTL_PORTAMENTO, 48}, {CC_FILTER_CUTOFF, 0}, {CC_FILTER_RESONANCE, 0},
                                {CC_ENV_FILT_A, 0}, {CC_ENV_FILT_D, 100}, {CC_ENV_FILT_S, 0}, {CC_ENV_FILT_R, 24},
                                {CC_ENV_FILT_AMT, 127}, {CC_ENV_AMP_A, 0}, {CC_ENV_AMP_D, 127}, {CC_ENV_AMP_S, 127},
                                {CC_ENV_AMP_R, 100}, {CC_OSC_1_VOLUME, 100}, {CC_CTL_VOLUME, 80}};
    for (auto &c : setup) wpoly.UpdateMidiControl(c[0], c[1]);
    wpoly.Init(sample_rate);
    std::vector<float> m(F);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == 0) { wpoly.NoteOn(48, 100); wpoly.NoteOn(55, 90); }
        if (t == 3 * B + 128) { wpoly.UpdateMidiControl(CC_FILTER_CUTOFF, 50); wpoly.UpdateMidiControl(CC_FILTER_RESONANCE, 40);
                                wpoly.NoteOn(60, 100); }
        if (t == 5 * B) { wpoly.UpdateMidiControl(CC_FILTER_TYPE, 60); wpoly.NoteOff(48, 0); }
        if (t == 2 * B) { wpoly.UpdateMidiControl(CC_DELAY_TIME, 3); wpoly.UpdateMidiControl(CC_DELAY_FEEDBACK, 80);
                          wpoly.UpdateMidiControl(CC_REVERB_BALANCE, 70); }
        if (t == 5 * B) wpoly.UpdateMidiControl(CC_DELAY_BALANCE, 100);
        float s = 0.f;
        wpoly.Process(&s);
        m[t] = s;
    }
    /* The chain oracle: one topology-1 rack instance fed delay_fx's input stream, which is m (both
       are the Polyvoice's output at the caller's frame).  Each fx object is one block late, so
       reverb_fx sees the chain's input one block behind and filter_fx two: a control that lands at
       caller boundary T reaches the chain's input frame T (delay_fx), T - B (reverb_fx) or T - 2B
       (filter_fx); the chain's output frame t is out[t + 3B]. */
    oracle_fxrack *ref = oracle_fxrack_create(1, sample_rate);
    oracle_fxrack_set(ref, 0, OFR_TOPOLOGY, 1.f);
    std::vector<float> yr(2 * (size_t)F, 0.f);
    auto at = [&](uint32_t t) {
        if (t == 2 * B) { oracle_fxrack_set(ref, 0, OFR_DELAY_TIME, ol::core::scale(3, 0, 127, 0, 1, 1));
                          oracle_fxrack_set(ref, 0, OFR_DELAY_FEEDBACK, ol::core::scale(80, 0, 127, 0, 1, 1)); }
        if (t == 2 * B - B) oracle_fxrack_set(ref, 0, OFR_REVERB_BALANCE, ol::core::scale(70, 0, 127, 0, 1, 1));
        /* called mid-block at 3B + 128: lands at 4B */
        if (t == 4 * B - 2 * B) { oracle_fxrack_set(ref, 0, OFR_FILTER_CUTOFF, ol::core::scale(50, 0, 127, 0, 20000, 1));
                                  oracle_fxrack_set(ref, 0, OFR_FILTER_RESONANCE, ol::core::scale(40, 0, 127, 0, 1, 1)); }
        if (t == 5 * B - 2 * B) oracle_fxrack_set(ref, 0, OFR_FILTER_TYPE, (float)(int)ol::core::scale(60, 0, 127, 0, 5, 1));
        if (t == 5 * B) oracle_fxrack_set(ref, 0, OFR_DELAY_BALANCE, ol::core::scale(100, 0, 127, 0, 1, 1));
    };
    for (uint32_t t = 0; t + 3 * B < F; ++t) {
        at(t);
        const float x[2] = {m[t], 0.f};
        float y[2];
        oracle_fxrack_process(ref, x, y, 1, 1);
        yr[2 * (size_t)(t + 3 * B)] = y[0];
        yr[2 * (size_t)(t + 3 * B) + 1] = y[1];
    }
    oracle_fxrack_destroy(ref);
    const size_t bad = first_bit_mismatch(out, yr);
    if (bad != (size_t)-1) std::printf("  first mismatch at %zu: %.9g vs %.9g\n", bad, out[bad], yr[bad]);
    EXPECT_TRUE(bad == (size_t)-1);
    bool moving = false;
    for (uint32_t t = 5 * B; t < F; ++t) moving = moving || out[2 * (size_t)t] != 0.f;
    EXPECT_TRUE(moving);

    /* (2) the voices against the oracle: members set before Init (no Update), then the notes */
    OracleVoices vref({1, 1, 1, 1});
    float mem[OVC_NPARAMS] = {0.f, 0.f, 0.f, 1.f, 0.f, 1.f, 0.2f, 0.f, 0.f, 0.8f, 0.01f, 1.f, 0.f, 1.f, 0.01f, 0.f};
    mem[OVC_PORTAMENTO] = ol::core::scale(48, 0, 127, 0, 1, 4);          /* SynthVoice.h:164-229 */
    mem[OVC_FILTER_CUTOFF] = ol::core::scale(0, 0, 127, 0, 20000, 2.5);
    mem[OVC_FILTER_RESONANCE] = 0.f;
    mem[OVC_FILTER_ATTACK] = 0.f;
    mem[OVC_FILTER_DECAY] = ol::core::scale(100, 0, 127, 0, 1, 3);
    mem[OVC_FILTER_SUSTAIN] = 0.f;
    mem[OVC_FILTER_RELEASE] = ol::core::scale(24, 0, 127, 0, 1, 1);
    mem[OVC_FILTER_ENV_AMOUNT] = ol::core::scale(127, 0, 127, 0, 1, 1);
    mem[OVC_AMP_ATTACK] = 0.f;
    mem[OVC_AMP_DECAY] = ol::core::scale(127, 0, 127, 0, 1, 1);
    mem[OVC_AMP_SUSTAIN] = ol::core::scale(127, 0, 127, 0, 1, 1);
    mem[OVC_AMP_RELEASE] = ol::core::scale(100, 0, 127, 0, 1, 1);
    mem[OVC_AMP_ENV_AMOUNT] = ol::core::scale(80, 0, 127, 0, 1, 1);
    for (size_t v = 0; v < 4; ++v) oracle_voice_init_members(vref.of(v), vref.slot[v], mem);
    std::vector<float> mr(F, 0.f);
    for (uint32_t t = 0; t + B < F; ++t) {
        if (t == 0) { vref.event(0, 1, 48); vref.event(1, 1, 55); }
        if (t == 4 * B) {                               /* CUTOFF / RESONANCE -> Update() of every voice */
            for (size_t v = 0; v < 4; ++v) {
                float cfg[OVC_NPARAMS];
                std::memcpy(cfg, mem, sizeof cfg);
                cfg[OVC_FILTER_CUTOFF] = ol::core::scale(50, 0, 127, 0, 20000, 2.5);
                cfg[OVC_FILTER_RESONANCE] = ol::core::scale(40, 0, 127, 0, 1, 1);
                oracle_voice_config(vref.of(v), vref.slot[v], cfg);
            }
            vref.event(2, 1, 60);
        }
        if (t == 5 * B) vref.event(0, 0, 48);
        const std::vector<float> f = vref.frame();
        float s = 0.f;
        for (float x : f) s += x;
        mr[t] = s;
    }
    EXPECT_TRUE(close_delayed(m, mr, F, "firmware voices (members before Init)"));
}

/* ol::fx::ChorusFx<2> (stereo) and <1> (mono: L = R = x, out = L) against the chorus oracle. */
TEST(RefChorusFx, StereoAndMonoBitExact) {
    const uint32_t F = 3 * B;
    ol::fx::ChorusFx<2> st;
    ol::fx::ChorusFx<1> mono;
    st.Init(48000.f);
    mono.Init(48000.f);
    st.setDepth(0.7f); st.setRate(0.6f); st.setPitch(1.5f);
    mono.setDepth(0.3f); mono.setMix(0.8f);
    oracle_chorus *ref = oracle_chorus_create(2, 48000.f, 0);
    oracle_chorus_set(ref, 0, OCH_DEPTH, 0.7f); oracle_chorus_set(ref, 0, OCH_RATE, 0.6f);
    oracle_chorus_set(ref, 0, OCH_PITCH, 1.5f);
    oracle_chorus_set(ref, 1, OCH_DEPTH, 0.3f); oracle_chorus_set(ref, 1, OCH_MIX, 0.8f);
    std::vector<float> xs = noise(2, F, 1, 5), xm = noise(1, F, 1, 6);
    std::vector<float> ys(2 * (size_t)F), ym(F);
    for (uint32_t t = 0; t < F; ++t) {
        const float in[2] = {xs[t], xs[F + t]};
        float out[2];
        st.Process(in, out);
        ys[t] = out[0]; ys[F + t] = out[1];
        mono.Process(&xm[t], &ym[t]);
    }
    /* oracle input [2][F][2]: instance 0 stereo, instance 1 mono on both channels */
    std::vector<float> x((size_t)2 * F * 2), yr(x.size());
    for (uint32_t t = 0; t < F; ++t) {
        x[(size_t)t * 2 + 0] = xs[t]; x[((size_t)F + t) * 2 + 0] = xs[F + t];
        x[(size_t)t * 2 + 1] = xm[t]; x[((size_t)F + t) * 2 + 1] = xm[t];
    }
    oracle_chorus_process(ref, x.data(), yr.data(), (int)F, 1);
    bool ok = true;
    for (uint32_t t = 0; t < F && ok; ++t) {
        const bool early = t < B;
        const float wl = early ? 0.f : yr[(size_t)(t - B) * 2], wr = early ? 0.f : yr[((size_t)F + t - B) * 2];
        const float wm = early ? 0.f : yr[(size_t)(t - B) * 2 + 1];
        ok = std::memcmp(&ys[t], &wl, 4) == 0 && std::memcmp(&ys[F + t], &wr, 4) == 0 && std::memcmp(&ym[t], &wm, 4) == 0;
        if (!ok) std::printf("  first mismatch t=%u\n", t);
    }
    EXPECT_TRUE(ok);
    oracle_chorus_destroy(ref);
}

int main() { return run_all_tests(); }
