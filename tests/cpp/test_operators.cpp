/*
 * tests/cpp/test_operators.cpp -- GPU parity of the C++ operator surface (include/olfx_fx.hpp).
 *
 * Written in the style of the reference's gtest suites (test/synth_test.cpp, test/fx_test.cpp):
 * the operators are driven through the same method names as the reference and compared with the
 * CPU oracle (oracle/liboracle.so, TEST INFRASTRUCTURE) on identical inputs. Dattorro, chorus
 * and pitch-shift must be bit-exact. The voice must be within 1e-5 of max(|ref|, rms(ref)), the
 * tolerance tests/test_gpu_parity.py documents for Svf's per-sample sinf.
 *
 * gtest is not in the image, so a small TEST/EXPECT harness stands in. The binary exits non-zero
 * on any failure. It needs a GPU; run it through tests/test_cpp_operators.py (-m gpu).
 */
#include <atomic>
#include <chrono>
#include <thread>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "olfx_adapter.hpp"
#include "olfx_fx.hpp"
#include "harness.h"


/* ol::fx::Reverb surface over N plates vs the bit-exact Dattorro oracle. */
TEST(Reverb, BankMatchesOracleBitExact) {
    const uint32_t n = 129, frames = 2048;
    olfx::ReverbBank verb(n, 48000.f);
    oracle_dattorro *ref = oracle_dattorro_create((int)n);
    Lcg r(11);
    verb.SetPredelay(0.1f);
    for (uint32_t i = 0; i < n; ++i) {
        float pf = r.uni(.3f, 1.f), d1 = r.uni(.5f, .9f), d2 = r.uni(.4f, .8f), dd = r.uni(.4f, .9f);
        float dec = r.uni(.25f, .95f), damp = r.uni(.05f, .95f);
        verb.SetPrefilter(i, pf); verb.SetInputDiffusion1(i, d1); verb.SetInputDiffusion2(i, d2);
        verb.SetDecayDiffusion(i, dd); verb.SetDecay(i, dec); verb.SetDamping(i, damp);
        const float v[ODT_NPARAMS] = {0.1f, pf, d1, d2, dd, dec, damp};
        for (int f = 0; f < ODT_NPARAMS; ++f) oracle_dattorro_set(ref, (int)i, f, v[f]);
    }
    std::vector<float> x = noise(2, frames, n, 5);
    std::vector<float> y = run_blocks([&](const float *a, float *b, uint32_t f) { verb.Process(a, b, f); },
                                      x, 2, 2, frames, n, 256);
    std::vector<float> yr(y.size());
    oracle_dattorro_process(ref, x.data(), 2, yr.data(), (int)frames, 8);
    size_t k = first_bit_mismatch(y, yr);
    if (k != (size_t)-1) std::printf("  first mismatch at %zu: %.9g vs %.9g\n", k, y[k], yr[k]);
    EXPECT_TRUE(k == (size_t)-1);
    EXPECT_EQ(verb.frames_processed(), (uint64_t)frames);
    oracle_dattorro_destroy(ref);
}

/* ChorusEffect init / setDepth / setRate / process vs the chorus spec oracle (bit-exact). */
TEST(ChorusEffect, BankMatchesOracleBitExact) {
    const uint32_t n = 257, frames = 1024;
    olfx::ChorusBank chorus(n, 48000.f);
    oracle_chorus *ref = oracle_chorus_create((int)n, 48000.f, 0);
    Lcg r(12);
    for (uint32_t i = 0; i < n; ++i) {
        float v[OCH_NPARAMS] = {r.uni(0, 3), r.uni(0, 1), r.uni(0, .95f), r.uni(0, 1),
                                r.uni(0, 1), r.uni(.08f, 1), r.uni(.01f, 1), r.uni(4, 10)};
        chorus.setPitch(i, v[OCH_PITCH]); chorus.setMix(i, v[OCH_MIX]); chorus.setQ(i, v[OCH_Q]);
        chorus.setCutoff(i, v[OCH_CUTOFF]); chorus.setPhase(i, v[OCH_PHASE]);
        chorus.setDepth(i, v[OCH_DEPTH]); chorus.setRate(i, v[OCH_RATE]); chorus.setWindow(i, v[OCH_WINDOW]);
        for (int f = 0; f < OCH_NPARAMS; ++f) oracle_chorus_set(ref, (int)i, f, v[f]);
    }
    std::vector<float> x = noise(2, frames, n, 6);
    std::vector<float> y = run_blocks([&](const float *a, float *b, uint32_t f) { chorus.process(a, b, f); },
                                      x, 2, 2, frames, n, 256);
    std::vector<float> yr(y.size());
    oracle_chorus_process(ref, x.data(), yr.data(), (int)frames, 8);
    EXPECT_TRUE(first_bit_mismatch(y, yr) == (size_t)-1);
    oracle_chorus_destroy(ref);
}

TEST(PitchShift, BankMatchesOracleBitExact) {
    const uint32_t n = 64, frames = 1024;
    olfx::PitchShiftBank ps(n, 48000.f);
    oracle_chorus *ref = oracle_chorus_create((int)n, 48000.f, 1);
    Lcg r(13);
    for (uint32_t i = 0; i < n; ++i) {
        float s = r.uni(0, 3), w = r.uni(4, 10);
        ps.SetShift(i, s); ps.SetWindow(i, w);
        oracle_chorus_set(ref, (int)i, OCH_PITCH, s);
        oracle_chorus_set(ref, (int)i, OCH_WINDOW, w);
    }
    std::vector<float> x = noise(2, frames, n, 7);
    std::vector<float> y = run_blocks([&](const float *a, float *b, uint32_t f) { ps.process(a, b, f); },
                                      x, 2, 2, frames, n, 128);
    std::vector<float> yr(y.size());
    oracle_chorus_process(ref, x.data(), yr.data(), (int)frames, 8);
    EXPECT_TRUE(first_bit_mismatch(y, yr) == (size_t)-1);
    oracle_chorus_destroy(ref);
}

/* SynthVoice Init / UpdateConfig / NoteOn / NoteOff / Process vs the DaisySP restatement, for the
   SvfFilter voice and the MoogFilter (daisysp::LadderFilter) voice. */
static void voice_bank_matches_oracle(olfx::VoiceBank::Filter filter) {
    const uint32_t n = 96, half = 1024;
    olfx::VoiceBank voices(n, 48000.f, 256, 0, filter);
    oracle_voice *ref = oracle_voice_create_model((int)n, 48000.f, filter == olfx::VoiceBank::Filter::Moog);
    Lcg r(14);
    std::vector<uint8_t> notes(n);
    for (uint32_t i = 0; i < n; ++i) {
        float c[OLFX_VC_NPARAMS] = {r.uni(100, 8000), r.uni(0, .9f), r.uni(0, 1), r.uni(0, 1),
                                    r.uni(.001f, .5f), r.uni(0, 1), r.uni(.001f, .5f), r.uni(0, 1),
                                    r.uni(.001f, .5f), r.uni(.2f, 1), r.uni(.001f, .5f), r.uni(0, 1),
                                    r.uni(.001f, .5f), r.uni(0, 1), r.uni(.001f, .5f), r.uni(0, .05f)};
        notes[i] = (uint8_t)(36 + (i * 7) % 61);
        voices.UpdateConfig(i, c);
        voices.NoteOn(i, notes[i], 100);
        oracle_voice_config(ref, (int)i, c);
        oracle_voice_note(ref, (int)i, 1, notes[i]);
    }
    std::vector<float> y(2 * (size_t)half * n), yr(y.size());
    voices.Process(y.data(), half);
    oracle_voice_process(ref, yr.data(), (int)half, 8);
    for (uint32_t i = 0; i < n; ++i) {
        voices.NoteOff(i, notes[i], 0);
        oracle_voice_note(ref, (int)i, 0, notes[i]);
    }
    voices.Process(y.data() + (size_t)half * n, half);
    oracle_voice_process(ref, yr.data() + (size_t)half * n, (int)half, 8);
    for (uint32_t i = 0; i < n; ++i) {          /* per voice: |y - ref| <= 1e-5 * max(|ref|, rms) */
        double ss = 0, mx = 0, err = 0;
        for (uint32_t f = 0; f < 2 * half; ++f) {
            double a = yr[(size_t)f * n + i];
            ss += a * a; mx = std::max(mx, std::fabs(a));
            err = std::max(err, std::fabs((double)y[(size_t)f * n + i] - a));
        }
        double scale = std::max(mx, std::sqrt(ss / (2 * half)));
        EXPECT_TRUE(std::isfinite(err) && err <= 1e-5 * std::max(scale, 1e-30));
    }
    oracle_voice_destroy(ref);
}

TEST(Synth, VoiceBankMatchesOracle) { voice_bank_matches_oracle(olfx::VoiceBank::Filter::Svf); }

TEST(Synth, MoogVoiceBankMatchesOracle) { voice_bank_matches_oracle(olfx::VoiceBank::Filter::Moog); }

/* test/synth_test.cpp:102-148 pins: the first sample after NoteOn is exactly 0, and later
   samples are neither 0 nor 1. */
TEST(Synth, VoiceNoteOnOffPins) {
    olfx::VoiceBank v(1, 48000.f);
    float y[4];
    v.NoteOn(0, 60, 100);
    v.NoteOff(0, 60, 0);
    v.Process(y, 4);
    EXPECT_EQ(y[0], 0.f);
    v.NoteOn(0, 60, 100);
    v.Process(y, 4);
    EXPECT_TRUE(y[1] != 0.f && y[1] != 1.f);
}

/* FxRack<2> driven by MIDI control changes (FxRack::UpdateMidiControl) vs the oracle given the
   same reference scaling (ol::core::scale with power 1 is exact: v * (1/127) * range). */
TEST(FxRack, MidiControlledRackMatchesOracle) {
    const uint32_t n = 40, frames = 1024;
    olfx::FxRackBank rack(n, 48000.f);
    oracle_fxrack *ref = oracle_fxrack_create((int)n, 48000.f);
    const float inv127 = 1.f / 127.f;
    for (uint32_t i = 0; i < n; ++i) {
        const uint8_t t = (uint8_t)(2 + 3 * i), fb = 64, cut = (uint8_t)(40 + i);
        rack.UpdateMidiControl(i, 35, t);        // CC_DELAY_TIME
        rack.UpdateMidiControl(i, 36, fb);       // CC_DELAY_FEEDBACK
        rack.UpdateMidiControl(i, 45, cut);      // CC_FX_FILTER_CUTOFF
        oracle_fxrack_set(ref, (int)i, OFR_DELAY_TIME, (float)t * inv127 * 1.f + 0.f);
        oracle_fxrack_set(ref, (int)i, OFR_DELAY_FEEDBACK, (float)fb * inv127 * 1.f + 0.f);
        oracle_fxrack_set(ref, (int)i, OFR_FILTER_CUTOFF, (float)cut * inv127 * 20000.f + 0.f);
    }
    std::vector<float> x = noise(2, frames, n, 10);
    std::vector<float> y = run_blocks([&](const float *a, float *b, uint32_t f) { rack.Process(a, b, f); },
                                      x, 2, 2, frames, n, 256);
    std::vector<float> yr(y.size());
    oracle_fxrack_process(ref, x.data(), yr.data(), (int)frames, 8);
    EXPECT_TRUE(first_bit_mismatch(y, yr) == (size_t)-1);
    oracle_fxrack_destroy(ref);
}

/* The Daisy synth firmware's callback chain (ol_daisy/app/synth/main.cpp:78-86) on every other
   instance of one rack bank: mono voice bus in channel 0, delay, stereo copy, reverb, filter. */
TEST(FxRack, DaisyFirmwareTopologyMatchesOracle) {
    const uint32_t n = 33, frames = 700;
    olfx::FxRackBank rack(n, 48000.f);
    oracle_fxrack *ref = oracle_fxrack_create((int)n, 48000.f);
    for (uint32_t i = 0; i < n; i += 2) {
        rack.SetTopology(i, olfx::FxRackBank::Topology::DaisyFirmware);
        oracle_fxrack_set(ref, (int)i, OFR_TOPOLOGY, 1.f);
    }
    std::vector<float> x = noise(2, frames, n, 11);
    std::vector<float> y = run_blocks([&](const float *a, float *b, uint32_t f) { rack.Process(a, b, f); },
                                      x, 2, 2, frames, n, 256);
    std::vector<float> yr(y.size());
    oracle_fxrack_process(ref, x.data(), yr.data(), (int)frames, 8);
    EXPECT_TRUE(first_bit_mismatch(y, yr) == (size_t)-1);
    bool ch1 = false;
    for (uint32_t f = 0; f < frames; ++f) ch1 |= y[(size_t)frames * n + (size_t)f * n] != 0.f;
    EXPECT_TRUE(ch1);
    oracle_fxrack_destroy(ref);
}

/* Error behaviour: failures throw olfx::Error carrying the C-ABI code; nothing is silent. */
/* The per-frame -> block adapter over the GPU rack, driven one frame at a time like the
   workout_buddy AudioCallback, with a MIDI CC queued mid-block: equals the oracle run in blocks
   with the CC applied at the block boundary, delayed by one block. */
TEST(Adapter, PerFrameRackMatchesOracleDelayed) {
    const uint32_t n = 24, B = 128, F = 1000;
    olfx::FxRackBank rack(n, 48000.f, B);
    olfx::BlockAdapter<olfx::FxRackBank> ad(rack, 2, 2, B);
    oracle_fxrack *ref = oracle_fxrack_create((int)n, 48000.f);
    std::vector<float> x = noise(2, F, n, 4242), ya(2 * (size_t)F * n), yd(ya.size());
    std::vector<float> fi(2 * n), fo(2 * n);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == 300) ad.QueueMidiControl(5, 45, 3);          // delay time -> short echo
        for (uint32_t c = 0; c < 2; ++c) std::memcpy(&fi[c * n], &x[((size_t)c * F + t) * n], n * 4);
        ad.ProcessFrame(fi.data(), fo.data());
        for (uint32_t c = 0; c < 2; ++c) std::memcpy(&ya[((size_t)c * F + t) * n], &fo[c * n], n * 4);
    }
    // oracle: blocks of B, the CC mapped by the product's host map at the boundary of block 2
    uint32_t done = 0;
    yd = run_blocks([&](const float *xi, float *yo, uint32_t b) {
        if (done == 2 * B) {
            uint32_t field;
            float v;
            olfx_control_map(OLFX_KIND_FXRACK, 45, OLFX_CTL_MIDI, 3.f, &field, &v);
            oracle_fxrack_set(ref, 5, (int)field, v);
        }
        oracle_fxrack_process(ref, xi, yo, (int)b, 4);
        done += b;
    }, x, 2, 2, F, n, B);
    bool ok = true;
    for (uint32_t c = 0; c < 2 && ok; ++c)
        for (uint32_t t = 0; t < F && ok; ++t)
            for (uint32_t i = 0; i < n && ok; ++i) {
                const float a = ya[((size_t)c * F + t) * n + i];
                const float d = t < B ? 0.f : yd[((size_t)c * F + t - B) * n + i];
                ok = std::memcmp(&a, &d, 4) == 0;
            }
    EXPECT_TRUE(ok);
    oracle_fxrack_destroy(ref);
}

TEST(Boundary, ErrorsThrowWithCode) {
    int code = 0;
    try { olfx::Engine bad(99, 4, 48000.f); } catch (const olfx::Error &e) { code = e.code(); }
    EXPECT_EQ(code, OLFX_E_KIND);
    olfx::ChorusBank c(8, 48000.f);
    code = 0;
    try { c.setDepth(8, 0.5f); } catch (const olfx::Error &e) { code = e.code(); }   /* out of range */
    EXPECT_EQ(code, OLFX_E_ARG);
    std::vector<float> buf(2 * 6 * 8);
    code = 0;
    try { c.process(buf.data(), buf.data(), 6); } catch (const olfx::Error &e) { code = e.code(); }  /* not x4 */
    EXPECT_EQ(code, OLFX_E_ARG);
    /* RNBO clamps to @max: depth 5 behaves as depth 1 (the host shadow keeps the value as set) */
    olfx::ChorusBank two(2, 48000.f);
    two.setDepth(0, 5.f);
    two.setDepth(1, 1.f);
    EXPECT_EQ(two.get(0, OLFX_CH_DEPTH), 5.f);
    std::vector<float> x = noise(2, 512, 1, 9), x2(2 * 512 * 2), y2(x2.size());
    for (size_t k = 0; k < x.size(); ++k) x2[2 * k] = x2[2 * k + 1] = x[k];
    two.process(x2.data(), y2.data(), 512);
    bool same = true;
    for (size_t k = 0; k < x.size(); ++k) same &= std::memcmp(&y2[2 * k], &y2[2 * k + 1], 4) == 0;
    EXPECT_TRUE(same);
}

/* ---- per-instance, per-sample operators (include/olfx_sample.h): the reference's objects one
   for one, called one frame at a time in frame-major order; output = the oracle delayed by one
   block; calls land at the first block boundary at or after them ---- */
TEST(PerSample, ChorusEffectReadmeSurface) {
    const uint32_t n = 3, B = 256, F = 4 * B;
    olfx::ChorusEffect fx[n];
    oracle_chorus *ref = oracle_chorus_create((int)n, 48000.f, 0);
    const float depth[n] = {0.5f, 0.9f, 0.2f}, rate[n] = {0.2f, 1.0f, 0.05f};
    for (uint32_t i = 0; i < n; ++i) {            /* README.md:119-121 */
        fx[i].init(48000.f);
        fx[i].setDepth(depth[i]);
        fx[i].setRate(rate[i]);
        oracle_chorus_set(ref, (int)i, OCH_DEPTH, depth[i]);
        oracle_chorus_set(ref, (int)i, OCH_RATE, rate[i]);
    }
    EXPECT_EQ(fx[0].latency(), B);
    std::vector<float> x = noise(1, F, n, 21), y((size_t)F * n);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 7) fx[1].setMix(0.9f);       /* mid-block 1: lands at frame 2B */
        for (uint32_t i = 0; i < n; ++i) y[(size_t)t * n + i] = fx[i].process(x[(size_t)t * n + i]);
    }
    /* oracle: stereo input with L = R = x, blocks of B, the mix change before block 2 */
    std::vector<float> x2(2 * (size_t)F * n);
    std::memcpy(x2.data(), x.data(), x.size() * 4);
    std::memcpy(x2.data() + x.size(), x.data(), x.size() * 4);
    uint32_t done = 0;
    std::vector<float> yr = run_blocks([&](const float *xi, float *yo, uint32_t b) {
        if (done == 2 * B) oracle_chorus_set(ref, 1, OCH_MIX, 0.9f);
        oracle_chorus_process(ref, xi, yo, (int)b, 1);
        done += b;
    }, x2, 2, 2, F, n, B);
    bool ok = true;
    for (uint32_t t = 0; t < F && ok; ++t)
        for (uint32_t i = 0; i < n && ok; ++i) {
            const float want = t < B ? 0.f : yr[(size_t)(t - B) * n + i];   /* channel 0 (L) */
            ok = std::memcmp(&y[(size_t)t * n + i], &want, 4) == 0;
            if (!ok) std::printf("  first mismatch t=%u i=%u: %.9g vs %.9g\n", t, i, y[(size_t)t * n + i], want);
        }
    EXPECT_TRUE(ok);
    oracle_chorus_destroy(ref);
}

TEST(PerSample, SynthVoiceNoteOffAtNextBoundary) {
    const uint32_t n = 2, B = 256, F = 4 * B;
    olfx::SynthVoice v[n];
    oracle_voice *ref = oracle_voice_create_model((int)n, 48000.f, 0);
    const uint8_t notes[n] = {60, 67};
    for (uint32_t i = 0; i < n; ++i) {
        float c[OLFX_VC_NPARAMS] = {2000.f + 1000.f * i, 0.3f, 0.1f, 0.5f, 0.01f, 0.f, 0.2f, 0.5f, 0.1f,
                                    1.f, 0.005f, 0.f, 0.1f, 0.7f, 0.05f, 0.f};
        v[i].Init(48000.f);
        v[i].UpdateConfig(c);
        v[i].NoteOn(notes[i], 100);
        oracle_voice_config(ref, (int)i, c);
        oracle_voice_note(ref, (int)i, 1, notes[i]);
    }
    std::vector<float> y((size_t)F * n);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 44)                          /* mid-block 1: NoteOff lands at frame 2B */
            for (uint32_t i = 0; i < n; ++i) v[i].NoteOff(notes[i], 0);
        for (uint32_t i = 0; i < n; ++i) v[i].Process(&y[(size_t)t * n + i]);
    }
    std::vector<float> yr((size_t)F * n);
    oracle_voice_process(ref, yr.data(), (int)(2 * B), 1);
    for (uint32_t i = 0; i < n; ++i) oracle_voice_note(ref, (int)i, 0, notes[i]);
    oracle_voice_process(ref, yr.data() + (size_t)2 * B * n, (int)(2 * B), 1);
    for (uint32_t i = 0; i < n; ++i) {            /* |y - ref| <= 1e-5 max(|ref|, rms), as the bank test */
        double ss = 0, mx = 0, err = 0;
        for (uint32_t t = B; t < F; ++t) {
            const double a = yr[(size_t)(t - B) * n + i];
            ss += a * a; mx = std::max(mx, std::fabs(a));
            err = std::max(err, std::fabs((double)y[(size_t)t * n + i] - a));
        }
        const double scale = std::max(mx, std::sqrt(ss / (F - B)));
        EXPECT_TRUE(std::isfinite(err) && err <= 1e-5 * std::max(scale, 1e-30));
        for (uint32_t t = 0; t < B; ++t) EXPECT_EQ(y[(size_t)t * n + i], 0.f);
    }
    oracle_voice_destroy(ref);
}

TEST(PerSample, FxRackPerFrameBitExact) {
    const uint32_t n = 2, B = 256, F = 3 * B;
    olfx::FxRack rack[n];
    oracle_fxrack *ref = oracle_fxrack_create((int)n, 48000.f);
    const float inv127 = 1.f / 127.f;
    for (uint32_t i = 0; i < n; ++i) {
        rack[i].Init(48000.f);
        const uint8_t t = (uint8_t)(1 + 2 * i);
        rack[i].UpdateMidiControl(35, t);         /* CC_DELAY_TIME: short echoes inside the run */
        oracle_fxrack_set(ref, (int)i, OFR_DELAY_TIME, (float)t * inv127 * 1.f + 0.f);
    }
    std::vector<float> x = noise(2, F, n, 31), y(2 * (size_t)F * n);
    for (uint32_t t = 0; t < F; ++t)
        for (uint32_t i = 0; i < n; ++i) {
            const float in[2] = {x[(size_t)t * n + i], x[((size_t)F + t) * n + i]};
            float out[2];
            rack[i].Process(in, out);
            y[(size_t)t * n + i] = out[0];
            y[((size_t)F + t) * n + i] = out[1];
        }
    std::vector<float> yr(y.size());
    oracle_fxrack_process(ref, x.data(), yr.data(), (int)F, 1);
    bool ok = true;
    for (uint32_t c = 0; c < 2 && ok; ++c)
        for (uint32_t t = 0; t < F && ok; ++t)
            for (uint32_t i = 0; i < n && ok; ++i) {
                const float want = t < B ? 0.f : yr[((size_t)c * F + t - B) * n + i];
                ok = std::memcmp(&y[((size_t)c * F + t) * n + i], &want, 4) == 0;
            }
    EXPECT_TRUE(ok);
    oracle_fxrack_destroy(ref);
}

TEST(PerSample, LockstepViolationThrows) {
    olfx::ChorusEffect a, b;
    a.init(48000.f);
    b.init(48000.f);
    int code = 0;
    try {
        for (uint32_t t = 0; t <= a.latency(); ++t) a.process(0.25f);   /* b never called */
    } catch (const olfx::Error &e) { code = e.code(); }
    EXPECT_EQ(code, OLFX_E_STATE);
    olfx::ChorusEffect c;
    code = 0;
    try { c.process(0.f); } catch (const olfx::Error &e) { code = e.code(); }   /* before init() */
    EXPECT_EQ(code, OLFX_E_STATE);
}

/* ol::synth::Polyvoice over per-sample SynthVoices (Polyvoice.h:11-86): NoteOn takes the first voice
   not playing, NoteOff the first playing that note, Process adds the voices in order.  Equals the
   voice bank with the same notes and buses (olfx_mix), one block later, bit for bit. */
TEST(PerSample, PolyvoiceEqualsBankBuses) {
    const uint32_t B = 256, F = 4 * B;
    const float cfg[OLFX_VC_NPARAMS] = {3000.f, 0.4f, 0.1f, 0.5f, 0.01f, 0.f, 0.2f, 0.5f, 0.1f,
                                        1.f, 0.005f, 0.f, 0.1f, 0.7f, 0.05f, 0.f};
    olfx::SynthVoice v[6];
    std::vector<olfx::SynthVoice *> ga = {&v[0], &v[1], &v[2]}, gb = {&v[3], &v[4], &v[5]};
    olfx::Polyvoice pa(ga), pb(gb);
    pa.Init(48000.f);
    pb.Init(48000.f);
    pa.UpdateConfig(cfg);
    pb.UpdateConfig(cfg);
    pa.NoteOn(60, 100);
    pa.NoteOn(64, 100);
    pb.NoteOn(67, 100);
    EXPECT_TRUE(v[0].Playing() == 60 && v[1].Playing() == 64 && v[2].Playing() == 0 && v[3].Playing() == 67);
    std::vector<float> y(2 * (size_t)F);
    for (uint32_t t = 0; t < F; ++t) {
        if (t == B + 9) pa.NoteOff(60, 0);        /* lands at frame 2B */
        float a = 0.f, b = 0.f;                   /* the caller zeroes the frame */
        pa.Process(&a);
        pb.Process(&b);
        y[2 * (size_t)t] = a;
        y[2 * (size_t)t + 1] = b;
    }
    EXPECT_TRUE(v[0].Playing() == 0 && !v[0].Gate() && v[1].Gate());
    olfx::VoiceBank bank(6, 48000.f, B);
    for (uint32_t i = 0; i < 6; ++i) bank.UpdateConfig(i, cfg);
    bank.NoteOn(0, 60, 100);
    bank.NoteOn(1, 64, 100);
    bank.NoteOn(3, 67, 100);
    bank.SetBuses({{0, 1, 2}, {3, 4, 5}});
    std::vector<float> vo((size_t)B * 6), bo(2 * (size_t)(F - B), 0.f);
    for (uint32_t blk = 0; blk < 3; ++blk) {
        if (blk == 2) bank.NoteOff(0, 60, 0);
        bank.Process(vo.data(), B);
        bank.Mix(vo.data(), bo.data() + (size_t)blk * B * 2, B);
    }
    bool ok = true;
    for (uint32_t t = 0; t < F && ok; ++t)
        for (uint32_t g = 0; g < 2 && ok; ++g) {
            const float want = t < B ? 0.f : bo[(size_t)(t - B) * 2 + g];
            ok = std::memcmp(&y[2 * (size_t)t + g], &want, 4) == 0;
            if (!ok) std::printf("  first mismatch t=%u bus=%u: %.9g vs %.9g\n", t, g, y[2 * (size_t)t + g], want);
        }
    EXPECT_TRUE(ok);
    EXPECT_TRUE(bo[(size_t)100 * 2] != 0.f && bo[(size_t)100 * 2 + 1] != 0.f);
}

/* Per-sample call rate of the pool (include/olfx_sample.h): N ChorusEffect objects called frame-major
   from one host thread, as a reference per-frame callback calls its operators.  The per-frame call
   takes no lock; the instance completing a block runs the generation on the GPU (host I/O). */
TEST(PerSample, CallsPerSecond) {
    const uint32_t n = 4096, blocks = 8;
    std::vector<olfx::ChorusEffect> fx(n);
    for (auto &f : fx) f.init(48000.f);
    const uint32_t B = fx[0].latency();
    float acc = 0.f;
    for (uint32_t i = 0; i < n; ++i) acc += fx[i].process(0.f);           /* first run: engine creation */
    const auto t0 = std::chrono::steady_clock::now();
    uint64_t calls = 0;
    for (uint32_t t = 1; t < blocks * B; ++t)
        for (uint32_t i = 0; i < n; ++i, ++calls) acc += fx[i].process(((t * 31 + i) & 255) * (1.f / 512.f) - 0.25f);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    std::printf("  per-sample calls/s: %.4g (%u instances x %u frames, %.3f s, %u-frame blocks)\n",
                calls / s, n, blocks * B - 1, s, B);
    EXPECT_TRUE(std::isfinite(acc));
}

/* The per-frame call from several host threads: each thread owns some of a generation's objects
   and the threads meet once per frame (frame-major across the generation, as the contract asks).
   No call takes a process-wide lock; the object that completes a block runs it.  The outputs must
   equal the oracle one block late, bit for bit. */
TEST(PerSample, ThreadedFrameMajorBitExact) {
    const uint32_t n = 8, nt = 4, B = 256, F = 3 * B;
    std::vector<olfx::ChorusEffect> fx(n);
    oracle_chorus *ref = oracle_chorus_create((int)n, 48000.f, 0);
    for (uint32_t i = 0; i < n; ++i) {
        fx[i].init(48000.f);
        fx[i].setDepth(0.1f + 0.1f * i);
        oracle_chorus_set(ref, (int)i, OCH_DEPTH, 0.1f + 0.1f * i);
    }
    std::vector<float> x = noise(1, F, n, 55), y((size_t)F * n, -1.f);
    std::atomic<uint32_t> arrived{0}, generation{0};
    std::atomic<int> errors{0};
    auto meet = [&]() {                               /* a spin barrier over nt threads */
        const uint32_t g = generation.load();
        if (arrived.fetch_add(1) + 1 == nt) { arrived.store(0); generation.fetch_add(1); }
        else while (generation.load() == g) std::this_thread::yield();
    };
    std::vector<std::thread> th;
    for (uint32_t w = 0; w < nt; ++w)
        th.emplace_back([&, w]() {
            for (uint32_t t = 0; t < F; ++t) {
                for (uint32_t i = w; i < n; i += nt) {
                    try { y[(size_t)t * n + i] = fx[i].process(x[(size_t)t * n + i]); }
                    catch (const olfx::Error &) { errors.fetch_add(1); }
                }
                meet();
            }
        });
    for (auto &t : th) t.join();
    EXPECT_EQ(errors.load(), 0);
    std::vector<float> x2(2 * (size_t)F * n), yr(x2.size());
    std::memcpy(x2.data(), x.data(), x.size() * 4);
    std::memcpy(x2.data() + x.size(), x.data(), x.size() * 4);
    oracle_chorus_process(ref, x2.data(), yr.data(), (int)F, 1);
    bool ok = true;
    for (uint32_t t = 0; t < F && ok; ++t)
        for (uint32_t i = 0; i < n && ok; ++i) {
            const float want = t < B ? 0.f : yr[(size_t)(t - B) * n + i];
            ok = std::memcmp(&y[(size_t)t * n + i], &want, 4) == 0;
            if (!ok) std::printf("  first mismatch t=%u i=%u: %.9g vs %.9g\n", t, i, y[(size_t)t * n + i], want);
        }
    EXPECT_TRUE(ok);
    oracle_chorus_destroy(ref);
}

int main() { return run_all_tests(); }
