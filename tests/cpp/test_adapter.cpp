/*
 * tests/cpp/test_adapter.cpp -- host logic of include/olfx_adapter.hpp (per-frame -> block
 * adapter), on the CPU.
 *
 * The adapter is generic over the bank, so here it drives CPU oracle banks (oracle/liboracle.so,
 * TEST INFRASTRUCTURE) through the same process()/size()/UpdateMidiControl() interface the GPU
 * banks expose; control values are mapped by the product's host-side olfx_control_map (no GPU
 * call). tests/cpp/test_operators.cpp runs the adapter over the real GPU banks.
 *
 * Checked: the adapter's output stream is the bank's block output delayed by exactly `block`
 * frames, bit for bit, whatever the caller's frame counts (one frame at a time, ragged JUCE-style
 * buffers, Daisy-style interleaved); queued MIDI CCs and note events land at the block boundary
 * after they were queued, in queue order; Queue() is safe from a second thread.
 */
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <thread>
#include <vector>

#include "olfx_adapter.hpp"
#include "../../oracle/oracle.h"

namespace {
int g_failures = 0, g_tests = 0;
#define EXPECT_TRUE(c) do { if (!(c)) { ++g_failures; std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); } } while (0)

/* FxRack<2> oracle behind the bank interface; CCs mapped exactly as the engine maps them. */
struct OracleRack {
    oracle_fxrack *h;
    uint32_t n;
    explicit OracleRack(uint32_t n_) : h(oracle_fxrack_create((int)n_, 48000.f)), n(n_) {}
    ~OracleRack() { oracle_fxrack_destroy(h); }
    uint32_t size() const { return n; }
    void process(const float *in, float *out, uint32_t frames, int, void *) {
        oracle_fxrack_process(h, in, out, (int)frames, 1);
    }
    void UpdateMidiControl(uint32_t i, uint8_t cc, uint8_t v) {
        uint32_t field;
        float pv;
        if (olfx_control_map(OLFX_KIND_FXRACK, cc, OLFX_CTL_MIDI, (float)v, &field, &pv) == OLFX_OK &&
            field != OLFX_FIELD_UPDATE_ONLY)
            oracle_fxrack_set(h, (int)i, (int)field, pv);
    }
};

struct OracleVoices {
    oracle_voice *h;
    uint32_t n;
    explicit OracleVoices(uint32_t n_) : h(oracle_voice_create((int)n_, 48000.f)), n(n_) {}
    ~OracleVoices() { oracle_voice_destroy(h); }
    uint32_t size() const { return n; }
    void process(const float *, float *out, uint32_t frames, int, void *) {
        oracle_voice_process(h, out, (int)frames, 1);
    }
    void NoteOn(uint32_t i, uint8_t note) { oracle_voice_note(h, (int)i, 1, note); }
    void NoteOff(uint32_t i, uint8_t note) { oracle_voice_note(h, (int)i, 0, note); }
};

std::vector<float> noise(uint32_t ch, uint32_t frames, uint32_t n, uint32_t seed) {
    std::vector<float> x((size_t)ch * frames * n);
    for (uint32_t c = 0; c < ch; ++c)
        for (uint32_t i = 0; i < n; ++i)
            oracle_xorshift_noise(seed + 7919u * i + 104729u * c, x.data() + (size_t)c * frames * n + i, frames, n);
    return x;
}

/* y_adapter[c][t][i] == y_direct[c][t - block][i] (0 for t < block), bit for bit */
bool delayed_equal(const std::vector<float> &ya, const std::vector<float> &yd, uint32_t ch, uint32_t frames,
                   uint32_t n, uint32_t block) {
    for (uint32_t c = 0; c < ch; ++c)
        for (uint32_t t = 0; t < frames; ++t)
            for (uint32_t i = 0; i < n; ++i) {
                const float a = ya[((size_t)c * frames + t) * n + i];
                const float d = t < block ? 0.f : yd[((size_t)c * frames + t - block) * n + i];
                if (std::memcmp(&a, &d, 4) != 0) return false;
            }
    return true;
}

void run(const char *name, const std::function<void()> &fn) {
    const int before = g_failures;
    ++g_tests;
    fn();
    std::printf("[%s] %s\n", g_failures == before ? "  OK  " : "FAILED", name);
}
}  // namespace

int main() {
    const uint32_t n = 5, B = 64, F = 1000;   // F is not a multiple of B

    run("Adapter.PerFrameIsBlockDelayed", [&] {
        std::vector<float> x = noise(2, F, n, 11), yd(2 * (size_t)F * n), ya(yd.size());
        OracleRack direct(n), viaa(n);
        direct.process(x.data(), yd.data(), F, OLFX_IO_HOST, nullptr);
        olfx::BlockAdapter<OracleRack> ad(viaa, 2, 2, B);
        std::vector<float> fi(2 * n), fo(2 * n);
        for (uint32_t t = 0; t < F; ++t) {
            for (uint32_t c = 0; c < 2; ++c) std::memcpy(&fi[c * n], &x[((size_t)c * F + t) * n], n * 4);
            ad.ProcessFrame(fi.data(), fo.data());
            for (uint32_t c = 0; c < 2; ++c) std::memcpy(&ya[((size_t)c * F + t) * n], &fo[c * n], n * 4);
        }
        EXPECT_TRUE(ad.latency() == B && ad.frames() == F);
        EXPECT_TRUE(delayed_equal(ya, yd, 2, F, n, B));
    });

    run("Adapter.RaggedBuffersAndInterleaved", [&] {
        std::vector<float> x = noise(2, F, n, 12), yd(2 * (size_t)F * n);
        OracleRack direct(n), r1(n), r2(n);
        direct.process(x.data(), yd.data(), F, OLFX_IO_HOST, nullptr);
        olfx::BlockAdapter<OracleRack> a1(r1, 2, 2, B), a2(r2, 2, 2, B);
        const uint32_t sizes[] = {1, 7, 100, 3, 64, 129, 0, 500};
        std::vector<float> y1(2 * (size_t)F * n), y2(y1.size());
        uint32_t t0 = 0;
        for (uint32_t k = 0; t0 < F; ++k) {
            const uint32_t m = std::min(sizes[k % 8], F - t0);
            std::vector<float> xb(2 * (size_t)m * n), yb(xb.size()), xi(xb.size()), yi(xb.size());
            for (uint32_t c = 0; c < 2 && m; ++c)    // (a zero-frame callback copies nothing)
                std::memcpy(xb.data() + (size_t)c * m * n, x.data() + ((size_t)c * F + t0) * n, (size_t)m * n * 4);
            for (uint32_t f = 0; f < m; ++f)          // [f][i][c]
                for (uint32_t i = 0; i < n; ++i)
                    for (uint32_t c = 0; c < 2; ++c) xi[((size_t)f * n + i) * 2 + c] = xb[((size_t)c * m + f) * n + i];
            a1.ProcessFrames(xb.data(), yb.data(), m);
            a2.ProcessInterleaved(xi.data(), yi.data(), m);
            for (uint32_t c = 0; c < 2; ++c)
                for (uint32_t f = 0; f < m; ++f)
                    for (uint32_t i = 0; i < n; ++i) {
                        y1[((size_t)c * F + t0 + f) * n + i] = yb[((size_t)c * m + f) * n + i];
                        y2[((size_t)c * F + t0 + f) * n + i] = yi[((size_t)f * n + i) * 2 + c];
                    }
            t0 += m;
        }
        EXPECT_TRUE(delayed_equal(y1, yd, 2, F, n, B));
        EXPECT_TRUE(delayed_equal(y2, yd, 2, F, n, B));
    });

    run("Adapter.QueuedControlsLandAtTheNextBoundary", [&] {
        // CCs queued while frames 130..139 are collected (block 2 = frames 128..191) apply before
        // block 2 is processed: the direct run applies them after 128 frames.
        std::vector<float> x = noise(2, F, n, 13), yd(2 * (size_t)F * n), ya(yd.size());
        OracleRack viaa(n);
        {   // direct: 128 frames, the three CCs in queue order, then the rest of the run
            const uint32_t rest = F - 2 * B;
            std::vector<float> xr(2 * (size_t)rest * n), yr(xr.size());
            for (uint32_t c = 0; c < 2; ++c)
                std::memcpy(&xr[(size_t)c * rest * n], &x[((size_t)c * F + 2 * B) * n], (size_t)rest * n * 4);
            std::vector<float> xh(2 * (size_t)2 * B * n), yh(xh.size());
            OracleRack d2(n);
            for (uint32_t c = 0; c < 2; ++c)
                std::memcpy(&xh[(size_t)c * 2 * B * n], &x[(size_t)c * F * n], (size_t)2 * B * n * 4);
            d2.process(xh.data(), yh.data(), 2 * B, OLFX_IO_HOST, nullptr);
            d2.UpdateMidiControl(1, 45, 20);
            d2.UpdateMidiControl(1, 45, 90);
            d2.UpdateMidiControl(3, 7, 100);
            d2.process(xr.data(), yr.data(), rest, OLFX_IO_HOST, nullptr);
            for (uint32_t c = 0; c < 2; ++c) {
                std::memcpy(&yd[(size_t)c * F * n], &yh[(size_t)c * 2 * B * n], (size_t)2 * B * n * 4);
                std::memcpy(&yd[((size_t)c * F + 2 * B) * n], &yr[(size_t)c * rest * n], (size_t)rest * n * 4);
            }
        }
        olfx::BlockAdapter<OracleRack> ad(viaa, 2, 2, B);
        std::vector<float> fi(2 * n), fo(2 * n);
        for (uint32_t t = 0; t < F; ++t) {
            if (t == 130) { ad.QueueMidiControl(1, 45, 20); ad.QueueMidiControl(1, 45, 90); }
            if (t == 139) ad.QueueMidiControl(3, 7, 100);
            for (uint32_t c = 0; c < 2; ++c) std::memcpy(&fi[c * n], &x[((size_t)c * F + t) * n], n * 4);
            ad.ProcessFrame(fi.data(), fo.data());
            for (uint32_t c = 0; c < 2; ++c) std::memcpy(&ya[((size_t)c * F + t) * n], &fo[c * n], n * 4);
        }
        EXPECT_TRUE(delayed_equal(ya, yd, 2, F, n, B));
    });

    run("Adapter.VoiceNotesAndCrossThreadQueue", [&] {
        // voices (no input channels): NoteOn queued from a second thread before block 0 is
        // collected; NoteOff queued at frame 300, while block 4 (frames 256..319) is collected ->
        // it applies from bank frame 256
        OracleVoices direct(n), viaa(n);
        for (uint32_t i = 0; i < n; ++i) direct.NoteOn(i, (uint8_t)(40 + 9 * i));
        std::vector<float> yd((size_t)F * n), ya(yd.size());
        direct.process(nullptr, yd.data(), 4 * B, OLFX_IO_HOST, nullptr);
        for (uint32_t i = 0; i < n; ++i) direct.NoteOff(i, 0);
        direct.process(nullptr, yd.data() + (size_t)4 * B * n, F - 4 * B, OLFX_IO_HOST, nullptr);
        olfx::BlockAdapter<OracleVoices> ad(viaa, 0, 1, B);
        std::atomic<int> queued{0};
        std::thread midi([&] {
            for (uint32_t i = 0; i < n; ++i) {
                ad.Queue([i](OracleVoices &v) { v.NoteOn(i, (uint8_t)(40 + 9 * i)); });
                ++queued;
            }
        });
        midi.join();
        EXPECT_TRUE(queued.load() == (int)n);
        std::vector<float> fo(n);
        // the first block is silence from the adapter; the queued NoteOns apply before block 0
        for (uint32_t t = 0; t < F; ++t) {
            if (t == 300)
                for (uint32_t i = 0; i < n; ++i) ad.Queue([i](OracleVoices &v) { v.NoteOff(i, 0); });
            ad.ProcessFrame(nullptr, fo.data());
            std::memcpy(&ya[(size_t)t * n], fo.data(), n * 4);
        }
        EXPECT_TRUE(delayed_equal(ya, yd, 1, F, n, B));
        float mx = 0;
        for (uint32_t t = B; t < F; ++t) mx = std::fmax(mx, std::fabs(ya[(size_t)t * n]));
        EXPECT_TRUE(mx > 0.f);
    });

    std::printf("%d tests, %d failures\n", g_tests, g_failures);
    return g_failures ? 1 : 0;
}
