/*
 * include/olfx_adapter.hpp -- per-frame -> block adapter for reference host callbacks
 * (header-only).
 *
 * The reference hosts drive their operators one frame at a time:
 *   - workout_buddy's AudioCallback(buddy, in1, in2, out1, out2) per frame
 *     (workouts/workout_buddy.h:84-85, called per frame at workout_buddy.cpp:82-90);
 *   - the Daisy firmware's interleaved callback, a per-frame loop over voice -> delay -> reverb
 *     -> filter (modules/ol_daisy/app/synth/main.cpp:74-90);
 *   - the JUCE host's processBlock over a host-sized buffer (modules/juce/host/host.cpp:682), with
 *     parameter changes drained from a mutex-guarded queue at the start of each callback
 *     (host.cpp:646-653).
 * An olfx engine wants whole blocks for every instance. BlockAdapter buffers one block of input
 * frames for all N instances, runs the bank once per block, and hands back the output with a
 * latency of exactly `block` frames: the adapter's output frame t is the bank's output frame
 * t - block (zeros before the first block completes). Any caller frame count works (ragged
 * JUCE buffers, one frame at a time, interleaved). Queued control changes and note events are
 * applied at the next block boundary, in queue order, the host.cpp:646-653 pattern; Queue() may
 * be called from another thread (a MIDI thread).
 *
 * Bank is any type with
 *     void process(const float *in, float *out, uint32_t n_frames, int io, void *stream);
 *     uint32_t size() const;
 * -- olfx::Engine and every bank of olfx_fx.hpp. The adapter uses host I/O (OLFX_IO_HOST). The
 * engine stages through pinned memory and synchronises, so process() returns with the outputs in
 * place. Bank errors propagate (olfx::Error); there is no fallback.
 */
#ifndef OLFX_ADAPTER_HPP
#define OLFX_ADAPTER_HPP

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <utility>
#include <vector>

#include "olfx.h"

namespace olfx {

template <class Bank>
class BlockAdapter {
public:
    /* in_ch / out_ch: the bank kind's channel counts (olfx_kind_info_get); block: frames per bank
       call, i.e. the added latency. */
    BlockAdapter(Bank &bank, uint32_t in_ch, uint32_t out_ch, uint32_t block)
        : bank_(bank), n_(bank.size()), ich_(in_ch), och_(out_ch), block_(block),
          in_((size_t)in_ch * block * bank.size(), 0.f), out_((size_t)out_ch * block * bank.size(), 0.f) {
        if (block == 0 || (block & 3u) || out_ch == 0)   // olfx_process takes multiples of 4 frames
            throw std::invalid_argument("BlockAdapter: block must be a positive multiple of 4, out_ch > 0");
    }

    uint32_t latency() const { return block_; }
    uint32_t size() const { return n_; }
    uint64_t frames() const { return frames_; }

    /* Thread-safe: f(bank) runs at the next block boundary, before the block is processed. */
    void Queue(std::function<void(Bank &)> f) {
        std::lock_guard<std::mutex> lk(mu_);
        queue_.push_back(std::move(f));
    }
    void QueueMidiControl(uint32_t i, uint8_t control, uint8_t value) {
        Queue([=](Bank &b) { b.UpdateMidiControl(i, control, value); });
    }
    void QueueHardwareControl(uint32_t i, uint8_t control, float value) {
        Queue([=](Bank &b) { b.UpdateHardwareControl(i, control, value); });
    }

    /* One frame for every instance: in [in_ch][n] (may be null when in_ch == 0), out [out_ch][n].
       The workout_buddy / Daisy per-frame shape, for N instances at once. */
    void ProcessFrame(const float *in, float *out) { ProcessFrames(in, out, 1); }

    /* `frames` frames: in [in_ch][frames][n], out [out_ch][frames][n] (JUCE processBlock shape). */
    void ProcessFrames(const float *in, float *out, uint32_t frames) {
        uint32_t done = 0;
        while (done < frames) {
            const uint32_t k = std::min(frames - done, block_ - pos_);
            for (uint32_t c = 0; c < ich_; ++c)
                std::memcpy(&in_[((size_t)c * block_ + pos_) * n_], &in[((size_t)c * frames + done) * n_],
                            (size_t)k * n_ * sizeof(float));
            for (uint32_t c = 0; c < och_; ++c)
                std::memcpy(&out[((size_t)c * frames + done) * n_], &out_[((size_t)c * block_ + pos_) * n_],
                            (size_t)k * n_ * sizeof(float));
            advance(k);
            done += k;
        }
    }

    /* Interleaved frames (the Daisy AudioHandle layout, extended to N instances):
       in[(f * n + i) * in_ch + c], out[(f * n + i) * out_ch + c]. */
    void ProcessInterleaved(const float *in, float *out, uint32_t frames) {
        for (uint32_t f = 0; f < frames; ++f) {
            for (uint32_t c = 0; c < ich_; ++c) {
                float *dst = &in_[((size_t)c * block_ + pos_) * n_];
                for (uint32_t i = 0; i < n_; ++i) dst[i] = in[((size_t)f * n_ + i) * ich_ + c];
            }
            for (uint32_t c = 0; c < och_; ++c) {
                const float *src = &out_[((size_t)c * block_ + pos_) * n_];
                for (uint32_t i = 0; i < n_; ++i) out[((size_t)f * n_ + i) * och_ + c] = src[i];
            }
            advance(1);
        }
    }

private:
    void advance(uint32_t k) {
        pos_ += k;
        frames_ += k;
        if (pos_ < block_) return;
        std::vector<std::function<void(Bank &)>> q;
        {
            std::lock_guard<std::mutex> lk(mu_);
            q.swap(queue_);
        }
        for (auto &f : q) f(bank_);
        // the previous block's outputs have all been read out: overwrite them in place
        bank_.process(ich_ ? in_.data() : nullptr, out_.data(), block_, OLFX_IO_HOST, nullptr);
        pos_ = 0;
    }

    Bank &bank_;
    const uint32_t n_, ich_, och_, block_;
    uint32_t pos_ = 0;
    uint64_t frames_ = 0;
    std::vector<float> in_, out_;
    std::mutex mu_;
    std::vector<std::function<void(Bank &)>> queue_;
};

}  // namespace olfx

#endif
