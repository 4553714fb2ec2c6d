// ol_dsp_amd/csrc/chorus.hip -- RNBO stereo chorus and gen~ pitch-shifter on gfx950.
//
// Spec (no executable oracle exists in the reference, parity "unpinned"):
//   mono-chorus.rnbopat: y = (1-mix) x + mix * lores~( delay~( pitchshift(x, pitch),
//                                                   D cycle~(rate_hz, phase) + D ), cutoff_hz, q )
//   pitchshift.gendsp / gencode at mono-chorus.rnbopat:962:
//       p0 = phasor(shift), p1 = (p0 + 0.5) % 1, W = mstosamps(window)
//       out = read(p1 W) cos((p1-.5)pi) + read(p0 W) cos((p0-.5)pi);  write(x) after the reads
//   stereo-chorus.rnbopat: L and R are two mono-chorus instances with shared params; L phase 1 and
//   R phase 0 are the same phase after wrap, so both channels see the same LFO.
//
// Mapping: one lane = one (instance, channel); a 256-thread workgroup = 2 x 64 instances x 2
// channels, channel-major per wave so audio I/O ([ch][frame][inst]) is 256-B coalesced.
// Rings are lane-private and contiguous ([inst][ch][size]) because every tap is modulated per
// instance.  The block is processed in chunks of 16 frames: per chunk each lane computes its 16
// tap delays up front, then stages the <= 24-float window each of its 3 taps touches into LDS with
// 6 x 16-B loads (the window moves ~1 position per frame, so consecutive chunks stream through the
// ring), and the serial recurrence reads the taps from LDS.  LDS is laid out [slot][thread] so the
// per-lane fractional reads are bank-conflict free.  Windows that cannot cover a chunk (the
// pitch-shifter phasor wrap, once per 1/shift s) fall back to direct ring reads for that lane.
#include "olfx_internal.h"

namespace olfx {

namespace {

constexpr int kChunk = 16;      // frames per chunk
constexpr int kWin = 24;        // floats staged per tap window (6 x float4)
constexpr int kThreads = 256;

__device__ __forceinline__ float unit24(uint32_t acc) {
    return (float)(acc >> 8) * 5.9604644775390625e-8f;   // exact: 24-bit fraction in [0,1)
}

// floor of a clamped fractional delay: di, fr with d in [dmin, dmax]
__device__ __forceinline__ void split_delay(float d, float dmin, float dmax, int &di, float &fr) {
    d = fminf(fmaxf(d, dmin), dmax);
    const uint32_t u = (uint32_t)d;
    di = (int)u;
    fr = d - (float)u;
}

__device__ __forceinline__ float lerp_pair(float x0, float x1, float fr) { return x0 + fr * (x1 - x0); }

}  // namespace

__global__ __launch_bounds__(kThreads, 2) void chorus_block_v2(ChorusArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];   // [3 taps][kWin][kThreads]
    const uint32_t tid = threadIdx.x;
    const uint32_t g = blockIdx.x * kThreads + tid;
    const uint32_t wave = g >> 6, lane = g & 63u;
    const uint32_t ch = wave & 1u;
    const uint32_t i = (wave >> 1) * 64u + lane;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const bool full = a.mode == 0;

    const uint32_t lfo_inc = a.coef[CHC_LFO_INC * n + i];
    const uint32_t lfo_off = a.coef[CHC_LFO_OFF * n + i];
    const uint32_t ps_inc = a.coef[CHC_PS_INC * n + i];
    const float D = __uint_as_float(a.coef[CHC_DEPTH * n + i]);
    const float W = __uint_as_float(a.coef[CHC_WINDOW * n + i]);
    const float b0 = __uint_as_float(a.coef[CHC_B0 * n + i]);
    const float b1 = __uint_as_float(a.coef[CHC_B1 * n + i]);
    const float b2 = __uint_as_float(a.coef[CHC_B2 * n + i]);
    const float a1 = __uint_as_float(a.coef[CHC_A1 * n + i]);
    const float a2 = __uint_as_float(a.coef[CHC_A2 * n + i]);
    const float mix = __uint_as_float(a.coef[CHC_MIX * n + i]);
    const float dry = __uint_as_float(a.coef[CHC_DRY * n + i]);

    uint32_t lfo_acc = a.state[CHS_LFO_ACC * n + i];
    uint32_t ps_acc = a.state[CHS_PS_ACC * n + i];
    float z1 = __uint_as_float(a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i]);
    float z2 = __uint_as_float(a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i]);

    const uint32_t pmask = a.psize - 1u, cmask = a.csize - 1u;
    const float pmax = (float)(a.psize - 2u), cmax = (float)(a.csize - 2u);
    float *pring = a.pitch_ring + ((size_t)i * 2 + ch) * a.psize;
    float *cring = a.chorus_ring + ((size_t)i * 2 + ch) * a.csize;
    const float *in = a.in + (size_t)ch * a.n_frames * n + i;
    float *out = a.out + (size_t)ch * a.n_frames * n + i;
    float *wP0 = lds + 0 * kWin * kThreads + tid;
    float *wP1 = lds + 1 * kWin * kThreads + tid;
    float *wC = lds + 2 * kWin * kThreads + tid;

    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += kChunk) {
        const uint32_t w0 = a.t0 + f0;
        const int C = (int)min((uint32_t)kChunk, a.n_frames - f0);   // multiple of 4

        // ---- inputs of the chunk, written to the pitch ring first (taps read delay >= 1) ----
        float x[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) x[k] = k < C ? in[(size_t)(f0 + k) * n] : 0.f;
#pragma unroll
        for (int k = 0; k < kChunk; k += 4)
            if (k < C) *(float4 *)(pring + ((w0 + k) & pmask)) = make_float4(x[k], x[k + 1], x[k + 2], x[k + 3]);

        // ---- per-frame control signals of the chunk (LFO, phasor, window gains) ----
        float dC[kChunk], dA[kChunk], dB[kChunk], gA[kChunk], gB[kChunk];
        int loA = 1 << 30, hiA = -(1 << 30), loB = 1 << 30, hiB = -(1 << 30), loC = 1 << 30, hiC = -(1 << 30);
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            const float lfo = cos2pi(unit24(lfo_acc + lfo_off));
            dC[k] = lfo * D + D;
            const float p0 = unit24(ps_acc);
            const float p1 = unit24(ps_acc + 0x80000000u);
            gA[k] = cos2pi((p0 - 0.5f) * 0.5f);
            gB[k] = cos2pi((p1 - 0.5f) * 0.5f);
            dA[k] = p0 * W;
            dB[k] = p1 * W;
            if (k < C) {
                lfo_acc += lfo_inc;
                ps_acc += ps_inc;
                int di; float fr;
                split_delay(dA[k], 1.0f, pmax, di, fr);
                loA = min(loA, k - di - 1); hiA = max(hiA, k - di);
                split_delay(dB[k], 1.0f, pmax, di, fr);
                loB = min(loB, k - di - 1); hiB = max(hiB, k - di);
                split_delay(dC[k], 0.0f, cmax, di, fr);
                loC = min(loC, k - di - 1); hiC = max(hiC, k - di);
            }
        }
        const int sA = loA & ~3, sB = loB & ~3, sC = loC & ~3;   // window starts rel. to w0
        const bool okA = hiA - sA < kWin, okB = hiB - sB < kWin, okC = hiC - sC < kWin;

        // ---- stage the tap windows into LDS (6 x 16 B each) ----
        if (okA) {
#pragma unroll
            for (int m = 0; m < kWin; m += 4) {
                const float4 v = *(const float4 *)(pring + ((w0 + sA + m) & pmask));
                wP0[(m + 0) * kThreads] = v.x; wP0[(m + 1) * kThreads] = v.y;
                wP0[(m + 2) * kThreads] = v.z; wP0[(m + 3) * kThreads] = v.w;
            }
        }
        if (okB) {
#pragma unroll
            for (int m = 0; m < kWin; m += 4) {
                const float4 v = *(const float4 *)(pring + ((w0 + sB + m) & pmask));
                wP1[(m + 0) * kThreads] = v.x; wP1[(m + 1) * kThreads] = v.y;
                wP1[(m + 2) * kThreads] = v.z; wP1[(m + 3) * kThreads] = v.w;
            }
        }
        if (full && okC) {
#pragma unroll
            for (int m = 0; m < kWin; m += 4) {
                const float4 v = *(const float4 *)(cring + ((w0 + sC + m) & cmask));
                wC[(m + 0) * kThreads] = v.x; wC[(m + 1) * kThreads] = v.y;
                wC[(m + 2) * kThreads] = v.z; wC[(m + 3) * kThreads] = v.w;
            }
        }

        // ---- the serial recurrence over the chunk ----
        float ps[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
            if (k < C) {
                int di; float fr;
                float tA, tB;
                split_delay(dA[k], 1.0f, pmax, di, fr);
                if (okA) {
                    const int j = k - di - sA;
                    tA = lerp_pair(wP0[j * kThreads], wP0[(j - 1) * kThreads], fr);
                } else {
                    const uint32_t q = w0 + k - di;
                    tA = lerp_pair(pring[q & pmask], pring[(q - 1u) & pmask], fr);
                }
                split_delay(dB[k], 1.0f, pmax, di, fr);
                if (okB) {
                    const int j = k - di - sB;
                    tB = lerp_pair(wP1[j * kThreads], wP1[(j - 1) * kThreads], fr);
                } else {
                    const uint32_t q = w0 + k - di;
                    tB = lerp_pair(pring[q & pmask], pring[(q - 1u) & pmask], fr);
                }
                const float p = tB * gB[k] + tA * gA[k];
                ps[k] = p;
                float y = p;
                if (full) {
                    // delay~ writes before it reads: this frame's sample is visible at delay 0
                    split_delay(dC[k], 0.0f, cmax, di, fr);
                    float wet;
                    if (okC) {
                        if (k - sC < kWin) wC[(k - sC) * kThreads] = p;
                        const int j = k - di - sC;
                        wet = lerp_pair(wC[j * kThreads], wC[(j - 1) * kThreads], fr);
                    } else {   // unreachable for |LFO slope| <= 0.04 frame/frame; kept exact
                        cring[(w0 + k) & cmask] = p;
                        const uint32_t q = w0 + k - di;
                        wet = lerp_pair(cring[q & cmask], cring[(q - 1u) & cmask], fr);
                    }
                    const float lp = b0 * wet + z1;
                    z1 = (b1 * wet - a1 * lp) + z2;
                    z2 = b2 * wet - a2 * lp;
                    y = x[k] * dry + lp * mix;
                }
                out[(size_t)(f0 + k) * n] = y;
            } else {
                ps[k] = 0.f;
            }
        }
        if (full) {
#pragma unroll
            for (int k = 0; k < kChunk; k += 4)
                if (k < C) *(float4 *)(cring + ((w0 + k) & cmask)) = make_float4(ps[k], ps[k + 1], ps[k + 2], ps[k + 3]);
        }
    }

    if (ch == 0) {
        a.state[CHS_LFO_ACC * n + i] = lfo_acc;
        a.state[CHS_PS_ACC * n + i] = ps_acc;
    }
    a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i] = __float_as_uint(z1);
    a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i] = __float_as_uint(z2);
}

hipError_t launch_chorus(const ChorusArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t groups = (a.n + 63) / 64;            // 64-instance groups, 2 waves each
    const uint32_t blocks = (groups * 2 * 64 + kThreads - 1) / kThreads;
    const size_t lds = (size_t)3 * kWin * kThreads * sizeof(float);
    hipLaunchKernelGGL(chorus_block_v2, dim3(blocks), dim3(kThreads), lds, s, a);
    return hipGetLastError();
}

}  // namespace olfx
