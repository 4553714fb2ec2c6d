// ol_dsp_amd/csrc/chorus_block.h -- chorus_block_v13: the stereo chorus / pitch-shifter a whole
// block at a time, frame-parallel where the spec is feed-forward.
//
// Spec (mono-chorus.rnbopat:962 gencode, :1793 delay~, :1808 lores~): per
// frame, the pitch-shifter's two taps, its crossfade gains and the chorus tap are pure functions of
// the frame index (the 64-bit phasors are closed-form: acc(t0 + k) = acc(t0) + k inc, exact) and of
// ring positions older than the frame.  Only lores~ (a TDF-II biquad) carries a recurrence.  So
// where v11 walks every (instance, channel) lane through 16-frame chunks -- a chain of dependent
// LDS and memory round trips per chunk at the two waves per SIMD the workload allows -- v13 works
// on whole blocks of G = 16 stereo instances:
//
//   fill     the instances' whole pitch rings (512 positions: exactly the taps' compulsory reads),
//            the chorus window the block's taps reach (<= 288 positions, bounded from the LFO at
//            the block's two ends), and the block's input rows land in LDS
//   phase 1  pitch-shifter, lanes = frames: psv -> the chorus window (LDS) and the chorus ring
//            (HBM, a 512-B run per wave); the input -> the pitch ring (HBM)
//   phase 2  chorus tap, lanes = frames: w -> LDS
//   phase 3  lores~ + mix, lanes = (instance, channel), 256 serial steps per lane
//   out      output rows from LDS
//
// One persistent workgroup per CU (8 waves, 137.5 KB of LDS) loops over its groups; the NEXT
// group's rings, window and input rows are loaded into registers while this group computes, and
// written to LDS once it is done (68 VGPRs of prefetch per lane: ~135 KB in flight per CU).  Every
// access is a whole-line or 512-B run except the 64-B input / output row pieces of a 16-instance
// group; groups 2k and 2k+1 (one 128-B line) run at the same time on the same XCD, so the line's
// second half is an L2 hit.
//
// Frame arithmetic is the spec's, operation for operation (bit-identical to the oracle
// oracle/chorus_ref.c chorus_frame and to v11): the precise tap delays of spec v2 (pitch_split,
// chorus_split: olfx_internal.h), x0 + fr (x1 - x0), psv = tB gB + tA gA, wet, the biquad,
// x dry + lp mix.
// Geometry: psize 512 and csize 2048 (sample rates ~25.6 .. 51 kHz); others use v11.
#pragma once
#include "chorus_stage_l.h"

// diagnostic builds (wrong results; tools/build_variant.sh): bit 0 skips lores~, bit 1 the chorus tap
#ifndef OLFX_CB_DIAG
#define OLFX_CB_DIAG 0
#endif

namespace olfx {
namespace cb {

constexpr int kG = 16;                         // stereo instances per group (one round of a workgroup)
constexpr int kS = 256;                        // frames per launch at most (the engine splits longer calls)
constexpr int kThreads = 512;                  // 8 waves: two per SIMD
constexpr int kWaves = kThreads / 64;
constexpr uint32_t kPsize = 512, kCsize = 2048;
constexpr int kPOld = (int)kPsize;             // pitch window: positions [t0 - 512, t0 + S)
constexpr int kPStride = 2 * (kPOld + kS) + 4; // floats per instance (+4: instance i starts at bank 4i)
constexpr int kCWin = 290;                     // chorus window positions (<= 268 used, the last is junk)
constexpr int kCStride = 2 * kCWin;
constexpr int kCParts = 144;                   // float4 (2 positions) loads per chorus window, at most
constexpr int kScW = 32;                       // scalar words per instance
// scalar words: coefficient and state fields as on the device ([CHC_N] then [CHS_N]), then the
// window geometry of the round
constexpr int kScState = CHC_N;                // 17..24: CHS_* words
constexpr int kScCoff = kScState + CHS_N;      // t0 - (first chorus window position)
constexpr int kScCw = kScCoff + 1;             // chorus window width (positions)
constexpr int kLdsFloats = kG * kPStride + kG * kCStride + 2 * kG * kScW;
static_assert(kScCw < kScW, "scalar slots");
static_assert(kLdsFloats * 4 <= 160 * 1024, "LDS budget");

// prefetch registers of one lane
constexpr int kPParts = kG * (int)kPsize / 2 / kThreads;       // 8: float4 pieces of the pitch rings
constexpr int kXParts = kG * 2 * kS / 4 / kThreads;           // 4: float4 pieces of the input rows
constexpr int kCLoads = (kG * kCParts + kThreads - 1) / kThreads;   // 5
constexpr int kScLoads = kG * (CHC_N + CHS_N);                // 400 lanes load one scalar word each
static_assert(kScLoads <= kThreads, "scalar loads");
static_assert(kScCw < kScW, "window geometry slots");

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void st2(ch::Rsrc r, uint32_t off, float2 v) {
    u32x2 w;
    w.x = __float_as_uint(v.x);
    w.y = __float_as_uint(v.y);
    __builtin_amdgcn_raw_buffer_store_b64(w, r, off, 0, ch::kStreamAux);
}

using ch::Rsrc;
using ch::rsrc;
using ch::ld4;
using ch::st4;

struct Pre {
    float4 p[kPParts];
    float4 x[kXParts];
    float4 c[kCLoads];
};

template <bool FULL>
struct Block {
    const ChorusArgs &a;
    float *P, *C, *Sc;            // LDS regions
    uint32_t tid, wave, lane;
    uint32_t n, S, t0;
    Rsrc rP, rC, rIn, rOut;

    __device__ __forceinline__ Block(const ChorusArgs &a_, float *lds) : a(a_) {
        P = lds;
        C = P + kG * kPStride;
        Sc = C + kG * kCStride;
        tid = threadIdx.x;
        wave = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
        lane = tid & 63u;
        n = a.n;
        S = a.n_frames;
        t0 = a.t0;
        rP = rsrc(a.pitch_ring, (uint64_t)n * 2 * kPsize * 4);
        rC = rsrc(a.chorus_ring, (uint64_t)n * 2 * kCsize * 4);
        rIn = rsrc(a.in, (a.plane + (uint64_t)S * n) * 4);
        rOut = rsrc(a.out, (a.plane + (uint64_t)S * n) * 4);
    }

    __device__ __forceinline__ float *sc(int buf, uint32_t j) { return Sc + (buf * kG + j) * kScW; }
    __device__ __forceinline__ static uint64_t w64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }
    __device__ __forceinline__ static uint32_t u(float v) { return __float_as_uint(v); }

    // ---- scalars of group g: lane tid < 400 loads word (tid % 25) of instance (tid / 25) ----
    __device__ __forceinline__ uint32_t load_scalar(uint32_t g) const {
        if (tid >= (uint32_t)kScLoads) return 0u;
        const uint32_t j = tid / (uint32_t)(CHC_N + CHS_N), w = tid % (uint32_t)(CHC_N + CHS_N);
        const uint32_t i = min(g * kG + j, n - 1u);
        return w < (uint32_t)CHC_N ? a.coef[w * n + i] : a.state[(w - CHC_N) * n + i];
    }
    __device__ __forceinline__ void store_scalar(int buf, uint32_t v) {
        if (tid >= (uint32_t)kScLoads) return;
        const uint32_t j = tid / (uint32_t)(CHC_N + CHS_N), w = tid % (uint32_t)(CHC_N + CHS_N);
        sc(buf, j)[w] = __uint_as_float(v);
    }

    // ---- the chorus window of instance j (scalars in buf): first position t0 - coff, width cw ----
    // The LFO at the block's first and last frame, computed exactly as the frames compute theirs; in
    // between the delay stays within [min, max] of them up to the LFO's curvature over the block
    // (D (1 - cos(pi f S / sr)) < 0.04 samples for every legal depth and rate at sr >= 25.6 kHz),
    // so floor(min - .25) .. floor(max + .25) bounds every frame's floor delay; width <= S + 12.
    __device__ __forceinline__ static double f64(float hi, float lo) { return __longlong_as_double((long long)w64(u(hi), u(lo))); }
    __device__ __forceinline__ void window(const float *s, int &coff, int &cw) const {
        const uint64_t lacc = w64(u(s[kScState + CHS_LFO_ACC]), u(s[kScState + CHS_LFO_LO]));
        const uint64_t linc = w64(u(s[CHC_LFO_INC]), u(s[CHC_LFO_INC_LO]));
        const uint64_t loff = w64(u(s[CHC_LFO_OFF]), u(s[CHC_LFO_OFF_LO]));
        const double D = f64(s[CHC_DEPTH], s[CHC_DEPTH_LO]);
        const double e0 = chorus_delay(lacc + loff, D, (double)(kCsize - 2u));
        const double e1 = chorus_delay(lacc + (uint64_t)(S - 1u) * linc + loff, D, (double)(kCsize - 2u));
        const int dhi = min((int)(fmax(e0, e1) + 0.25), (int)kCsize - 2);
        const int dlo = (int)fmax(fmin(e0, e1) - 0.25, 0.0);
        coff = (dhi + 2) & ~1;                     // t0 - first position (t0 is 4-aligned: even start)
        cw = coff + (int)S - dlo;                  // positions first .. t0 + S - 1 - dlo
    }

    // ---- issue the loads of group g (its scalars already in LDS buffer buf) into registers ----
    __device__ __forceinline__ void issue(uint32_t g, int buf, Pre &pr) {
        const uint32_t i0 = g * kG;
        // pitch rings: piece id -> instance id >> 8, positions t0 - 512 + 2 (id & 255) (+1)
#pragma unroll
        for (int m = 0; m < kPParts; ++m) {
            const uint32_t id = (uint32_t)m * kThreads + tid, j = id >> 8, pp = id & 255u;
            const uint32_t i = i0 + j;
            const uint32_t off = i < n ? (i << 12) + ((t0 + 2u * pp) & (kPsize - 1u)) * 8u : 0xFFFFFFF0u;
            pr.p[m] = ld4(rP, off);
        }
        // input rows: row id >> 2 = (frame, channel), instances 4 (id & 3) .. + 3
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kThreads + tid, row = id >> 2, q = id & 3u;
            const uint32_t f = row >> 1, c = row & 1u, i = i0 + 4u * q;
            const bool ok = f < S && i < n;
            pr.x[m] = ld4(rIn, ok ? c * (uint32_t)a.plane * 4u + f * n * 4u + i * 4u : 0xFFFFFFF0u);
        }
        if (FULL) {
            // chorus windows: piece id -> instance id / 144, positions t0 - coff + 2 (id % 144) (+1),
            // only those older than the block (the block's own are its phase-1 outputs)
#pragma unroll
            for (int m = 0; m < kCLoads; ++m) {
                const uint32_t id = (uint32_t)m * kThreads + tid;
                const uint32_t j = min(id / (uint32_t)kCParts, (uint32_t)kG - 1u), cp = id % (uint32_t)kCParts;
                int coff, cw;
                window(sc(buf, j), coff, cw);
                const int rel = 2 * (int)cp - coff;           // position - t0
                const uint32_t i = i0 + j;
                const bool ok = id < (uint32_t)(kG * kCParts) && i < n && rel < 0 && 2 * (int)cp < cw;
                pr.c[m] = ld4(rC, ok ? (i << 14) + ((t0 + (uint32_t)rel) & (kCsize - 1u)) * 8u : 0xFFFFFFF0u);
            }
        }
    }

    // ---- registers -> LDS (the previous group's readers are done) ----
    __device__ __forceinline__ void fill(int buf, const Pre &pr) {
#pragma unroll
        for (int m = 0; m < kPParts; ++m) {
            const uint32_t id = (uint32_t)m * kThreads + tid, j = id >> 8, pp = id & 255u;
            *(float4 *)(P + j * kPStride + 4u * pp) = pr.p[m];
        }
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kThreads + tid, row = id >> 2, q = id & 3u;
            const uint32_t f = row >> 1, c = row & 1u;
            float *d = P + (4u * q) * kPStride + 2u * ((uint32_t)kPOld + f) + c;
            d[0] = pr.x[m].x;
            d[kPStride] = pr.x[m].y;
            d[2 * kPStride] = pr.x[m].z;
            d[3 * kPStride] = pr.x[m].w;
        }
        if (FULL) {
#pragma unroll
            for (int m = 0; m < kCLoads; ++m) {
                const uint32_t id = (uint32_t)m * kThreads + tid;
                if (id < (uint32_t)(kG * kCParts)) {
                    const uint32_t j = id / (uint32_t)kCParts, cp = id % (uint32_t)kCParts;
                    *(float4 *)(C + j * kCStride + 4u * cp) = pr.c[m];
                }
            }
            // the window geometry of this round, once per instance
            if (tid < (uint32_t)kG) {
                int coff, cw;
                window(sc(buf, tid), coff, cw);
                sc(buf, tid)[kScCoff] = __int_as_float(coff);
                sc(buf, tid)[kScCw] = __int_as_float(cw);
            }
        }
    }

    // ---- phase 1: the pitch-shifter, lanes = frames (wave w: instances 2w, 2w + 1) ----
    __device__ __forceinline__ void phase1(uint32_t g, int buf) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t j = 2u * wave + (uint32_t)h, i = g * kG + j;
            const float *s = sc(buf, j);
            const uint64_t pacc = w64(u(s[kScState + CHS_PS_ACC]), u(s[kScState + CHS_PS_LO]));
            const uint64_t pinc = w64(u(s[CHC_PS_INC]), u(s[CHC_PS_INC_LO]));
            const uint32_t wi = u(s[CHC_WINDOW]), wf = u(s[CHC_WINDOW_LO]);
            const float *pw = P + j * kPStride;
            float *cwin = C + j * kCStride;
            const int coff = FULL ? __float_as_int(s[kScCoff]) : 0;
#pragma unroll
            for (int m = 0; m < kS / 64; ++m) {
                // a fixed trip count (frames past S compute harmlessly, their stores dropped): the
                // compiler then knows how many stores follow a load, and waits for the load only
                const uint32_t k = lane + 64u * (uint32_t)m;
                const bool live = i < n && k < S;
                const uint32_t ph = ch::hi32(pacc + (uint64_t)k * pinc);
                float gA, gB;
                win_gains(ch::unit24(ph), gA, gB);
                uint32_t diA, diB;
                float fA, fB;
                pitch_split(ph, wi, wf, kPsize - 2u, diA, fA);
                pitch_split(ph + 0x80000000u, wi, wf, kPsize - 2u, diB, fB);   // p1 = (p0 + 1/2) % 1
                const float *qA = pw + 2 * (kPOld + (int)k - (int)diA);
                const float *qB = pw + 2 * (kPOld + (int)k - (int)diB);
                const float2 a0 = *(const float2 *)qA, a1 = *(const float2 *)(qA - 2);
                const float2 b0 = *(const float2 *)qB, b1 = *(const float2 *)(qB - 2);
                const float tAL = ch::lerp_pair(a0.x, a1.x, fA), tAR = ch::lerp_pair(a0.y, a1.y, fA);
                const float tBL = ch::lerp_pair(b0.x, b1.x, fB), tBR = ch::lerp_pair(b0.y, b1.y, fB);
                const float2 psv = make_float2(tBL * gB + tAL * gA, tBR * gB + tAR * gA);
                const float2 x = *(const float2 *)(pw + 2 * (kPOld + (int)k));
                // the input into the pitch ring, psv into the chorus ring (512-B runs per wave)
                st2(rP, live ? (i << 12) + ((t0 + k) & (kPsize - 1u)) * 8u : 0xFFFFFFF0u, x);
                if (FULL) {
                    st2(rC, live ? (i << 14) + ((t0 + k) & (kCsize - 1u)) * 8u : 0xFFFFFFF0u, psv);
                    // delay~ writes before it reads: psv into the window (past its end: the junk slot)
                    const uint32_t slot = min((uint32_t)coff + k, (uint32_t)kCWin - 1u);
                    *(float2 *)(cwin + 2u * slot) = psv;
                } else {
                    // the pitch-shifter's output: the chorus window region is unused in this mode
                    // (the pitch window's history is still being read by other lanes)
                    *(float2 *)(cwin + 2u * k) = psv;
                }
            }
        }
    }

    // ---- phase 2: the chorus tap, lanes = frames; w over the dead pitch-window history ----
    __device__ __forceinline__ void phase2(int buf) {
        if (OLFX_CB_DIAG & 2) return;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const uint32_t j = 2u * wave + (uint32_t)h;
            const float *s = sc(buf, j);
            const uint64_t lacc = w64(u(s[kScState + CHS_LFO_ACC]), u(s[kScState + CHS_LFO_LO]));
            const uint64_t linc = w64(u(s[CHC_LFO_INC]), u(s[CHC_LFO_INC_LO]));
            const uint64_t loff = w64(u(s[CHC_LFO_OFF]), u(s[CHC_LFO_OFF_LO]));
            const double D = f64(s[CHC_DEPTH], s[CHC_DEPTH_LO]);
            const int coff = __float_as_int(s[kScCoff]);
            const float *cwin = C + j * kCStride;
            float *wv = P + j * kPStride;
#pragma unroll
            for (int m = 0; m < kS / 64; ++m) {
                const uint32_t k = lane + 64u * (uint32_t)m;
                uint32_t di;
                float fr;
                chorus_split(lacc + (uint64_t)k * linc + loff, D, (double)(kCsize - 2u), di, fr);
                // (a slot outside [1, kCWin - 2] would mean the window bound failed: clamped, never
                // out of the instance's region)
                const int slot = min(max(coff + (int)k - (int)di, 1), kCWin - 2);
                const float2 c0 = *(const float2 *)(cwin + 2 * slot), c1 = *(const float2 *)(cwin + 2 * slot - 2);
                *(float2 *)(wv + 2u * k) = make_float2(ch::lerp_pair(c0.x, c1.x, fr), ch::lerp_pair(c0.y, c1.y, fr));
            }
        }
    }

    // ---- phase 3: lores~ and the mix, one lane per (instance, channel): wave 0, lanes 0..31 ----
    __device__ __forceinline__ void phase3(uint32_t g, int buf) {
        if (wave != 0 || lane >= 2u * kG || (OLFX_CB_DIAG & 1)) return;
        const uint32_t j = lane >> 1, c = lane & 1u, i = g * kG + j;
        const float *s = sc(buf, j);
        const float b0 = s[CHC_B0], b1 = s[CHC_B1], b2 = s[CHC_B2], a1 = s[CHC_A1], a2 = s[CHC_A2];
        const float mix = s[CHC_MIX], dry = s[CHC_DRY];
        float z1 = s[kScState + (c ? CHS_Z1R : CHS_Z1L)], z2 = s[kScState + (c ? CHS_Z2R : CHS_Z2L)];
        float *wv = P + j * kPStride + c;
        const float *xv = P + j * kPStride + 2 * kPOld + c;
        // 4-frame steps (S is a multiple of 4); the next step's LDS reads are issued before this
        // step's recurrence, so their latency hides under it
        float wet[4], x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            wet[q] = wv[2 * q];
            x[q] = xv[2 * q];
        }
        for (uint32_t k0 = 0; k0 < S; k0 += 4) {
            float wn[4], xn[4];
            const uint32_t k1 = min(k0 + 4u, (uint32_t)kS - 4u);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                wn[q] = wv[2 * (k1 + q)];
                xn[q] = xv[2 * (k1 + q)];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const float lp = b0 * wet[q] + z1;
                z1 = (b1 * wet[q] - a1 * lp) + z2;
                z2 = b2 * wet[q] - a2 * lp;
                wv[2 * (k0 + q)] = x[q] * dry + lp * mix;
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                wet[q] = wn[q];
                x[q] = xn[q];
            }
        }
        if (i < n) {
            a.state[(c ? CHS_Z1R : CHS_Z1L) * n + i] = __float_as_uint(z1);
            a.state[(c ? CHS_Z2R : CHS_Z2L) * n + i] = __float_as_uint(z2);
        }
    }

    // the phasors after the block (lanes 32..47 of wave 0: beside phase 3)
    __device__ __forceinline__ void phasors(uint32_t g, int buf) {
        if (wave != 0 || lane < 32u || lane >= 32u + kG) return;
        const uint32_t j = lane - 32u, i = g * kG + j;
        if (i >= n) return;
        const float *s = sc(buf, j);
        const uint64_t lacc = w64(u(s[kScState + CHS_LFO_ACC]), u(s[kScState + CHS_LFO_LO])) +
                              (uint64_t)S * w64(u(s[CHC_LFO_INC]), u(s[CHC_LFO_INC_LO]));
        const uint64_t pacc = w64(u(s[kScState + CHS_PS_ACC]), u(s[kScState + CHS_PS_LO])) +
                              (uint64_t)S * w64(u(s[CHC_PS_INC]), u(s[CHC_PS_INC_LO]));
        a.state[CHS_LFO_ACC * n + i] = (uint32_t)(lacc >> 32);
        a.state[CHS_LFO_LO * n + i] = (uint32_t)lacc;
        a.state[CHS_PS_ACC * n + i] = (uint32_t)(pacc >> 32);
        a.state[CHS_PS_LO * n + i] = (uint32_t)pacc;
    }

    // ---- output rows from LDS (chorus: over the pitch-window history; pitch-shift: the chorus
    // window region) ----
    __device__ __forceinline__ void out(uint32_t g) {
        const uint32_t i0 = g * kG;
        const float *Y = FULL ? P : C;
        constexpr uint32_t kYs = FULL ? (uint32_t)kPStride : (uint32_t)kCStride;
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kThreads + tid, row = id >> 2, q = id & 3u;
            const uint32_t f = row >> 1, c = row & 1u, i = i0 + 4u * q;
            const float *sv = Y + (4u * q) * kYs + 2u * f + c;
            const float4 v = make_float4(sv[0], sv[kYs], sv[2 * kYs], sv[3 * kYs]);
            const bool ok = f < S && i < n;
            st4<ch::kStreamAux>(rOut, ok ? c * (uint32_t)a.plane * 4u + f * n * 4u + i * 4u : 0xFFFFFFF0u, v);
        }
    }
};

}  // namespace cb
}  // namespace olfx
