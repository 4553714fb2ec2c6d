// ol_dsp_amd/csrc/chorus_pc.h -- chorus_block_v14: chorus_block_v13's block-at-once stereo chorus
// with lores~ on its own wave, overlapped with the next group's work.
//
// v13 (chorus_block.h) computes the pitch-shifter and the chorus tap frame-parallel, then runs
// lores~ (the spec's only recurrence: 256 dependent biquad steps per (instance, channel), ~5-8 us
// on one wave) while every other wave of the workgroup waits at a barrier: the LDS that the next
// group is loaded into still holds what lores~ reads.  Measured: lores~ added its whole length to
// every round (diagnostic builds without it: 0.33 -> 0.21 ms).  v14 gives lores~ a wave of its own
// and its inputs a region of their own, so it runs while the producer waves fill and compute the
// next group:
//
//   producers (waves 0-6)                          consumer (wave 7)
//   p1(r)  pitch-shifter, lanes = frames
//   issue(r+1) loads -> registers
//   wait  p3 done(r-1); out(r-1) rows from W
//   p2(r)  chorus tap: (w, x dry) -> W             -> wready(r)
//   fill(r+1) registers -> P, C                      p3(r): lores~ over W, y over w in W
//   p1(r+1) ...                                      -> p3 done(r)
//
// A group is 12 stereo instances (LDS: pitch windows 74 KB + chorus windows 28 KB + W 49 KB + scalars,
// 154 KB; v13's 16 left no room for W).  Producers synchronise among themselves and with the consumer
// through LDS counters (lds_flags.h), never s_barrier, so the consumer never waits for them mid-round.
// Scalars are triple-buffered by round (the consumer reads round r's while the producers write r+1's
// and r+2's).  Frame arithmetic, layouts and the chorus window bound are v13's (spec v2, bit-exact
// against oracle/chorus_ref.c).
#pragma once
#include "chorus_block.h"
#include "lds_flags.h"

namespace olfx {
namespace pc {

using cb::kS;
using cb::kPsize;
using cb::kCsize;
using cb::kPOld;
using cb::kPStride;
using cb::kCWin;
using cb::kCStride;
using cb::kCParts;
using cb::kScW;
using cb::kScState;
using cb::kScCoff;
using cb::kScCw;
using ch::Rsrc;
using ch::rsrc;
using ch::ld4;
using ch::st4;

constexpr int kG = 12;                         // stereo instances per group
constexpr int kThreads = 512;
constexpr int kProd = 7;                       // producer waves; wave 7 runs lores~
constexpr uint32_t kPL = kProd * 64;           // producer lanes
constexpr int kWStride = 2 * 2 * kS + 4;       // W floats per instance: [k][ch][w, x dry] (+4: bank spread)
constexpr int kNBuf = 3;                       // scalar buffers (round r uses r % 3)
constexpr int kFlags = 4;                      // LDS words: producer barrier, wready, p3done
constexpr int kLdsFloats = kG * kPStride + kG * kCStride + kG * kWStride + kNBuf * kG * kScW + kFlags;
static_assert(kLdsFloats * 4 <= 160 * 1024, "LDS budget");

constexpr int kPParts = (kG * (int)kPsize / 2 + (int)kPL - 1) / (int)kPL;     // 7
constexpr int kXRows = 2 * kS;                                                  // (frame, channel) rows
constexpr int kXParts = (kXRows * (kG / 4) + (int)kPL - 1) / (int)kPL;          // 4
constexpr int kCLoads = (kG * kCParts + (int)kPL - 1) / (int)kPL;               // 4
constexpr int kItems = kG * (kS / 64);                                          // 48 (instance, quarter)
constexpr int kItemsPerWave = (kItems + kProd - 1) / kProd;                     // 7
constexpr int kScLoads = kG * (CHC_N + CHS_N);
static_assert(kScLoads <= (int)kPL, "scalar loads");

struct Pre {
    float4 p[kPParts];
    float4 x[kXParts];
    float4 c[kCLoads];
};

struct Block {
    const ChorusArgs &a;
    float *P, *C, *W, *Sc;
    uint32_t *flags;              // [0] producer barrier arrivals, [1] wready, [2] p3done
    uint32_t tid, wave, lane;
    uint32_t n, S, t0;
    Rsrc rP, rC, rIn, rOut;
    uint32_t pbar;                // producer barrier generation (arrivals expected: kProd x pbar)

    __device__ __forceinline__ Block(const ChorusArgs &a_, float *lds) : a(a_) {
        P = lds;
        C = P + kG * kPStride;
        W = C + kG * kCStride;
        Sc = W + kG * kWStride;
        flags = (uint32_t *)(Sc + kNBuf * kG * kScW);
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
        pbar = 0;
    }

    __device__ __forceinline__ float *sc(int buf, uint32_t j) { return Sc + (buf * kG + j) * kScW; }
    __device__ __forceinline__ static uint64_t w64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }
    __device__ __forceinline__ static uint32_t u(float v) { return __float_as_uint(v); }
    __device__ __forceinline__ static double f64(float hi, float lo) { return __longlong_as_double((long long)w64(u(hi), u(lo))); }

    // ---- synchronisation through LDS counters ----
    // producers only: every producer wave arrives, then waits for all kProd arrivals of this
    // generation (the counter only grows)
    __device__ __forceinline__ void producer_barrier() {
        ++pbar;
        __builtin_amdgcn_s_waitcnt(0xC07F);           // lgkmcnt(0): this wave's LDS accesses done
        if (lane == 0) __hip_atomic_fetch_add(&flags[0], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t want = (uint32_t)kProd * pbar;
        wait_for([&] { return flag_get(&flags[0]) >= want; });
    }
    __device__ __forceinline__ void signal(int f, uint32_t v) {
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (lane == 0) flag_put(&flags[f], v);
    }
    __device__ __forceinline__ void wait_flag(int f, uint32_t v) {
        wait_for([&] { return flag_get(&flags[f]) >= v; });
    }

    // ---- scalars of group g: producer lane tid < 300 loads word (tid % 25) of instance (tid / 25) ----
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

    // the chorus window of one instance (v13's bound: chorus_block.h Block::window)
    __device__ __forceinline__ void window(const float *s, int &coff, int &cw) const {
        const uint64_t lacc = w64(u(s[kScState + CHS_LFO_ACC]), u(s[kScState + CHS_LFO_LO]));
        const uint64_t linc = w64(u(s[CHC_LFO_INC]), u(s[CHC_LFO_INC_LO]));
        const uint64_t loff = w64(u(s[CHC_LFO_OFF]), u(s[CHC_LFO_OFF_LO]));
        const double D = f64(s[CHC_DEPTH], s[CHC_DEPTH_LO]);
        const double e0 = chorus_delay(lacc + loff, D, (double)(kCsize - 2u));
        const double e1 = chorus_delay(lacc + (uint64_t)(S - 1u) * linc + loff, D, (double)(kCsize - 2u));
        const int dhi = min((int)(fmax(e0, e1) + 0.25), (int)kCsize - 2);
        const int dlo = (int)fmax(fmin(e0, e1) - 0.25, 0.0);
        coff = (dhi + 2) & ~1;
        cw = coff + (int)S - dlo;
    }

    // ---- group g's loads into registers (producers; its scalars already in buffer buf) ----
    __device__ __forceinline__ void issue(uint32_t g, int buf, Pre &pr) {
        const uint32_t i0 = g * kG;
#pragma unroll
        for (int m = 0; m < kPParts; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid, j = id >> 8, pp = id & 255u;
            const uint32_t i = i0 + j;
            const bool ok = j < (uint32_t)kG && i < n;
            pr.p[m] = ld4(rP, ok ? (i << 12) + ((t0 + 2u * pp) & (kPsize - 1u)) * 8u : 0xFFFFFFF0u);
        }
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid, row = id / 3u, q = id % 3u;
            const uint32_t f = row >> 1, c = row & 1u, i = i0 + 4u * q;
            const bool ok = row < (uint32_t)kXRows && f < S && i < n;
            pr.x[m] = ld4(rIn, ok ? c * (uint32_t)a.plane * 4u + f * n * 4u + i * 4u : 0xFFFFFFF0u);
        }
#pragma unroll
        for (int m = 0; m < kCLoads; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid;
            const uint32_t j = min(id / (uint32_t)kCParts, (uint32_t)kG - 1u), cp = id % (uint32_t)kCParts;
            int coff, cw;
            window(sc(buf, j), coff, cw);
            const int rel = 2 * (int)cp - coff;
            const uint32_t i = i0 + j;
            const bool ok = id < (uint32_t)(kG * kCParts) && i < n && rel < 0 && 2 * (int)cp < cw;
            pr.c[m] = ld4(rC, ok ? (i << 14) + ((t0 + (uint32_t)rel) & (kCsize - 1u)) * 8u : 0xFFFFFFF0u);
        }
    }

    // ---- registers -> P, C and the window geometry (producers) ----
    __device__ __forceinline__ void fill(int buf, const Pre &pr) {
#pragma unroll
        for (int m = 0; m < kPParts; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid, j = id >> 8, pp = id & 255u;
            if (j < (uint32_t)kG) *(float4 *)(P + j * kPStride + 4u * pp) = pr.p[m];
        }
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid, row = id / 3u, q = id % 3u;
            if (row < (uint32_t)kXRows) {
                const uint32_t f = row >> 1, c = row & 1u;
                float *d = P + (4u * q) * kPStride + 2u * ((uint32_t)kPOld + f) + c;
                d[0] = pr.x[m].x;
                d[kPStride] = pr.x[m].y;
                d[2 * kPStride] = pr.x[m].z;
                d[3 * kPStride] = pr.x[m].w;
            }
        }
#pragma unroll
        for (int m = 0; m < kCLoads; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid;
            if (id < (uint32_t)(kG * kCParts)) {
                const uint32_t j = id / (uint32_t)kCParts, cp = id % (uint32_t)kCParts;
                *(float4 *)(C + j * kCStride + 4u * cp) = pr.c[m];
            }
        }
        if (tid < (uint32_t)kG) {
            int coff, cw;
            window(sc(buf, tid), coff, cw);
            sc(buf, tid)[kScCoff] = __int_as_float(coff);
            sc(buf, tid)[kScCw] = __int_as_float(cw);
        }
    }

    // ---- p1: the pitch-shifter (producers; item = (instance, 64-frame quarter), lanes = frames) ----
    __device__ __forceinline__ void phase1(uint32_t g, int buf) {
#pragma unroll
        for (int m = 0; m < kItemsPerWave; ++m) {
            // a fixed trip count: past the last item a wave recomputes it (identical LDS writes, its
            // HBM stores dropped), so the compiler knows how many stores follow each load
            const uint32_t it0 = wave + (uint32_t)kProd * (uint32_t)m;
            const bool dup = it0 >= (uint32_t)kItems;
            const uint32_t it = dup ? (uint32_t)kItems - 1u : it0;
            const uint32_t j = it >> 2, k = ((it & 3u) << 6) + lane, i = g * kG + j;
            const float *s = sc(buf, j);
            const uint64_t pacc = w64(u(s[kScState + CHS_PS_ACC]), u(s[kScState + CHS_PS_LO]));
            const uint64_t pinc = w64(u(s[CHC_PS_INC]), u(s[CHC_PS_INC_LO]));
            const uint32_t wi = u(s[CHC_WINDOW]), wf = u(s[CHC_WINDOW_LO]);
            const float *pw = P + j * kPStride;
            float *cwin = C + j * kCStride;
            const int coff = __float_as_int(s[kScCoff]);
            const bool live = i < n && k < S && !dup;
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
            cb::st2(rP, live ? (i << 12) + ((t0 + k) & (kPsize - 1u)) * 8u : 0xFFFFFFF0u, x);
            cb::st2(rC, live ? (i << 14) + ((t0 + k) & (kCsize - 1u)) * 8u : 0xFFFFFFF0u, psv);
            const uint32_t slot = min((uint32_t)coff + k, (uint32_t)kCWin - 1u);   // delay~ writes first
            *(float2 *)(cwin + 2u * slot) = psv;
        }
    }

    // ---- p2: the chorus tap and x dry (producers) -> W [j][k][ch][w, x dry] ----
    __device__ __forceinline__ void phase2(int buf) {
#pragma unroll
        for (int m = 0; m < kItemsPerWave; ++m) {
            const uint32_t it = min(wave + (uint32_t)kProd * (uint32_t)m, (uint32_t)kItems - 1u);
            const uint32_t j = it >> 2, k = ((it & 3u) << 6) + lane;
            const float *s = sc(buf, j);
            const uint64_t lacc = w64(u(s[kScState + CHS_LFO_ACC]), u(s[kScState + CHS_LFO_LO]));
            const uint64_t linc = w64(u(s[CHC_LFO_INC]), u(s[CHC_LFO_INC_LO]));
            const uint64_t loff = w64(u(s[CHC_LFO_OFF]), u(s[CHC_LFO_OFF_LO]));
            const double D = f64(s[CHC_DEPTH], s[CHC_DEPTH_LO]);
            const float dry = s[CHC_DRY];
            const int coff = __float_as_int(s[kScCoff]);
            const float *cwin = C + j * kCStride;
            uint32_t di;
            float fr;
            chorus_split(lacc + (uint64_t)k * linc + loff, D, (double)(kCsize - 2u), di, fr);
            const int slot = min(max(coff + (int)k - (int)di, 1), kCWin - 2);
            const float2 c0 = *(const float2 *)(cwin + 2 * slot), c1 = *(const float2 *)(cwin + 2 * slot - 2);
            const float2 x = *(const float2 *)(P + j * kPStride + 2 * (kPOld + (int)k));
            // x dry: the mix's first product (y = x dry + lp mix, the spec's order)
            *(float4 *)(W + j * kWStride + 4u * k) =
                make_float4(ch::lerp_pair(c0.x, c1.x, fr), x.x * dry, ch::lerp_pair(c0.y, c1.y, fr), x.y * dry);
        }
    }

    // ---- p3: lores~ and the mix (the consumer wave; lane = (instance, channel), 24 lanes) ----
    __device__ __forceinline__ void phase3(uint32_t g, int buf) {
        if (lane >= 2u * kG) {
            // lanes 32..43: the phasors after the block
            if (lane < 32u || lane >= 32u + kG) return;
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
            return;
        }
        const uint32_t j = lane >> 1, c = lane & 1u, i = g * kG + j;
        const float *s = sc(buf, j);
        const float b0 = s[CHC_B0], b1 = s[CHC_B1], b2 = s[CHC_B2], a1 = s[CHC_A1], a2 = s[CHC_A2];
        const float mix = s[CHC_MIX];
        float z1 = s[kScState + (c ? CHS_Z1R : CHS_Z1L)], z2 = s[kScState + (c ? CHS_Z2R : CHS_Z2L)];
        float *wv = W + j * kWStride + 2u * c;           // (w, x dry) of frame k at wv + 4 k
        // 4-frame steps, the next step's reads issued before this step's recurrence
        float2 q[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) q[t] = *(const float2 *)(wv + 4 * t);
        for (uint32_t k0 = 0; k0 < S; k0 += 4) {
            float2 qn[4];
            const uint32_t k1 = min(k0 + 4u, (uint32_t)kS - 4u);
#pragma unroll
            for (int t = 0; t < 4; ++t) qn[t] = *(const float2 *)(wv + 4 * (k1 + t));
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const float wet = q[t].x;
                const float lp = b0 * wet + z1;
                z1 = (b1 * wet - a1 * lp) + z2;
                z2 = b2 * wet - a2 * lp;
                wv[4 * (k0 + t)] = q[t].y + lp * mix;       // y over w
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) q[t] = qn[t];
        }
        if (i < n) {
            a.state[(c ? CHS_Z1R : CHS_Z1L) * n + i] = __float_as_uint(z1);
            a.state[(c ? CHS_Z2R : CHS_Z2L) * n + i] = __float_as_uint(z2);
        }
    }

    // ---- output rows of group g from W (producers, after its p3); valid = false: stores dropped
    // (a fixed number of stores on every path) ----
    __device__ __forceinline__ void out(uint32_t g, bool valid) {
        const uint32_t i0 = g * kG;
#pragma unroll
        for (int m = 0; m < kXParts; ++m) {
            const uint32_t id = (uint32_t)m * kPL + tid, row = id / 3u, q = id % 3u;
            const uint32_t f = row >> 1, c = row & 1u, i = i0 + 4u * q;
            const bool ok = valid && row < (uint32_t)kXRows && f < S && i < n;
            const float *sv = W + (4u * q) * kWStride + 4u * min(f, (uint32_t)kS - 1u) + 2u * c;
            const float4 v = make_float4(sv[0], sv[kWStride], sv[2 * kWStride], sv[3 * kWStride]);
            st4<ch::kStreamAux>(rOut, ok ? c * (uint32_t)a.plane * 4u + f * n * 4u + i * 4u : 0xFFFFFFF0u, v);
        }
    }
};

}  // namespace pc
}  // namespace olfx
