// ol_dsp_amd/csrc/chorus_stage.h -- the RNBO stereo chorus / gen~ pitch-shifter as a per-lane device stage.
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
// Mapping: one lane = one (instance, channel); a wave = 32 instances x 2 channels (lane 2j+ch).
// Rings are instance-private ([inst][size][2], stereo-interleaved: L and R share every tap
// position) because every tap is modulated per instance.  The block is processed in chunks of 16 frames.  Each tap of a chunk touches a window
// of <= 24 consecutive ring positions (the pitch taps are monotone inside a chunk unless the
// phasor wraps; the chorus tap moves < 0.6 positions per chunk for every legal depth/rate).
//
// Memory shape (profiles/r1): per-lane scattered 16-B accesses saturated the TA/TCP with one L2
// request per 16 B (TA busy 87 %, TCP pending-stall 85 %), so both directions are COOPERATIVE:
//   * window loads: 6 consecutive lanes fetch one owner's contiguous 96-B window (owners' window
//     starts broadcast with ds_bpermute), ~11 contiguous segments per wave-load;
//   * ring stores: each lane stages its 16 new samples in its wave's LDS region, then 4 lanes
//     write one owner's 64-B run, 16 runs per wave-store.
// Windows land in LDS as [wave][tap][slot][lane]: the per-frame fractional reads of the serial
// recurrence are bank-conflict free (x0/x1 one ds_read2st64 apart).  All global traffic uses
// buffer ops with 32-bit offsets (frame offsets in SGPRs): fewer VGPRs, no 64-bit address math.
// Software pipeline (one chunk ahead): while chunk c computes, chunk c+1's inputs and windows are
// in flight; window positions that chunk c / c+1 themselves produce (inputs not yet in the pitch
// ring, chorus outputs not yet in the chorus ring) are patched into LDS from registers.  A pitch
// window that cannot cover its chunk (phasor wrap, once per 1/shift s) falls back to direct ring
// reads for that lane and chunk.
#pragma once
#include <type_traits>

#include "olfx_internal.h"

namespace olfx {
namespace ch {

constexpr int kThreads = 256;
constexpr int kRow = 64;                    // LDS slot stride: one wave's lanes

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc rsrc(const void *p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0,
                                             (int)(uint32_t)(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes), 0x00020000);
}
// cache policy of the streamed accesses (block input/output, ring stores): 0 = default,
// 2 = nt (gfx950 aux bit 1).  A/B knob; the shipped value is measured.
#ifndef OLFX_STREAM_AUX
#define OLFX_STREAM_AUX 0
#endif
constexpr int kStreamAux = OLFX_STREAM_AUX;

template <int AUX = 0>
__device__ __forceinline__ float ld1(Rsrc r, uint32_t voff, uint32_t soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
}
template <int AUX = 0>
__device__ __forceinline__ void st1(Rsrc r, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, AUX);
}
__device__ __forceinline__ float4 ld4(Rsrc r, uint32_t voff) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <int AUX = 0>
__device__ __forceinline__ void st4(Rsrc r, uint32_t voff, float4 v) {
    u32x4 u;
    u.x = __float_as_uint(v.x); u.y = __float_as_uint(v.y); u.z = __float_as_uint(v.z); u.w = __float_as_uint(v.w);
    __builtin_amdgcn_raw_buffer_store_b128(u, r, voff, 0, AUX);
}

// exchange a value with the neighbouring lane (lanes 2j <-> 2j+1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ float swap_pair(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

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

__device__ __forceinline__ int floor_delay(float d, float dmin, float dmax) {
    return (int)(uint32_t)fminf(fmaxf(d, dmin), dmax);
}

__device__ __forceinline__ float lerp_pair(float x0, float x1, float fr) { return x0 + fr * (x1 - x0); }

// cos(2 pi x) for |x| <= 0.25: cos2pi() (olfx_internal.h) with its range reduction folded away.
// There u = x - rint(x) = x, a = |x| <= 0.25 never takes the reflected branch, and
// (x 2pi)^2 == (|x| 2pi)^2 exactly: bit-identical results, six fewer instructions.
__device__ __forceinline__ float cos2pi_q(float x) {
    const float th = x * 6.28318530717958647692f;
    const float t2 = th * th;
    return 1.0f + t2 * (-0.5f + t2 * (4.16666666666666666667e-2f +
           t2 * (-1.38888888888888888889e-3f + t2 * (2.48015873015873015873e-5f +
           t2 * (-2.75573192239858906526e-7f + t2 * (2.08767569878680989792e-9f +
           t2 * (-1.14707455977297247139e-11f)))))));
}
// a value of lane 2j (EVEN) or 2j+1 (odd) to both lanes of the pair: DPP quad_perm [0,0,2,2] / [1,1,3,3]
__device__ __forceinline__ float pair_even(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xA0, 0xF, 0xF, false));
}
__device__ __forceinline__ float pair_odd(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xF5, 0xF, 0xF, false));
}
// split_delay with the clamp as one v_med3 (identical to fminf(fmaxf()) for non-NaN delays,
// and delays here are phasor arithmetic, never NaN)
__device__ __forceinline__ void split_delay3(float d, float dmin, float dmax, int &di, float &fr) {
    d = __builtin_amdgcn_fmed3f(d, dmin, dmax);
    const uint32_t u = (uint32_t)d;
    di = (int)u;
    fr = d - (float)u;
}


// Window geometry of one chunk for one lane: starts (relative to the chunk's first write
// position, multiples of 4) of the two pitch windows and the chorus window.
struct Plan {
    int sA, sB, sC;
    bool okA, okB;
};

template <int kWin>
__device__ __forceinline__ Plan plan_chunk(uint32_t lfo_acc, uint32_t lfo_inc, uint32_t lfo_off, uint32_t ps_acc,
                                           uint32_t ps_inc, int C, float D, float W, float pmax, float cmax,
                                           bool full) {
    Plan p;
    const uint32_t last = (uint32_t)(C - 1);
    // pitch taps: d = p W is monotone in p; p is monotone over the chunk unless its phasor wraps
    {
        const uint32_t a0 = ps_acc, a1 = ps_acc + last * ps_inc;
        const int d0 = floor_delay(unit24(a0) * W, 1.0f, pmax), d1 = floor_delay(unit24(a1) * W, 1.0f, pmax);
        const int lo = -d1 - 1, hi = (int)last - d0;
        p.sA = lo & ~3;
        p.okA = a1 >= a0 && hi - p.sA < kWin;
    }
    {
        const uint32_t a0 = ps_acc + 0x80000000u, a1 = a0 + last * ps_inc;
        const int d0 = floor_delay(unit24(a0) * W, 1.0f, pmax), d1 = floor_delay(unit24(a1) * W, 1.0f, pmax);
        const int lo = -d1 - 1, hi = (int)last - d0;
        p.sB = lo & ~3;
        p.okB = a1 >= a0 && hi - p.sB < kWin;
    }
    // chorus tap: |d'| <= 2 pi D f_lfo / sr <= 0.038 frame/frame for depth <= 12 ms, rate <= 0.5 Hz,
    // so every frame of the chunk lies within +-1 of the endpoint delays
    p.sC = 0;
    if (full) {
        const float e0 = cos2pi(unit24(lfo_acc + lfo_off)) * D + D;
        const float e1 = cos2pi(unit24(lfo_acc + last * lfo_inc + lfo_off)) * D + D;
        const int dhi = floor_delay(fmaxf(e0, e1) + 1.0f, 0.0f, cmax);
        p.sC = (-dhi - 1) & ~3;
    }
    return p;
}


// One (instance, channel) lane of the chorus / pitch-shifter as a resumable stage: begin() once
// per launch with the first chunk's input, chunk() per 16-frame chunk (input in registers,
// output returned in registers), finish() at the end.  A wave holds 32 instances x 2 channels,
// lane = 2 j + ch.  Used by chorus_block (input from the audio buffer) and by the fused chain
// (stage 1 from the audio buffer, stage 2 fed by stage 1's output in the same lane).
template <bool FULL>
struct ChStage {
    static constexpr int kChunk = 16, kWin = 24, kSlots = kWin + 1;
    static constexpr int kRegion = 3 * kSlots * kRow;   // floats of LDS per wave (4,800)
    static constexpr int kStride = 36;                  // staging floats per instance (32 + pad)
    static constexpr uint32_t kPsvBase = 32u * kStride;
    static_assert(2 * 32 * kStride <= kRegion, "staging must fit in the window region");

    uint32_t lane, j, ch, inst0, n, i;
    bool valid;
    uint32_t lfo_inc, lfo_off, ps_inc;
    float D, W, b0, b1, b2, a1, a2, mix, dry;
    uint32_t lfo_acc, ps_acc;
    float z1, z2;
    uint32_t pmask, cmask, pstride, cstride, own_pb;
    float pmax, cmax;
    Rsrc rP, rC;
    float *region;
    float4 vA[6], vB[6], vC[6];
    Plan pl;
    float psv[kChunk];
    uint32_t wpos;                                      // ring write position of the next chunk
    bool started;

    __device__ __forceinline__ void init(const ChorusArgs &a, float *lds_region, uint32_t lane_, uint32_t inst0_) {
        lane = lane_; j = lane >> 1; ch = lane & 1u; inst0 = inst0_; n = a.n;
        const uint32_t i_raw = inst0 + j;
        valid = i_raw < n;                              // invalid lanes still help load windows
        i = valid ? i_raw : n - 1;
        lfo_inc = a.coef[CHC_LFO_INC * n + i];
        lfo_off = a.coef[CHC_LFO_OFF * n + i];
        ps_inc = a.coef[CHC_PS_INC * n + i];
        D = __uint_as_float(a.coef[CHC_DEPTH * n + i]);
        W = __uint_as_float(a.coef[CHC_WINDOW * n + i]);
        b0 = __uint_as_float(a.coef[CHC_B0 * n + i]);
        b1 = __uint_as_float(a.coef[CHC_B1 * n + i]);
        b2 = __uint_as_float(a.coef[CHC_B2 * n + i]);
        a1 = __uint_as_float(a.coef[CHC_A1 * n + i]);
        a2 = __uint_as_float(a.coef[CHC_A2 * n + i]);
        mix = __uint_as_float(a.coef[CHC_MIX * n + i]);
        dry = __uint_as_float(a.coef[CHC_DRY * n + i]);
        lfo_acc = a.state[CHS_LFO_ACC * n + i];
        ps_acc = a.state[CHS_PS_ACC * n + i];
        z1 = __uint_as_float(a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i]);
        z2 = __uint_as_float(a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i]);
        pmask = a.psize - 1u; cmask = a.csize - 1u;
        pmax = (float)(a.psize - 2u); cmax = (float)(a.csize - 2u);
        rP = rsrc(a.pitch_ring, (uint64_t)n * 2 * a.psize * 4);
        rC = rsrc(a.chorus_ring, (uint64_t)n * 2 * a.csize * 4);
        pstride = a.psize * 8u; cstride = a.csize * 8u; // bytes per instance ring
        own_pb = i * pstride + ch * 4u;                 // this lane's samples in its pitch ring
        region = lds_region;
        wpos = a.t0;
        started = false;
    }

    // cooperative-load geometry: in part-load r (0..5) of a tap, this lane fetches piece m
    // (positions 2m, 2m+1 of both channels = 16 B) of instance jj's stereo window; 4 consecutive
    // lanes cover 64 contiguous bytes of one instance, 16 instances per load
    __device__ __forceinline__ uint32_t ljj(int r) const { return (((uint32_t)r * 64u + lane) >> 2) & 31u; }
    __device__ __forceinline__ uint32_t lm(int r) const { return ((((uint32_t)r * 64u + lane) >> 7) << 2) | (lane & 3u); }

    __device__ __forceinline__ void load_windows(const Plan &p, uint32_t w) {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            const uint32_t jj = ljj(r), m2 = 2u * lm(r);
            const int src = (int)(jj << 3);             // lane 2 jj holds instance jj's plan
            const int oA = __builtin_amdgcn_ds_bpermute(src, p.sA);
            const int oB = __builtin_amdgcn_ds_bpermute(src, p.sB);
            const int oC = __builtin_amdgcn_ds_bpermute(src, p.sC);
            const uint32_t oi = min(inst0 + jj, n - 1);  // lanes past n load a harmless duplicate
            vA[r] = ld4(rP, oi * pstride + ((w + oA + m2) & pmask) * 8u);
            vB[r] = ld4(rP, oi * pstride + ((w + oB + m2) & pmask) * 8u);
            if (FULL) vC[r] = ld4(rC, oi * cstride + ((w + oC + m2) & cmask) * 8u);
        }
    }
    // de-interleave each piece into the two channel columns of its instance: (L,R) pairs are
    // adjacent columns of one slot row, one 8-B LDS write per position
    __device__ __forceinline__ void stage_windows() {
#pragma unroll
        for (int r = 0; r < 6; ++r) {
            float *pA = region + 2u * lm(r) * kRow + 2u * ljj(r);
            float *pB = pA + kSlots * kRow, *pC = pA + 2 * kSlots * kRow;
            *(float2 *)pA = make_float2(vA[r].x, vA[r].y);
            *(float2 *)(pA + kRow) = make_float2(vA[r].z, vA[r].w);
            *(float2 *)pB = make_float2(vB[r].x, vB[r].y);
            *(float2 *)(pB + kRow) = make_float2(vB[r].z, vB[r].w);
            if (FULL) {
                *(float2 *)pC = make_float2(vC[r].x, vC[r].y);
                *(float2 *)(pC + kRow) = make_float2(vC[r].z, vC[r].w);
            }
        }
    }
    // Cooperative ring store of a chunk: the lanes have staged [instance][frame][ch] at
    // region + base; 8 consecutive lanes then write one instance's 128-B stereo run.
    __device__ __forceinline__ void stage_run(const float (&v)[kChunk], uint32_t base) {
        float *st = region + base + j * kStride + ch;
#pragma unroll
        for (int k = 0; k < kChunk; ++k) st[2 * k] = v[k];
    }
    __device__ __forceinline__ void coop_store(bool pitch, uint32_t base, uint32_t w, int C) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = (uint32_t)r * 64u + lane, o = q >> 3, f2 = 2u * (q & 7u);
            const float4 v = *(const float4 *)(region + base + o * kStride + 2u * f2);
            const uint32_t oi = inst0 + o;
            if (oi < n && (int)f2 < C) {
                if (pitch) st4<kStreamAux>(rP, oi * pstride + ((w + f2) & pmask) * 8u, v);
                else st4<kStreamAux>(rC, oi * cstride + ((w + f2) & cmask) * 8u, v);
            }
        }
    }

    // first chunk (C frames) of the launch: its inputs go to the pitch ring before its windows
    // are loaded
    __device__ __forceinline__ void begin(const float (&x)[kChunk], int C) {
        stage_run(x, 0);
        coop_store(true, 0, wpos, C);
        pl = plan_chunk<kWin>(lfo_acc, lfo_inc, lfo_off, ps_acc, ps_inc, C, D, W, pmax, cmax, FULL);
        load_windows(pl, wpos);
    }

    // One chunk of C frames (multiple of 4) with input x; Cn = frames of the next chunk of this
    // launch (0 = none).  sink(k, y) receives frame k's output as soon as it is computed (chorus:
    // the mixed output; pitch-shift: the wet signal); it is not called for frames k >= C.
    template <class Sink>
    __device__ __forceinline__ void chunk(const float (&x)[kChunk], int C, int Cn, Sink &&sink) {
        const uint32_t w0 = wpos;
        const Plan cur = pl;
        float *wP0 = region + 0 * kSlots * kRow + lane;
        float *wP1 = region + 1 * kSlots * kRow + lane;
        float *wC = region + 2 * kSlots * kRow + lane;

        // ---- 1. this chunk's inputs -> pitch ring (cooperative; the first chunk did it in
        //         begin()), using the wave's LDS region while it is free ----
        if (started) {
            stage_run(x, 0);
            coop_store(true, 0, w0, C);
        }
        // ---- 2. staged windows -> LDS, patched with positions still held in registers ----
        stage_windows();
        if (started) {
            // this chunk's inputs were not in the pitch ring when its windows were loaded
            if (cur.sA > -kWin) {
#pragma unroll
                for (int k = 0; k < kChunk; ++k)
                    if (k < C && k - cur.sA < kWin) wP0[(k - cur.sA) * kRow] = x[k];
            }
            if (cur.sB > -kWin) {
#pragma unroll
                for (int k = 0; k < kChunk; ++k)
                    if (k < C && k - cur.sB < kWin) wP1[(k - cur.sB) * kRow] = x[k];
            }
            // nor were the previous chunk's pitch-shifter outputs in the chorus ring
            if (FULL && cur.sC > -kWin - kChunk) {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    const int jw = k - kChunk - cur.sC;
                    if (jw >= 0 && jw < kWin) wC[jw * kRow] = psv[k];
                }
            }
        }
        started = true;

        // ---- 3. issue the next chunk's window loads (consumed next chunk).  Unconditional: after
        //         the last chunk they read valid ring memory and are dropped (loads under a branch
        //         cost precise waitcnt tracking of the whole pipeline at the merge) ----
        pl = plan_chunk<kWin>(lfo_acc + (uint32_t)C * lfo_inc, lfo_inc, lfo_off, ps_acc + (uint32_t)C * ps_inc,
                              ps_inc, Cn > 0 ? Cn : 4, D, W, pmax, cmax, FULL);
        load_windows(pl, w0 + kChunk);

        // ---- 4. the serial recurrence over this chunk ----
        // GENERIC = partial chunk or some lane's pitch window misses (phasor wrap): per-frame
        // guards and per-lane fallback reads.  The common case runs branch-free.
        // The LFO and the two window gains are the same for both channels of an instance (shared
        // phasors), and the two lanes of a pair are adjacent: for each frame pair, each lane
        // evaluates the three cosines of ONE frame (its channel's index) and swaps them with its
        // partner by DPP -- half the transcendental work, identical bits.
        float pl_lfo[2], pl_gA[2], pl_gB[2];
        auto frame = [&](auto generic_tag, int k) {
            constexpr bool GENERIC = decltype(generic_tag)::value;
            if ((k & 1) == 0) {
                const uint32_t la = lfo_acc + ch * lfo_inc, pa = ps_acc + ch * ps_inc;
                const float m_lfo = cos2pi(unit24(la + lfo_off));
                const float m_gA = cos2pi((unit24(pa) - 0.5f) * 0.5f);
                const float m_gB = cos2pi((unit24(pa + 0x80000000u) - 0.5f) * 0.5f);
                const float o_lfo = swap_pair(m_lfo), o_gA = swap_pair(m_gA), o_gB = swap_pair(m_gB);
                pl_lfo[0] = ch ? o_lfo : m_lfo; pl_lfo[1] = ch ? m_lfo : o_lfo;
                pl_gA[0] = ch ? o_gA : m_gA;    pl_gA[1] = ch ? m_gA : o_gA;
                pl_gB[0] = ch ? o_gB : m_gB;    pl_gB[1] = ch ? m_gB : o_gB;
            }
            if (GENERIC && k >= C) { psv[k] = 0.f; return; }
            const float lfo = pl_lfo[k & 1];
            const float dch = lfo * D + D;
            const float p0 = unit24(ps_acc);
            const float p1 = unit24(ps_acc + 0x80000000u);
            const float gA = pl_gA[k & 1];
            const float gB = pl_gB[k & 1];
            lfo_acc += lfo_inc;
            ps_acc += ps_inc;
            int di; float fr;
            float tA, tB;
            split_delay(p0 * W, 1.0f, pmax, di, fr);
            if (GENERIC && !cur.okA) {
                const uint32_t q = w0 + k - di;
                tA = lerp_pair(ld1(rP, own_pb + (q & pmask) * 8u, 0), ld1(rP, own_pb + ((q - 1u) & pmask) * 8u, 0), fr);
            } else {
                const int jw = k - di - cur.sA;
                tA = lerp_pair(wP0[jw * kRow], wP0[(jw - 1) * kRow], fr);
            }
            split_delay(p1 * W, 1.0f, pmax, di, fr);
            if (GENERIC && !cur.okB) {
                const uint32_t q = w0 + k - di;
                tB = lerp_pair(ld1(rP, own_pb + (q & pmask) * 8u, 0), ld1(rP, own_pb + ((q - 1u) & pmask) * 8u, 0), fr);
            } else {
                const int jw = k - di - cur.sB;
                tB = lerp_pair(wP1[jw * kRow], wP1[(jw - 1) * kRow], fr);
            }
            const float p = tB * gB + tA * gA;
            psv[k] = p;
            float out = p;
            if (FULL) {
                // delay~ writes before it reads: this frame's sample is visible at delay 0; slots
                // past the window land in the junk slot (no branch)
                wC[min(k - cur.sC, kWin) * kRow] = p;
                split_delay(dch, 0.0f, cmax, di, fr);
                const int jw = k - di - cur.sC;
                const float wet = lerp_pair(wC[jw * kRow], wC[(jw - 1) * kRow], fr);
                const float lp = b0 * wet + z1;
                z1 = (b1 * wet - a1 * lp) + z2;
                z2 = b2 * wet - a2 * lp;
                out = x[k] * dry + lp * mix;
            }
            sink(k, out);
        };
        if (C == kChunk && __all(cur.okA && cur.okB)) {
            // fast path in phases, with frame()'s per-frame arithmetic (bit-identical): the
            // pitch-shifter for all 16 frames (its reads all in flight together), its outputs
            // into the chorus window (a frame never reads a position newer than its own), then
            // the chorus tap + lores~ (see chorus_stage_l.h)
            const float Ws = W * 5.9604644775390625e-8f;
            float gA0 = 0.f, gA1 = 0.f, gB0 = 0.f, gB1 = 0.f;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                if ((k & 1) == 0) {
                    const uint32_t pa = ps_acc + ch * ps_inc;
                    const float m_gA = cos2pi_q((unit24(pa) - 0.5f) * 0.5f);
                    const float m_gB = cos2pi_q((unit24(pa + 0x80000000u) - 0.5f) * 0.5f);
                    gA0 = pair_even(m_gA); gA1 = pair_odd(m_gA);
                    gB0 = pair_even(m_gB); gB1 = pair_odd(m_gB);
                }
                const float d0 = (float)(ps_acc >> 8) * Ws;
                const float d1 = (float)((ps_acc + 0x80000000u) >> 8) * Ws;
                ps_acc += ps_inc;
                int di; float fr;
                split_delay3(d0, 1.0f, pmax, di, fr);
                int jw = k - di - cur.sA;
                const float tA = lerp_pair(wP0[jw * kRow], wP0[(jw - 1) * kRow], fr);
                split_delay3(d1, 1.0f, pmax, di, fr);
                jw = k - di - cur.sB;
                const float tB = lerp_pair(wP1[jw * kRow], wP1[(jw - 1) * kRow], fr);
                psv[k] = tB * ((k & 1) ? gB1 : gB0) + tA * ((k & 1) ? gA1 : gA0);
            }
            if (FULL) {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) wC[min(k - cur.sC, kWin) * kRow] = psv[k];
                float l0 = 0.f, l1 = 0.f;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    if ((k & 1) == 0) {
                        const float m_lfo = cos2pi(unit24(lfo_acc + ch * lfo_inc + lfo_off));
                        l0 = pair_even(m_lfo); l1 = pair_odd(m_lfo);
                    }
                    const float dch = ((k & 1) ? l1 : l0) * D + D;
                    lfo_acc += lfo_inc;
                    int di; float fr;
                    split_delay3(dch, 0.0f, cmax, di, fr);
                    const int jw = k - di - cur.sC;
                    const float wet = lerp_pair(wC[jw * kRow], wC[(jw - 1) * kRow], fr);
                    const float lp = b0 * wet + z1;
                    z1 = (b1 * wet - a1 * lp) + z2;
                    z2 = b2 * wet - a2 * lp;
                    sink(k, x[k] * dry + lp * mix);
                }
            } else {
                lfo_acc += (uint32_t)kChunk * lfo_inc;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) sink(k, psv[k]);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) frame(std::true_type{}, k);
        }
        if (FULL) {   // the chunk's windows are dead: stage its pitch-shifter outputs, store cooperatively
            stage_run(psv, kPsvBase);
            coop_store(false, kPsvBase, w0, C);
        }
        wpos = w0 + (uint32_t)C;
    }

    __device__ __forceinline__ void finish(const ChorusArgs &a) const {
        if (!valid) return;
        if (ch == 0) {
            a.state[CHS_LFO_ACC * n + i] = lfo_acc;
            a.state[CHS_PS_ACC * n + i] = ps_acc;
        }
        a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i] = __float_as_uint(z1);
        a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i] = __float_as_uint(z2);
    }
};

}  // namespace ch
}  // namespace olfx
