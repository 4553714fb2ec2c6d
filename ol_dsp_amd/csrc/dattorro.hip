// ol_dsp_amd/csrc/dattorro.hip -- Dattorro plate reverb kernel: one wavefront lane per instance.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
// The network, its ring layout and the chunked carry/prefetch scheme are in dattorro_stage.h.
//
// Pre-delay (verb.cpp:137-139: per instance, 0..4800 samples).  With one pre-delay for every
// instance (the common case, and SURVEY 8d's workload) the pre-delay ring is position-major like
// every other ring and its tap is one coalesced 16-B group per lane and chunk (PreTap).  With
// per-instance pre-delays, those groups lie in 64 different 128-B lines per wave instruction, and
// successive chunks of a lane touch one line eight times after it has left the caches: the gather
// read 8x its bytes (dattorro_rpd +30 %, round 3).  Gather mode (the engine switches when the
// pre-delays differ) keeps that ring instance-major, read and written in whole 128-B lines: inside
// the network's own launch (dattorro_block_v4f, round 5: one 32-frame piece ahead, through LDS) or,
// for audio rows that are not 16-B aligned, in dattorro_predelay_v2 ahead of it (its pre-delayed
// block as a coalesced stream, PreBlock).  Measured (65,536 instances, random pre-delays, same box):
// v4f 0.589 ms, the round-4 pre-pass + network 0.597, the uniform reverb 0.554 (1.063x).
#include <cstdlib>

#include "dattorro_stage.h"
#include "chorus_stage.h"
#include "lds_flags.h"

namespace olfx {

// Uniform mode: IN1 (the second input diffuser, 128 positions, verb.cpp:180) is read and written
// in LDS for the launch (LdsTap): its 8 B/frame of ring traffic become 512 B in and out per
// instance and launch (rocprof, same box: 571 -> 557 us).  Gather mode keeps IN1 in HBM: with the
// LDS ring its network measured 527 -> 554 us.
template <bool GATHER>
__global__ __launch_bounds__(64, 1) void dattorro_block_v4(DattorroArgs a) {
    __shared__ float4 in1_ring[GATHER ? 1u : kDtSize[DT_IN1] / 4u * 64u];      // 32 KB: [group][lane]
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;

    using Pre = typename std::conditional<GATHER, olfx::dt::PreBlock, olfx::dt::PreTap>::type;
    using In1 = typename std::conditional<GATHER, olfx::dt::Tap<DT_IN1, 107, 0>, olfx::dt::LdsTap<DT_IN1, 107>>::type;
    DT_STAGE_X(a, i, Pre, (In1));
    if constexpr (!GATHER) {
        in1.lds = in1_ring + threadIdx.x;
        in1.lds_in(a, i);
    }
    dt_prime(a.t0);

    // raw input frames are prefetched one chunk ahead like the taps (gather mode: no input here)
    float in_l[4] = {0.f, 0.f, 0.f, 0.f}, in_r[4] = {0.f, 0.f, 0.f, 0.f}, nx_l[4], nx_r[4];
    if (!GATHER) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            in_l[k] = a.in[(size_t)k * n + i];
            in_r[k] = stereo ? a.in[plane + (size_t)k * n + i] : 0.f;
        }
    }
    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        const bool has_next = f0 + 4 < a.n_frames;
        // this chunk's input: (l + r) / 2, ReverbFx.cpp:13-16
        float xin[4], o_l[4], o_r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xin[k] = stereo ? (in_l[k] + in_r[k]) / 2 : in_l[k];
        // next chunk's inputs, loaded unconditionally (clamped to the last frame in the last chunk)
        const uint32_t fn = has_next ? f0 + 4 : f0;
        if (!GATHER) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                nx_l[k] = a.in[(size_t)(fn + k) * n + i];
                nx_r[k] = stereo ? a.in[plane + (size_t)(fn + k) * n + i] : 0.f;
            }
        }
        dt_step(a.t0 + f0, has_next, xin, o_l, o_r);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a.out[(size_t)(f0 + k) * n + i] = o_l[k];
            a.out[plane + (size_t)(f0 + k) * n + i] = o_r[k];
        }
        if (!GATHER) {
#pragma unroll
            for (int k = 0; k < 4; ++k) { in_l[k] = nx_l[k]; in_r[k] = nx_r[k]; }
        }
    }
    dt_finish();
    if constexpr (!GATHER) in1.lds_out(a, i);
}

// ---------------------------------------------------------------------------------------------
// dattorro_block_v5: the network as three recurrences, one wave each (round 6).  Within a launch
// of at most kV5MaxFrames frames the network is three independent recurrences joined only by
// feed-forward values:
//   DI  (wave 0): pre-delay, pre-LPF and the 4 input all-passes (verb.cpp:273-282) -> x;
//   TA  (wave 1): tank half 0 (verb.cpp:284-295, i = 0): AP1A, DL1A, damping, AP2A, DL2A;
//   TB  (wave 2): tank half 1: AP1B, DL1B, damping, AP2B, DL2B.
// The halves exchange data only through postDampingDelay[1 - i]'s main tap (verb.cpp:286), 3163
// (TA reads DL2B) and 3720 (TB reads DL2A) samples back: within a launch shorter than that they
// read only what earlier launches wrote, and each wave reads back only rings it writes itself.  x
// goes to both halves through an LDS queue.  The stereo taps (verb.cpp:302-325) are split at
// their sum order: L = pL - oL5 - oL6 + oL7 with pL = oL1 + oL2 - oL3 + oL4 on half 1's rings and
// oL5..7 on half 0's; R the mirror image.  So half 1 sends pL to half 0, which finishes L, and
// half 0 sends pR to half 1, which finishes R (one float per frame each way, through LDS, one
// step late so neither waits on the other's current step) -- the reference's exact additions.
// Per 4-frame step: DI 5 taps, each half 11 taps (3 network + 1 modulated + 7 output) and 4
// ring writes, where v4's single wave carried all 27: a workgroup of 64 instances runs three
// waves (16,384 instances: 768 waves instead of 256), each with the register set of its own taps.
// ---------------------------------------------------------------------------------------------
namespace {
constexpr uint32_t kV5Depth = 4;          // LDS queue slots (4-frame steps) per hand-off
constexpr uint32_t kV5MaxFrames = 2048;   // < 3163 - queue skew: no cross-half read within a launch
enum { V5F_X = 0, V5F_XT0, V5F_XT1, V5F_P0, V5F_P1, V5F_PT0, V5F_PT1, V5F_N };
// V5F_X: steps of x published by DI; V5F_XT<h>: steps of x half h has taken; V5F_P<h>: partial
// sums half h has published; V5F_PT<h>: half h's partials the other half has taken

// The taps of tank half H.  P1..P4: the partial sum this half sends (half 0: pR = oR1 + oR2 -
// oR3 + oR4 on DL1A, DL1A, AP2A, DL2A; half 1: pL = oL1 + oL2 - oL3 + oL4 on DL1B, DL1B, AP2B,
// DL2B); T5..T7: the terms that finish the other half's sum into this half's channel (half 0,
// L: oL5 DL1A, oL6 AP2A, oL7 DL2A; half 1, R: oR5 DL1B, oR6 AP2B, oR7 DL2B).
template <int H> struct V5Half;
template <> struct V5Half<0> {
    static constexpr int kAP1 = DT_AP1A, kDL1 = DT_DL1A, kAP2 = DT_AP2A, kDL2 = DT_DL2A, kLp = DTS_LP_DAMP_A;
    using FB = olfx::dt::Tap<DT_DL2B, 3163, 0>;
    using DL1 = olfx::dt::Tap<DT_DL1A, 4453, 0>;
    using AP2 = olfx::dt::Tap<DT_AP2A, 1800, 0>;
    using AP1 = olfx::dt::ModTap<DT_AP1A, kDtDelay[DT_AP1A]>;
    using P1 = olfx::dt::Tap<DT_DL1A, kDl1A_o1, 1>;
    using P2 = olfx::dt::Tap<DT_DL1A, kDl1A_o2, 1>;
    using P3 = olfx::dt::Tap<DT_AP2A, kAp2A_o2, 1>;
    using P4 = olfx::dt::Tap<DT_DL2A, kDl2A_o2, 1>;
    using T5 = olfx::dt::Tap<DT_DL1A, kDl1A_o3, 1>;
    using T6 = olfx::dt::Tap<DT_AP2A, kAp2A_o1, 1>;
    using T7 = olfx::dt::Tap<DT_DL2A, kDl2A_o1, 1>;
};
template <> struct V5Half<1> {
    static constexpr int kAP1 = DT_AP1B, kDL1 = DT_DL1B, kAP2 = DT_AP2B, kDL2 = DT_DL2B, kLp = DTS_LP_DAMP_B;
    using FB = olfx::dt::Tap<DT_DL2A, 3720, 0>;
    using DL1 = olfx::dt::Tap<DT_DL1B, 4217, 0>;
    using AP2 = olfx::dt::Tap<DT_AP2B, 2656, 0>;
    using AP1 = olfx::dt::ModTap<DT_AP1B, kDtDelay[DT_AP1B]>;
    using P1 = olfx::dt::Tap<DT_DL1B, kDl1B_o1, 1>;
    using P2 = olfx::dt::Tap<DT_DL1B, kDl1B_o2, 1>;
    using P3 = olfx::dt::Tap<DT_AP2B, kAp2B_o2, 1>;
    using P4 = olfx::dt::Tap<DT_DL2B, kDl2B_o2, 1>;
    using T5 = olfx::dt::Tap<DT_DL1B, kDl1B_o3, 1>;
    using T6 = olfx::dt::Tap<DT_AP2B, kAp2B_o1, 1>;
    using T7 = olfx::dt::Tap<DT_DL2B, kDl2B_o1, 1>;
};

__device__ __forceinline__ float4 f4(const float (&v)[4]) { return make_float4(v[0], v[1], v[2], v[3]); }

// one tank half over the launch: x from qx, its partial to qmine, the other's from qother
template <int H>
__device__ __forceinline__ void v5_tank(const DattorroArgs &a, uint32_t i, uint32_t lane, bool live, uint32_t steps,
                                        const float4 *qx, float4 *qmine, const float4 *qother, uint32_t *flags) {
    using Hf = V5Half<H>;
    const uint32_t n = a.n, t0 = a.t0;
    const float g_dd1 = a.coef[DTC_DD1 * n + i];
    const float g_damp = a.coef[DTC_DAMPING * n + i];
    const float g_decay = a.coef[DTC_DECAY * n + i];
    const float g_dd2 = a.coef[DTC_DD2 * n + i];
    float lp = a.state[Hf::kLp * n + i];
    typename Hf::FB fb; typename Hf::DL1 dl1; typename Hf::AP2 ap2; typename Hf::AP1 ap1;
    typename Hf::P1 p1; typename Hf::P2 p2; typename Hf::P3 p3; typename Hf::P4 p4;
    typename Hf::T5 t5; typename Hf::T6 t6; typename Hf::T7 t7;
#define V5_TAPS(OP) OP(fb) OP(dl1) OP(ap2) OP(p1) OP(p2) OP(p3) OP(p4) OP(t5) OP(t6) OP(t7)
#define V5_PRIME(T) T.prime(a, t0, i);
#define V5_PREFETCH(T) T.prefetch(a, t, i);
#define V5_ADVANCE(T) T.advance();
    V5_TAPS(V5_PRIME)
    ap1.prime(a, t0, i);
    float* const out = a.out + (H ? a.plane : 0);
    float q5[4], q6[4], q7[4];                        // the previous step's finishing terms
    auto finish = [&](uint32_t s) {                   // channel H of step s: the other half's partial + q5..q7
        const uint32_t slot = s % kV5Depth;
        wait_for([&] { return flag_get(flags + V5F_P0 + (1 - H)) > s; });
        const float4 po = qother[slot * 64u + lane];
        flag_put(flags + V5F_PT0 + (1 - H), s + 1);
        const float pv[4] = {po.x, po.y, po.z, po.w};
        if (live) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float o = pv[k];
                o -= q5[k]; o -= q6[k]; o += q7[k];
                out[(size_t)(4u * s + (uint32_t)k) * n + i] = o;
            }
        }
    };
    for (uint32_t s = 0; s < steps; ++s) {
        const uint32_t t = t0 + 4u * s, slot = s % kV5Depth;
        V5_TAPS(V5_PREFETCH)
        ap1.prefetch(a, t, i);
        ap1.resolve();
        wait_for([&] { return flag_get(flags + V5F_X) > s; });
        const float4 xv = qx[slot * 64u + lane];
        flag_put(flags + V5F_XT0 + H, s + 1);
        const float x[4] = {xv.x, xv.y, xv.z, xv.w};
        float w_ap1[4], w_dl1[4], w_ap2[4], w_dl2[4], pm[4], n5[4], n6[4], n7[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {                 // verb.cpp:286-294; the APF gain is -dd1
            float y = x[k] + fb.get(k) * g_decay;
            float d = ap1.v[k];
            y += d * g_dd1; w_ap1[k] = y; y = d + y * -g_dd1;
            w_dl1[k] = y;
            lp += (dl1.get(k) - lp) * g_damp;
            y = lp * g_decay;
            d = ap2.get(k);
            y += d * -g_dd2; w_ap2[k] = y; y = d + y * g_dd2;
            w_dl2[k] = y;
            float p = p1.get(k);
            p += p2.get(k); p -= p3.get(k); p += p4.get(k);
            pm[k] = p;
            n5[k] = t5.get(k); n6[k] = t6.get(k); n7[k] = t7.get(k);
        }
        const uint32_t gw = t >> 2;
        *olfx::dt::grpu<Hf::kAP1>(a, gw, i) = f4(w_ap1);
        *olfx::dt::grpu<Hf::kDL1>(a, gw, i) = f4(w_dl1);
        *olfx::dt::grpu<Hf::kAP2>(a, gw, i) = f4(w_ap2);
        *olfx::dt::grpu<Hf::kDL2>(a, gw, i) = f4(w_dl2);
        // this step's partial out, then the previous step's channel
        wait_for([&] { return flag_get(flags + V5F_PT0 + H) + kV5Depth > s; });
        qmine[slot * 64u + lane] = f4(pm);
        flag_put(flags + V5F_P0 + H, s + 1);
        if (s > 0) finish(s - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) { q5[k] = n5[k]; q6[k] = n6[k]; q7[k] = n7[k]; }
        V5_TAPS(V5_ADVANCE)
        ap1.advance();
    }
    if (steps) finish(steps - 1);
    if (live) a.state[Hf::kLp * n + i] = lp;
#undef V5_TAPS
#undef V5_PRIME
#undef V5_PREFETCH
#undef V5_ADVANCE
}
}  // namespace

__global__ __launch_bounds__(192) void dattorro_block_v5(DattorroArgs a) {
    __shared__ float4 in1_ring[kDtSize[DT_IN1] / 4u * 64u];     // DI's IN1 ring (32 KB), as v4
    __shared__ float4 qx[kV5Depth * 64u], q0[kV5Depth * 64u], q1[kV5Depth * 64u];
    __shared__ uint32_t flags[V5F_N];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t role = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t n = a.n;
    const uint32_t i0 = blockIdx.x * 64u + lane;
    const bool live = i0 < n;
    const uint32_t i = live ? i0 : n - 1u;             // dead lanes mirror instance n - 1 (same bits)
    if (tid < V5F_N) flags[tid] = 0;
    __syncthreads();
    const uint32_t steps = a.n_frames / 4u;
    if (role == 1) {
        v5_tank<0>(a, i, lane, live, steps, qx, q0, q1, flags);
        return;
    }
    if (role == 2) {
        v5_tank<1>(a, i, lane, live, steps, qx, q1, q0, flags);
        return;
    }
    // ---- DI: input (l + r) / 2 (ReverbFx.cpp:13-16), pre-delay, pre-LPF, 4 input all-passes ----
    const uint32_t t0 = a.t0;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;
    const float g_pre = a.coef[DTC_PREFILTER * n + i];
    const float g_in1 = a.coef[DTC_IN1 * n + i];
    const float g_in2 = a.coef[DTC_IN2 * n + i];
    const uint32_t dpre = (uint32_t)a.coef[DTC_PREDELAY * n + i];
    float lp_pre = a.state[DTS_LP_PRE * n + i];
    olfx::dt::Tap<DT_IN0, 142, 0> in0;
    olfx::dt::LdsTap<DT_IN1, 107> in1;
    olfx::dt::Tap<DT_IN2, 379, 0> in2;
    olfx::dt::Tap<DT_IN3, 277, 0> in3;
    olfx::dt::PreTap pre;
    in1.lds = in1_ring + lane;
    in1.lds_in(a, i);
    in0.prime(a, t0, i); in1.prime(a, t0, i); in2.prime(a, t0, i); in3.prime(a, t0, i);
    pre.prime(a, t0, dpre, i);
    float in_l[4], in_r[4], nx_l[4], nx_r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        in_l[k] = a.in[(size_t)k * n + i];
        in_r[k] = stereo ? a.in[plane + (size_t)k * n + i] : 0.f;
    }
    for (uint32_t s = 0; s < steps; ++s) {
        const uint32_t t = t0 + 4u * s, slot = s % kV5Depth;
        const uint32_t fn = s + 1 < steps ? 4u * s + 4u : 4u * s;   // next inputs, clamped
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            nx_l[k] = a.in[(size_t)(fn + k) * n + i];
            nx_r[k] = stereo ? a.in[plane + (size_t)(fn + k) * n + i] : 0.f;
        }
        in0.prefetch(a, t, i); in1.prefetch(a, t, i); in2.prefetch(a, t, i); in3.prefetch(a, t, i);
        pre.prefetch(a, t, dpre, i);
        float xin[4], xpd[4], w0[4], w1[4], w2[4], w3[4], xo[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xin[k] = stereo ? (in_l[k] + in_r[k]) / 2 : in_l[k];
        pre.resolve(xin, dpre, xpd);
#pragma unroll
        for (int k = 0; k < 4; ++k) {                 // verb.cpp:273-282
            lp_pre += (xpd[k] - lp_pre) * g_pre;
            float x = lp_pre;
            float d = in0.get(k);
            x += d * -g_in1; w0[k] = x; x = d + x * g_in1;
            d = in1.get(k);
            x += d * -g_in1; w1[k] = x; x = d + x * g_in1;
            d = in2.get(k);
            x += d * -g_in2; w2[k] = x; x = d + x * g_in2;
            d = in3.get(k);
            x += d * -g_in2; w3[k] = x; x = d + x * g_in2;
            xo[k] = x;
        }
        const uint32_t gw = t >> 2;
        pre.write(a, gw, i, xin);
        *olfx::dt::grpu<DT_IN0>(a, gw, i) = f4(w0);
        in1.write(a, gw, i, f4(w1));
        *olfx::dt::grpu<DT_IN2>(a, gw, i) = f4(w2);
        *olfx::dt::grpu<DT_IN3>(a, gw, i) = f4(w3);
        wait_for([&] {
            return flag_get(flags + V5F_XT0) + kV5Depth > s && flag_get(flags + V5F_XT1) + kV5Depth > s;
        });
        qx[slot * 64u + lane] = f4(xo);
        flag_put(flags + V5F_X, s + 1);
        in0.advance(); in1.advance(); in2.advance(); in3.advance();
        pre.advance(xin);
#pragma unroll
        for (int k = 0; k < 4; ++k) { in_l[k] = nx_l[k]; in_r[k] = nx_r[k]; }
    }
    if (live) a.state[DTS_LP_PRE * n + i] = lp_pre;
    in1.lds_out(a, i);
}

constexpr uint32_t kPreSize = kDtSize[DT_PRE];

// dattorro_predelay_v2: gather mode's pre-pass in whole 128-B lines (round 4's first form, one lane
// per instance in 4-frame chunks moving 16-B pieces -- 64 lines per instruction, each line touched
// by 8 chunks -- made the mode 0.78 ms against 0.54 uniform and is gone).  One wave per workgroup = 64 instances,
// 32-frame chunks aligned to the ring's lines (chunk positions [T, T + 32), T % 32 == 0):
//   - a chunk's ring write is exactly one line per instance, stored cooperatively (8 lanes x 16 B
//     per line, 8 lines per instruction) from the LDS history `hist`;
//   - its pre-delayed reads [T - d, T - d + 32) lie in two lines Lq = (T - d) / 32 and Lq + 1; the
//     window `win` holds both in LDS, and each chunk loads only the next one (Lq + 2, cooperatively,
//     one chunk ahead), since the window advances by exactly one line per chunk;
//   - positions >= T - 32 (d <= k + 32) come from `hist`, which holds the previous chunk's and this
//     chunk's inputs.  The line prefetched during chunk c was issued before chunk c's ring store:
//     every earlier chunk's store precedes it, so its only possibly stale positions are chunk c's
//     own line [T, T + 32) -- when it is that line, hist's copy replaces it.
// Frames outside [t0, t0 + n_frames) in the first and last chunks are neither stored nor output;
// the first chunk's history positions [T, t0) and [T - 32, T) are loaded into `hist` from the ring.
// The pre-delayed block goes out as [F/4][n][4] (coalesced).
namespace {
constexpr uint32_t kPdLine = 32;                   // positions per 128-B line
constexpr uint32_t kPdLines = kPreSize / kPdLine;   // 256
constexpr uint32_t kPdRow = 65;                    // LDS floats per instance row (odd: lanes spread over banks)
}

__global__ __launch_bounds__(64) void dattorro_predelay_v2(DattorroArgs a) {
    __shared__ float hist[64 * kPdRow];            // [instance][P & 63]: inputs of positions [T - 32, T + 32)
    __shared__ float win[64 * kPdRow];             // [instance][P & 63]: ring lines Lq, Lq + 1
    const uint32_t lane = threadIdx.x, n = a.n, F = a.n_frames, t0 = a.t0;
    const uint32_t i0 = blockIdx.x * 64u, i = i0 + lane, nv = min(n - i0, 64u);
    const bool live = i < n;
    const bool stereo = a.in_ch == 2;
    const uint32_t d = (uint32_t)a.coef[DTC_PREDELAY * n + min(i, n - 1u)];
    // cooperative line accesses: in instruction m, lane L serves instance 8 m + L / 8, piece L % 8
    const uint32_t pc = lane & 7u;
    uint32_t dj[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) dj[m] = (uint32_t)a.coef[DTC_PREDELAY * n + min(i0 + 8u * m + (lane >> 3), n - 1u)];
    const ch::Rsrc rRing = ch::rsrc(a.pre_im + (size_t)i0 * kPreSize, (uint64_t)nv * kPreSize * 4u);
    auto line_off = [&](int m, uint32_t line) {    // byte offset of piece pc of instance 8 m + L / 8's line
        const uint32_t j = 8u * (uint32_t)m + (lane >> 3);
        return j < nv ? j * kPreSize * 4u + (line & (kPdLines - 1u)) * 128u + pc * 16u : 0xFFFFFFF0u;
    };
    auto to_lds = [&](float *dst, int m, uint32_t line, float4 v) {   // piece -> row slot (line & 1) * 32 + 4 pc
        float *r = dst + (8u * (uint32_t)m + (lane >> 3)) * kPdRow + (line & 1u) * kPdLine + 4u * pc;
        r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // input frame rows: f = T + k - t0, loaded when 0 <= f < F (else 0 through an out-of-range offset)
    const ch::Rsrc rIn0 = ch::rsrc(a.in, ((uint64_t)F * n) * 4u);
    const ch::Rsrc rIn1 = ch::rsrc(stereo ? a.in + a.plane : a.in, ((uint64_t)F * n) * 4u);
    auto load_x = [&](uint32_t T, float (&x0)[kPdLine], float (&x1)[kPdLine]) {
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const uint32_t f = T + k - t0;                 // wraps above F when T + k < t0
            const uint32_t off = f < F && live ? (f * n + i) * 4u : 0xFFFFFFF0u;
            x0[k] = ch::ld1(rIn0, off, 0);
            x1[k] = ch::ld1(rIn1, off, 0);
        }
    };
    const uint32_t T0 = t0 & ~(kPdLine - 1u);
    const uint32_t nch = (t0 + F - T0 + kPdLine - 1u) / kPdLine;
    // history lines T0 / 32 - 1 and T0 / 32, window lines Lq and Lq + 1 of the first chunk
    {
        float4 h[2][8], w[2][8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            h[0][m] = ch::ld4(rRing, line_off(m, T0 / kPdLine - 1u));
            h[1][m] = ch::ld4(rRing, line_off(m, T0 / kPdLine));
            w[0][m] = ch::ld4(rRing, line_off(m, (T0 - dj[m]) / kPdLine));
            w[1][m] = ch::ld4(rRing, line_off(m, (T0 - dj[m]) / kPdLine + 1u));
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            to_lds(hist, m, T0 / kPdLine - 1u, h[0][m]);
            to_lds(hist, m, T0 / kPdLine, h[1][m]);
            to_lds(win, m, (T0 - dj[m]) / kPdLine, w[0][m]);
            to_lds(win, m, (T0 - dj[m]) / kPdLine + 1u, w[1][m]);
        }
    }
    float x0[kPdLine], x1[kPdLine];
    load_x(T0, x0, x1);
    const ch::Rsrc rBlk = ch::rsrc(a.pre_block, (uint64_t)F * n * 4u);
    float *hrow = hist + lane * kPdRow, *wrow = win + lane * kPdRow;
    for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t T = T0 + c * kPdLine;
        // the next chunk's window line and inputs, issued before this chunk's ring store
        float4 nl[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) nl[m] = ch::ld4(rRing, line_off(m, (T - dj[m]) / kPdLine + 2u));
        float n0[kPdLine], n1[kPdLine];
        load_x(T + kPdLine, n0, n1);
        // this chunk's mono input (l + r) / 2 into the history (positions before t0 keep the ring's)
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const float xm = stereo ? (x0[k] + x1[k]) / 2 : x0[k];
            if (T + k - t0 < F) hrow[(T + k) & 63u] = xm;
        }
        wave_sync();
        // the pre-delayed samples: positions T + k - d, from the history when >= T - 32
        float v[kPdLine];
        const uint32_t q = T - d;
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const float *src = d <= k + kPdLine ? hrow + ((T + k - d) & 63u) : wrow + ((q + k) & 63u);
            v[k] = *src;
        }
#pragma unroll
        for (uint32_t g = 0; g < kPdLine / 4u; ++g) {
            const uint32_t f = T + 4u * g - t0;            // a group is wholly inside or outside (t0 % 4 == 0)
            ch::st4(rBlk, f < F && live ? ((f >> 2) * n + i) * 16u : 0xFFFFFFF0u,
                make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]));
        }
        // the chunk's ring line, cooperatively from the history (pieces outside the block dropped)
        float4 hv[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const float *r = hist + (8u * (uint32_t)m + (lane >> 3)) * kPdRow + (T & 63u) + 4u * pc;
            hv[m] = make_float4(r[0], r[1], r[2], r[3]);
            const uint32_t f = T + 4u * pc - t0;
            ch::st4(rRing, f < F ? line_off(m, T / kPdLine) : 0xFFFFFFF0u, hv[m]);
        }
        wave_sync();
        // the window advances one line: Lq + 2 replaces Lq (its reads are done); if Lq + 2 is this
        // chunk's own line, its prefetch predates the store above: hist's copy instead
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t l2 = (T - dj[m]) / kPdLine + 2u;
            to_lds(win, m, l2, ((l2 ^ (T / kPdLine)) & (kPdLines - 1u)) == 0u ? hv[m] : nl[m]);
        }
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) { x0[k] = n0[k]; x1[k] = n1[k]; }
        wave_sync();
    }
}

// dattorro_block_v4f: gather mode in ONE launch (round 5; VERDICT r4: the pre-pass round-tripped
// the pre-delayed block through HBM).  The network's own wave (64 instances) keeps the pre-delay
// path in LDS, one 32-frame piece ahead, with no serial dependence on the network:
//   M[2][64][36]: a piece's mono input (l + r) / 2, [instance][frame]: loaded as cooperative rows
//                 (2 dwordx4 per lane and chunk: 4 frames x 64 instances x 2 channels) during the
//                 piece before, transposed on the way into LDS; the network's xin comes from here;
//   W[2][64][36]: each instance's 36 ring positions from A = (T - d) & ~3 (its pre-delayed samples
//                 of the piece, T = the piece's first position), loaded cooperatively (8 instances x
//                 128 B per instruction, one per chunk, and the 36th-position group) during the
//                 piece before.
// At its first chunk a piece writes its own input into the instance-major ring (8 cooperative
// 128-B stores, 8 instances each), so the window loads for the next piece, issued after, see every
// position before that piece; positions inside the piece itself (d <= f) are read from M
// (dt::PreFused).  A pre-delay up to 8191 reads positions the launch has not yet overwritten:
// ring slots are only written one piece at a time, at the piece's start, and a window load reads
// before the piece that would overwrite it, as DelayBuffer_process reads after its write only for
// d = 0 (verb.cpp:107-110).  Dead lanes of the last wave mirror instance n - 1 exactly (its input
// row, its window, its state), so their stores duplicate lane n - 1's.  Needs 16-B aligned input
// rows (n % 4 == 0, plane % 4 == 0, in 16-B aligned); dattorro_predelay_v2 + dattorro_block_v4<true>
// otherwise.  LDS 36 KB per wave: four waves per CU, as v4 (IN1 stays in HBM here).
namespace {
constexpr uint32_t kFuS = 36;                      // LDS row stride (floats): 16-B aligned rows
constexpr uint32_t kFuPiece = 32;                  // frames per piece
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
}  // namespace

__global__ __launch_bounds__(64, 1) void dattorro_block_v4f(DattorroArgs a) {
    __shared__ __attribute__((aligned(16))) float fM[2][64 * kFuS];
    __shared__ __attribute__((aligned(16))) float fW[2][64 * kFuS];
    const uint32_t lane = threadIdx.x, n = a.n, F = a.n_frames, t0 = a.t0;
    const uint32_t i0 = blockIdx.x * 64u;
    const uint32_t i = min(i0 + lane, n - 1u);            // dead lanes mirror instance n - 1
    const uint32_t jrow = i - i0;                          // the LDS row this lane computes on
    const bool stereo = a.in_ch == 2;
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    const ch::Rsrc rIn0 = ch::rsrc(a.in, (uint64_t)F * n * 4u);
    const ch::Rsrc rIn1 = ch::rsrc(stereo ? a.in + a.plane : a.in, (uint64_t)F * n * 4u);
    const uint32_t nv = min(n - i0, 64u);
    const ch::Rsrc rRing = ch::rsrc(a.pre_im + (size_t)i0 * kPreSize, (uint64_t)nv * kPreSize * 4u);

    using Tin1 = olfx::dt::Tap<DT_IN1, 107, 0>;
    DT_STAGE_X(a, i, olfx::dt::PreFused, (Tin1));
    dt_prime(t0);

    // cooperative geometry: input rows -- row r = lane / 16 (frame 4c + r), instances 4 (lane % 16)..;
    // ring lines -- instance 8 m + lane / 8, 16-B group lane % 8
    const uint32_t rq = lane & 15u, rr = lane >> 4, lj = lane >> 3, lg = lane & 7u;
    auto load_rows = [&](uint32_t f, float4 &l, float4 &r) {     // frame f of the block, 4 instances
        const uint32_t off = f < F && 4u * rq < nv ? (f * n + i0 + 4u * rq) * 4u : kOob;
        l = ch::ld4(rIn0, off);
        r = stereo ? ch::ld4(rIn1, off) : l;
    };
    auto put_rows = [&](float *M, uint32_t fp, const float4 &l, const float4 &r) {   // fp: frame in piece
        float *dst = M + 4u * rq * kFuS + fp;
        dst[0] = stereo ? (l.x + r.x) / 2 : l.x;
        dst[kFuS] = stereo ? (l.y + r.y) / 2 : l.y;
        dst[2 * kFuS] = stereo ? (l.z + r.z) / 2 : l.z;
        dst[3 * kFuS] = stereo ? (l.w + r.w) / 2 : l.w;
    };
    // window group of the piece starting at T: instance 8 m + lj, positions A + 4 lg (lg < 8), with d
    // of that instance from its own lane
    auto win_off = [&](uint32_t T, uint32_t j, uint32_t d, uint32_t g) {
        const uint32_t A = (T - d) & ~3u;
        return j < nv ? (j * kPreSize + ((A + 4u * g) & (kPreSize - 1u))) * 4u : kOob;
    };
    auto d_of = [&](uint32_t j) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(j << 2), (int)dpre); };
    // the piece starting at frame fp0 of the block: its window rows into W (all nine groups) and
    // its input rows into M -- the prologue's form of what each chunk does for the next piece
    auto fill_piece = [&](float *M, float *W, uint32_t fp0) {
        const uint32_t T = t0 + fp0;
#pragma unroll
        for (uint32_t m = 0; m < 8; ++m) {
            const uint32_t j = 8u * m + lj;
            const float4 v = ch::ld4(rRing, win_off(T, j, d_of(j), lg));
            *(float4 *)(W + j * kFuS + 4u * lg) = v;
        }
        const float4 v8 = ch::ld4(rRing, win_off(T, lane, d_of(lane), 8));
        *(float4 *)(W + lane * kFuS + 32u) = v8;
#pragma unroll
        for (uint32_t c = 0; c < 8; ++c) {
            float4 l, r;
            load_rows(fp0 + 4u * c + rr, l, r);
            put_rows(M, 4u * c + rr, l, r);
        }
    };
    fill_piece(fM[0], fW[0], 0);
    wave_sync();

    const uint32_t pieces = (F + kFuPiece - 1u) / kFuPiece;
    const ch::Rsrc rOut0 = ch::rsrc(a.out, (uint64_t)F * n * 4u);
    const ch::Rsrc rOut1 = ch::rsrc(a.out + a.plane, (uint64_t)F * n * 4u);
    const bool live = i0 + lane < n;
    for (uint32_t p = 0; p < pieces; ++p) {
        float *M = fM[p & 1u], *W = fW[p & 1u], *Mn = fM[(p + 1u) & 1u], *Wn = fW[(p + 1u) & 1u];
        const uint32_t fp0 = p * kFuPiece, T = t0 + fp0, Tn = T + kFuPiece;
        // 1. this piece's input into the instance-major ring (frames < F only), before any window
        //    load of the next piece
#pragma unroll
        for (uint32_t m = 0; m < 8; ++m) {
            const uint32_t j = 8u * m + lj;
            const float4 v = *(const float4 *)(M + j * kFuS + 4u * lg);
            const uint32_t off = j < nv && fp0 + 4u * lg < F ? (j * kPreSize + ((T + 4u * lg) & (kPreSize - 1u))) * 4u : kOob;
            ch::st4(rRing, off, v);
        }
        // the next piece's 36th-position group, after this piece's ring stores
        const bool more = fp0 + kFuPiece < F;
        const float4 w8 = ch::ld4(rRing, more ? win_off(Tn, lane, dpre, 8) : kOob);
        const uint32_t dfix = dpre, off0 = (T - dfix) & 3u;
        pre.m = M + jrow * kFuS;
        pre.w = W + jrow * kFuS;
        pre.off0 = off0;
#pragma unroll 1
        for (uint32_t c = 0; c < 8; ++c) {
            const uint32_t f0 = fp0 + 4u * c;
            if (f0 >= F) break;
            // 2. the next piece's loads: its frames 4c .. 4c + 3 (input rows) and window group m = c
            float4 nl, nr;
            load_rows(fp0 + kFuPiece + 4u * c + rr, nl, nr);
            const uint32_t jw = 8u * c + lj;
            const float4 nw = ch::ld4(rRing, more ? win_off(Tn, jw, d_of(jw), lg) : kOob);
            // 3. the chunk: xin from M, the pre-delayed samples from M / W (PreFused)
            const float4 xv = *(const float4 *)(pre.m + 4u * c);
            const float xin[4] = {xv.x, xv.y, xv.z, xv.w};
            pre.fc = (int)(4u * c);
            float o_l[4], o_r[4];
            dt_step(t0 + f0, f0 + 4u < F, xin, o_l, o_r);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t off = live ? ((f0 + (uint32_t)k) * n + i0 + lane) * 4u : kOob;
                ch::st1(rOut0, off, 0, o_l[k]);
                ch::st1(rOut1, off, 0, o_r[k]);
            }
            // 4. the next piece's rows into LDS (its buffers: nothing of this piece reads them)
            put_rows(Mn, 4u * c + rr, nl, nr);
            *(float4 *)(Wn + jw * kFuS + 4u * lg) = nw;
        }
        *(float4 *)(Wn + lane * kFuS + 32u) = w8;
        wave_sync();
    }
    if (i0 + lane < n) dt_finish();
}

// the pre-delay ring between layouts: position-major groups [size/4][n][4] <-> instance-major
// [n][size]; one thread per (group, instance), reads or writes coalesced on the position-major side
__global__ __launch_bounds__(256) void dattorro_pre_convert(DattorroArgs a, int to_im) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, g = blockIdx.y;
    if (i >= a.n) return;
    float4 *pm = (float4 *)a.ring[DT_PRE] + (size_t)g * a.n + i;
    float4 *im = (float4 *)(a.pre_im + (size_t)i * kPreSize) + g;
    if (to_im) *im = *pm;
    else *pm = *im;
}

// 3 = the fused dattorro_block_v4f when the rows allow it (16-B aligned input rows), else 2 =
// dattorro_predelay_v2 + dattorro_block_v4<true>
int predelay_kernel(uint32_t n, uint64_t plane, const float *in) {
    return n % 4u == 0u && plane % 4u == 0u && ((uintptr_t)in & 15u) == 0u ? 3 : 2;
}

// A/B knob while the split network is measured against v4 (OLFX_DT_V4=1: the single-wave network)
static bool dt_use_v4() {
    static const bool v4 = [] { const char *e = std::getenv("OLFX_DT_V4"); return e && e[0] == '1'; }();
    return v4;
}

const char *dattorro_uniform_kernel() { return dt_use_v4() ? "dattorro_block_v4" : "dattorro_block_v5"; }

hipError_t launch_dattorro(const DattorroArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.t0 & 3u) || (a.n_frames & 3u)) return hipErrorInvalidValue;   // 4-frame chunks
    // the modulated taps' buffer loads take 32-bit offsets into their (1024-position) rings
    if ((uint64_t)kDtSize[DT_AP1A] * a.n * 4u >= (1ull << 32) || (uint64_t)kDtSize[DT_AP1B] * a.n * 4u >= (1ull << 32))
        return hipErrorInvalidValue;
    const uint32_t threads = 64;      // one wave per workgroup: spreads small engines over all CUs
    const uint32_t blocks = (a.n + threads - 1) / threads;
    if (a.pre_im) {
        // per-workgroup ring resources: 64 instances x 32 KB; inputs and the block by 32-bit offsets
        if ((uint64_t)a.n_frames * a.n * 4u >= (1ull << 32)) return hipErrorInvalidValue;
        if (predelay_kernel(a.n, a.plane, a.in) == 3) {
            hipLaunchKernelGGL(dattorro_block_v4f, dim3(blocks), dim3(threads), 0, s, a);   // one launch
        } else {
            hipLaunchKernelGGL(dattorro_predelay_v2, dim3((a.n + 63) / 64), dim3(64), 0, s, a);
            hipLaunchKernelGGL(dattorro_block_v4<true>, dim3(blocks), dim3(threads), 0, s, a);
        }
    } else if (dt_use_v4()) {
        hipLaunchKernelGGL(dattorro_block_v4<false>, dim3(blocks), dim3(threads), 0, s, a);
    } else {
        // pieces of at most kV5MaxFrames (the halves' cross taps then read earlier launches only)
        for (uint32_t f0 = 0; f0 < a.n_frames; f0 += kV5MaxFrames) {
            DattorroArgs p = a;
            p.n_frames = min(kV5MaxFrames, a.n_frames - f0);
            p.t0 = (a.t0 + f0) & 0xFFFFu;
            p.in = a.in + (size_t)f0 * a.n;
            p.out = a.out + (size_t)f0 * a.n;
            hipLaunchKernelGGL(dattorro_block_v5, dim3(blocks), dim3(192), 0, s, p);
        }
    }
    return hipGetLastError();
}

hipError_t launch_dattorro_pre_convert(const DattorroArgs &a, bool to_im, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(dattorro_pre_convert, dim3((a.n + 255) / 256, kPreSize / 4), dim3(256), 0, s, a, to_im ? 1 : 0);
    return hipGetLastError();
}

}  // namespace olfx
