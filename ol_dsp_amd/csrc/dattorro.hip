// ol_dsp_amd/csrc/dattorro.hip -- Dattorro plate reverb, one wavefront lane per instance.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
//
// Layout: ring l is [kDtSize[l]/4][n][4] floats -- groups of 4 consecutive positions of one
// instance, instances fastest.  All instances of an engine share the stream time t and every tap
// delay, so a wave reading one tap for a 4-frame chunk issues ONE 16-B-per-lane load that covers
// 1 KB contiguous.  The block is processed in 4-frame chunks aligned to t % 4 == 0:
//   * a tap with delay d reads positions t0 - d + k (k = 0..3) = a window of 2 groups shifted by
//     s = (-d) & 3, a compile-time constant for the 24 fixed taps: each chunk loads ONE new group
//     per tap and carries the other from the previous chunk (every ring byte is read once);
//   * the group for the next chunk is prefetched before the current chunk's serial recurrence,
//     so ~30 x 1 KB loads per wave are in flight while it computes (1 wave per SIMD at 65,536
//     instances; latency hiding comes from this ILP, not occupancy);
//   * the 13 ring writes of a chunk leave as one 16-B store per line.
// Every fixed delay is >= 107 samples, so no chunk reads a group written by itself or by its
// predecessor.  The pre-delay is per instance (0..4800 samples, verb.cpp:137-139): its tap loads
// the two groups around t0 - d of the lane's own ring (one 16-B load each; coalesced whenever the
// wave's instances share d) and takes frames of the current chunk (d < 4) from registers.  Groups
// written by earlier chunks of this launch are read back by the same lane, in program order.
// No MFMA: scalar recurrences.
// Bound: HBM.
#include "olfx_internal.h"

namespace olfx {

namespace {

__device__ __forceinline__ float el(const float4 &v, int e) {
    return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

template <int L>
__device__ __forceinline__ float4 *grp(const DattorroArgs &a, uint32_t g, uint32_t i) {
    constexpr uint32_t gm = kDtSize[L] / 4u - 1u;
    return (float4 *)a.ring[L] + ((size_t)(g & gm) * a.n + i);
}

// A fixed tap: delay D, read at t + OFF (OFF = 1 for the output taps, verb.cpp:298,302-325).
template <int L, uint32_t D, uint32_t OFF>
struct Tap {
    static constexpr uint32_t S = (OFF - D) & 3u;     // shift of the window inside its groups
    float4 cur, nxt, pre;
    __device__ __forceinline__ static uint32_t g0(uint32_t t0) { return (t0 + OFF - D) >> 2; }
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        cur = *grp<L>(a, g0(t0), i);
        if (S) nxt = *grp<L>(a, g0(t0) + 1u, i);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        pre = *grp<L>(a, g0(t0) + (S ? 2u : 1u), i);
    }
    __device__ __forceinline__ float get(int k) const {
        return (int)S + k < 4 ? el(cur, (int)S + k) : el(nxt, (int)S + k - 4);
    }
    __device__ __forceinline__ void advance() {
        if (S) { cur = nxt; nxt = pre; } else { cur = pre; }
    }
};

// A tap whose delay changes at run time (the modulated tank all-passes, the pre-delay ring):
// both groups are loaded for each chunk (uniform shift chosen with a scalar branch).
template <int L>
struct VarTap {
    float4 a0, a1;
    float v[4];
    __device__ __forceinline__ void load(const DattorroArgs &a, uint32_t q, uint32_t i) {
        a0 = *grp<L>(a, q >> 2, i);
        a1 = *grp<L>(a, (q >> 2) + 1u, i);
    }
    __device__ __forceinline__ void resolve(uint32_t s) {        // s wave-uniform: scalar branch
        switch (s) {
        case 0: v[0] = a0.x; v[1] = a0.y; v[2] = a0.z; v[3] = a0.w; break;
        case 1: v[0] = a0.y; v[1] = a0.z; v[2] = a0.w; v[3] = a1.x; break;
        case 2: v[0] = a0.z; v[1] = a0.w; v[2] = a1.x; v[3] = a1.y; break;
        default: v[0] = a0.w; v[1] = a1.x; v[2] = a1.y; v[3] = a1.z; break;
        }
    }
    __device__ __forceinline__ void resolve_lane(uint32_t s) {   // s per lane: selects
        const float w[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = s == 0 ? w[k] : (s == 1 ? w[k + 1] : (s == 2 ? w[k + 2] : w[k + 3]));
    }
};

}  // namespace

__global__ __launch_bounds__(64, 1) void dattorro_block_v2(DattorroArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;

    const float g_pre = a.coef[DTC_PREFILTER * n + i];
    const float g_in1 = a.coef[DTC_IN1 * n + i];
    const float g_in2 = a.coef[DTC_IN2 * n + i];
    const float g_dd1 = a.coef[DTC_DD1 * n + i];
    const float g_damp = a.coef[DTC_DAMPING * n + i];
    const float g_decay = a.coef[DTC_DECAY * n + i];
    const float g_dd2 = a.coef[DTC_DD2 * n + i];
    const uint32_t dpre = (uint32_t)a.coef[DTC_PREDELAY * n + i];   // samples, exact integer
    float lp_pre = a.state[DTS_LP_PRE * n + i];
    float lp_a = a.state[DTS_LP_DAMP_A * n + i];
    float lp_b = a.state[DTS_LP_DAMP_B * n + i];

    const size_t plane = (size_t)a.n_frames * n;
    const bool stereo = a.in_ch == 2;

    // main-time taps (read at t)
    Tap<DT_IN0, 142, 0> in0; Tap<DT_IN1, 107, 0> in1; Tap<DT_IN2, 379, 0> in2; Tap<DT_IN3, 277, 0> in3;
    Tap<DT_DL2B, 3163, 0> fbA; Tap<DT_DL2A, 3720, 0> fbB;
    Tap<DT_DL1A, 4453, 0> dl1a; Tap<DT_DL1B, 4217, 0> dl1b;
    Tap<DT_AP2A, 1800, 0> ap2a; Tap<DT_AP2B, 2656, 0> ap2b;
    // output taps (read at t + 1)
    Tap<DT_DL1B, kDl1B_o1, 1> oL1; Tap<DT_DL1B, kDl1B_o2, 1> oL2; Tap<DT_AP2B, kAp2B_o2, 1> oL3;
    Tap<DT_DL2B, kDl2B_o2, 1> oL4; Tap<DT_DL1A, kDl1A_o3, 1> oL5; Tap<DT_AP2A, kAp2A_o1, 1> oL6;
    Tap<DT_DL2A, kDl2A_o1, 1> oL7;
    Tap<DT_DL1A, kDl1A_o1, 1> oR1; Tap<DT_DL1A, kDl1A_o2, 1> oR2; Tap<DT_AP2A, kAp2A_o2, 1> oR3;
    Tap<DT_DL2A, kDl2A_o2, 1> oR4; Tap<DT_DL1B, kDl1B_o3, 1> oR5; Tap<DT_AP2B, kAp2B_o1, 1> oR6;
    Tap<DT_DL2B, kDl2B_o1, 1> oR7;
    VarTap<DT_AP1A> ap1a; VarTap<DT_AP1B> ap1b; VarTap<DT_PRE> pre;

#define DT_ALL_TAPS(OP) OP(in0) OP(in1) OP(in2) OP(in3) OP(fbA) OP(fbB) OP(dl1a) OP(dl1b) OP(ap2a) OP(ap2b) \
    OP(oL1) OP(oL2) OP(oL3) OP(oL4) OP(oL5) OP(oL6) OP(oL7) OP(oR1) OP(oR2) OP(oR3) OP(oR4) OP(oR5) OP(oR6) OP(oR7)
#define DT_PRIME(T) T.prime(a, a.t0, i);
#define DT_PREFETCH(T) T.prefetch(a, t0, i);
#define DT_ADVANCE(T) T.advance();

    DT_ALL_TAPS(DT_PRIME)

    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        const uint32_t t0 = a.t0 + f0;                 // multiple of 4
        const uint32_t t16 = t0 & 0xFFFFu;

        // ---- this chunk's variable taps and inputs ----
        const uint32_t ex = dt_ap1_extra(t16);         // constant over the chunk (changes at 2048k)
        const uint32_t qa = t0 - (kDtDelay[DT_AP1A] + ex), qb = t0 - (kDtDelay[DT_AP1B] + ex);
        ap1a.load(a, qa, i);
        ap1b.load(a, qb, i);
        const uint32_t qp = t0 - dpre;
        pre.load(a, qp, i);                            // groups of earlier chunks (or stale: see below)
        float xin[4], xpd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float l = a.in[(size_t)(f0 + k) * n + i];
            if (stereo) l = (l + a.in[plane + (size_t)(f0 + k) * n + i]) / 2;
            xin[k] = l;
        }
        // ---- prefetch the fixed taps' next group (consumed by the next chunk) ----
        if (f0 + 4 < a.n_frames) { DT_ALL_TAPS(DT_PREFETCH) }

        ap1a.resolve(qa & 3u);
        ap1b.resolve(qb & 3u);
        pre.resolve_lane(qp & 3u);
#pragma unroll
        for (int k = 0; k < 4; ++k) {                  // frame t0+k-d lies in this chunk when d <= k
            float v = pre.v[k];
#pragma unroll
            for (int j = 0; j <= k; ++j) v = dpre == (uint32_t)(k - j) ? xin[j] : v;
            xpd[k] = v;
        }

        // ---- the serial recurrence, 4 frames (verb.cpp:273-299, 302-325) ----
        float w_in0[4], w_in1[4], w_in2[4], w_in3[4], w_ap1a[4], w_dl1a[4], w_ap2a[4], w_dl2a[4];
        float w_ap1b[4], w_dl1b[4], w_ap2b[4], w_dl2b[4], o_l[4], o_r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            lp_pre += (xpd[k] - lp_pre) * g_pre;
            float x = lp_pre;
            float d = in0.get(k);
            x += d * -g_in1; w_in0[k] = x; x = d + x * g_in1;
            d = in1.get(k);
            x += d * -g_in1; w_in1[k] = x; x = d + x * g_in1;
            d = in2.get(k);
            x += d * -g_in2; w_in2[k] = x; x = d + x * g_in2;
            d = in3.get(k);
            x += d * -g_in2; w_in3[k] = x; x = d + x * g_in2;
            {   // tank half A; the APF gain is -dd1, so in += delayed * dd1
                float y = x + fbA.get(k) * g_decay;
                d = ap1a.v[k];
                y += d * g_dd1; w_ap1a[k] = y; y = d + y * -g_dd1;
                w_dl1a[k] = y;
                lp_a += (dl1a.get(k) - lp_a) * g_damp;
                y = lp_a * g_decay;
                d = ap2a.get(k);
                y += d * -g_dd2; w_ap2a[k] = y; y = d + y * g_dd2;
                w_dl2a[k] = y;
            }
            {   // tank half B
                float y = x + fbB.get(k) * g_decay;
                d = ap1b.v[k];
                y += d * g_dd1; w_ap1b[k] = y; y = d + y * -g_dd1;
                w_dl1b[k] = y;
                lp_b += (dl1b.get(k) - lp_b) * g_damp;
                y = lp_b * g_decay;
                d = ap2b.get(k);
                y += d * -g_dd2; w_ap2b[k] = y; y = d + y * g_dd2;
                w_dl2b[k] = y;
            }
            float l = oL1.get(k);
            l += oL2.get(k); l -= oL3.get(k); l += oL4.get(k); l -= oL5.get(k); l -= oL6.get(k); l += oL7.get(k);
            float r = oR1.get(k);
            r += oR2.get(k); r -= oR3.get(k); r += oR4.get(k); r -= oR5.get(k); r -= oR6.get(k); r += oR7.get(k);
            o_l[k] = l;
            o_r[k] = r;
        }

        // ---- writes: one 16-B group per line, then the output frames ----
        const uint32_t gw = t0 >> 2;
        *grp<DT_PRE>(a, gw, i) = make_float4(xin[0], xin[1], xin[2], xin[3]);
        *grp<DT_IN0>(a, gw, i) = make_float4(w_in0[0], w_in0[1], w_in0[2], w_in0[3]);
        *grp<DT_IN1>(a, gw, i) = make_float4(w_in1[0], w_in1[1], w_in1[2], w_in1[3]);
        *grp<DT_IN2>(a, gw, i) = make_float4(w_in2[0], w_in2[1], w_in2[2], w_in2[3]);
        *grp<DT_IN3>(a, gw, i) = make_float4(w_in3[0], w_in3[1], w_in3[2], w_in3[3]);
        *grp<DT_AP1A>(a, gw, i) = make_float4(w_ap1a[0], w_ap1a[1], w_ap1a[2], w_ap1a[3]);
        *grp<DT_DL1A>(a, gw, i) = make_float4(w_dl1a[0], w_dl1a[1], w_dl1a[2], w_dl1a[3]);
        *grp<DT_AP2A>(a, gw, i) = make_float4(w_ap2a[0], w_ap2a[1], w_ap2a[2], w_ap2a[3]);
        *grp<DT_DL2A>(a, gw, i) = make_float4(w_dl2a[0], w_dl2a[1], w_dl2a[2], w_dl2a[3]);
        *grp<DT_AP1B>(a, gw, i) = make_float4(w_ap1b[0], w_ap1b[1], w_ap1b[2], w_ap1b[3]);
        *grp<DT_DL1B>(a, gw, i) = make_float4(w_dl1b[0], w_dl1b[1], w_dl1b[2], w_dl1b[3]);
        *grp<DT_AP2B>(a, gw, i) = make_float4(w_ap2b[0], w_ap2b[1], w_ap2b[2], w_ap2b[3]);
        *grp<DT_DL2B>(a, gw, i) = make_float4(w_dl2b[0], w_dl2b[1], w_dl2b[2], w_dl2b[3]);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a.out[(size_t)(f0 + k) * n + i] = o_l[k];
            a.out[plane + (size_t)(f0 + k) * n + i] = o_r[k];
        }
        DT_ALL_TAPS(DT_ADVANCE)
    }
#undef DT_ALL_TAPS
#undef DT_PRIME
#undef DT_PREFETCH
#undef DT_ADVANCE

    a.state[DTS_LP_PRE * n + i] = lp_pre;
    a.state[DTS_LP_DAMP_A * n + i] = lp_a;
    a.state[DTS_LP_DAMP_B * n + i] = lp_b;
}

hipError_t launch_dattorro(const DattorroArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.t0 & 3u) || (a.n_frames & 3u)) return hipErrorInvalidValue;   // 4-frame chunks
    const uint32_t threads = 64;      // one wave per workgroup: spreads small engines over all CUs
    const uint32_t blocks = (a.n + threads - 1) / threads;
    hipLaunchKernelGGL(dattorro_block_v2, dim3(blocks), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
