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
// predecessor.  The two modulated all-pass taps and the per-instance pre-delay tap are carried
// the same way (one new group per chunk; see ModTap / PreTap), so every ring byte is read once.
// Groups written by earlier chunks of this launch are read back by the lane that wrote them, in
// program order.  No MFMA: scalar recurrences.
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

// A modulated tank all-pass tap (verb.cpp:262-270): delay D + ex(t), with ex wave-uniform and
// constant for 512 chunks at a time.  Carried like a fixed tap (one new group per chunk); when ex
// steps, both groups are reloaded (a wave-uniform branch, once per 2048 frames).
template <int L, uint32_t D>
struct ModTap {
    float4 cur, nxt, pre;
    float v[4];
    uint32_t q;                                       // position of the chunk's frame 0
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        q = t0 - (D + dt_ap1_extra(t0 & 0xFFFFu));
        cur = *grp<L>(a, q >> 2, i);
        nxt = *grp<L>(a, (q >> 2) + 1u, i);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t i) {
        pre = *grp<L>(a, (q >> 2) + 2u, i);
    }
    __device__ __forceinline__ void resolve() {       // shift q & 3 (wave-uniform) by selects
        const uint32_t s = q & 3u;
        const float w[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = s == 0 ? w[k] : (s == 1 ? w[k + 1] : (s == 2 ? w[k + 2] : w[k + 3]));
    }
    __device__ __forceinline__ void advance(const DattorroArgs &a, uint32_t t0n, uint32_t i) {
        const uint32_t qn = t0n - (D + dt_ap1_extra(t0n & 0xFFFFu));
        if (qn == q + 4u) {
            cur = nxt; nxt = pre;
        } else {                                      // ex stepped: the window moved by one
            cur = *grp<L>(a, qn >> 2, i);
            nxt = *grp<L>(a, (qn >> 2) + 1u, i);
        }
        q = qn;
    }
};

// The per-instance pre-delay tap (verb.cpp:137-139, :273).  Delay d is constant over a launch.
//   d >= 9 : carried ring window with a per-lane shift (t0 - d) & 3: the group prefetched during
//            chunk c (before chunk c's own store) is ((t0 - d) >> 2) + 2 <= chunk c-1's group;
//   d <= 8 : frames of this chunk come from registers, older frames of this launch from the input
//            buffer (re-summed exactly like xin), frames of earlier launches from the ring.  This
//            branch is skipped by every wave whose lanes all have d >= 9.
// Lanes of one wave that share d issue coalesced loads.
struct PreTap {
    float4 cur, nxt, pre;
    uint32_t s;
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t d, uint32_t i) {
        const uint32_t q = t0 - d;
        s = q & 3u;
        cur = *grp<DT_PRE>(a, q >> 2, i);
        nxt = *grp<DT_PRE>(a, (q >> 2) + 1u, i);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t d, uint32_t i) {
        pre = *grp<DT_PRE>(a, ((t0 - d) >> 2) + 2u, i);
    }
    // xpd[k] = mono input at t0 + k - d
    __device__ __forceinline__ void resolve(const DattorroArgs &a, const float xin[4], uint32_t f0,
                                            uint32_t t0, uint32_t d, uint32_t i, bool stereo,
                                            float xpd[4]) const {
        const float w[8] = {cur.x, cur.y, cur.z, cur.w, nxt.x, nxt.y, nxt.z, nxt.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
            xpd[k] = s == 0 ? w[k] : (s == 1 ? w[k + 1] : (s == 2 ? w[k + 2] : w[k + 3]));
        if (d <= 8u) {
            const size_t plane = a.plane;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float v;
                if ((uint32_t)k >= d) {                          // this chunk
                    v = xin[0];
#pragma unroll
                    for (int j = 1; j <= k; ++j) v = (uint32_t)(k - j) == d ? xin[j] : v;
                } else if (f0 + k >= d) {                        // earlier chunk of this launch
                    const size_t f = f0 + k - d;
                    v = a.in[f * a.n + i];
                    if (stereo) v = (v + a.in[plane + f * a.n + i]) / 2;
                } else {                                         // an earlier launch
                    const uint32_t p = t0 + k - d;
                    v = el(*grp<DT_PRE>(a, p >> 2, i), (int)(p & 3u));
                }
                xpd[k] = v;
            }
        }
    }
    __device__ __forceinline__ void advance() { cur = nxt; nxt = pre; }
};

}  // namespace

__global__ __launch_bounds__(64, 1) void dattorro_block_v3(DattorroArgs a) {
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

    const size_t plane = a.plane;
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
    ModTap<DT_AP1A, kDtDelay[DT_AP1A]> ap1a; ModTap<DT_AP1B, kDtDelay[DT_AP1B]> ap1b; PreTap pre;

#define DT_ALL_TAPS(OP) OP(in0) OP(in1) OP(in2) OP(in3) OP(fbA) OP(fbB) OP(dl1a) OP(dl1b) OP(ap2a) OP(ap2b) \
    OP(oL1) OP(oL2) OP(oL3) OP(oL4) OP(oL5) OP(oL6) OP(oL7) OP(oR1) OP(oR2) OP(oR3) OP(oR4) OP(oR5) OP(oR6) OP(oR7)
#define DT_PRIME(T) T.prime(a, a.t0, i);
#define DT_PREFETCH(T) T.prefetch(a, t0, i);
#define DT_ADVANCE(T) T.advance();

    DT_ALL_TAPS(DT_PRIME)
    ap1a.prime(a, a.t0, i);
    ap1b.prime(a, a.t0, i);
    pre.prime(a, a.t0, dpre, i);

    // raw input frames are prefetched one chunk ahead like the taps
    float in_l[4], in_r[4], nx_l[4], nx_r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        in_l[k] = a.in[(size_t)k * n + i];
        in_r[k] = stereo ? a.in[plane + (size_t)k * n + i] : 0.f;
    }

    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        const uint32_t t0 = a.t0 + f0;                 // multiple of 4

        // ---- this chunk's inputs: (l + r) / 2, ReverbFx.cpp:13-16 ----
        float xin[4], xpd[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xin[k] = stereo ? (in_l[k] + in_r[k]) / 2 : in_l[k];
        // ---- prefetch the next chunk's inputs and every tap's next group ----
        if (f0 + 4 < a.n_frames) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                nx_l[k] = a.in[(size_t)(f0 + 4 + k) * n + i];
                nx_r[k] = stereo ? a.in[plane + (size_t)(f0 + 4 + k) * n + i] : 0.f;
            }
            DT_ALL_TAPS(DT_PREFETCH)
            ap1a.prefetch(a, i);
            ap1b.prefetch(a, i);
            pre.prefetch(a, t0, dpre, i);
        }
        ap1a.resolve();
        ap1b.resolve();
        pre.resolve(a, xin, f0, t0, dpre, i, stereo, xpd);

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
        if (f0 + 4 < a.n_frames) {
            ap1a.advance(a, t0 + 4u, i);
            ap1b.advance(a, t0 + 4u, i);
        }
        pre.advance();
#pragma unroll
        for (int k = 0; k < 4; ++k) { in_l[k] = nx_l[k]; in_r[k] = nx_r[k]; }
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
    hipLaunchKernelGGL(dattorro_block_v3, dim3(blocks), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
