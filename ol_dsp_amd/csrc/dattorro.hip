// ol_dsp_amd/csrc/dattorro.hip -- Dattorro plate reverb, one wavefront lane per instance.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
//
// Layout: ring l is [kDtSize[l]][n] floats (position-major, instance fastest).  Every instance of
// an engine shares the stream time t and all tap delays, so for each (sample, tap) the 64 lanes of
// a wave touch 64 consecutive floats = one 256-B coalesced segment.  Tap addresses depend only on
// t, never on data, so loads are issued ahead of the serial recurrence.  No MFMA: the work is a
// scalar recurrence per instance.  Bound: HBM.
#include "olfx_internal.h"

namespace olfx {

namespace {

template <int L>
__device__ __forceinline__ float *row(const DattorroArgs &a, uint32_t t, uint32_t delay, uint32_t i) {
    constexpr uint32_t mask = kDtSize[L] - 1u;
    return a.ring[L] + (size_t)((t - delay) & mask) * a.n + i;
}

}  // namespace

// One lane = one instance; loops over the frames of the block.
__global__ __launch_bounds__(256) void dattorro_block_v1(DattorroArgs a) {
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
    float lp_pre = a.state[DTS_LP_PRE * n + i];
    float lp_a = a.state[DTS_LP_DAMP_A * n + i];
    float lp_b = a.state[DTS_LP_DAMP_B * n + i];

    const size_t plane = (size_t)a.n_frames * n;
    const uint32_t dpre = a.pre_delay;

    for (uint32_t f = 0; f < a.n_frames; ++f) {
        const uint32_t t = (a.t0 + f) & 0xFFFFu;
        const uint32_t ex = dt_ap1_extra(t);

        // ---- gather every tap of this frame (addresses depend on t only) ----
        float xin = a.in[(size_t)f * n + i];
        if (a.in_ch == 2) xin = (xin + a.in[plane + (size_t)f * n + i]) / 2;
        const float d_pre = dpre ? *row<DT_PRE>(a, t, dpre, i) : xin;
        const float d_in0 = *row<DT_IN0>(a, t, kDtDelay[DT_IN0], i);
        const float d_in1 = *row<DT_IN1>(a, t, kDtDelay[DT_IN1], i);
        const float d_in2 = *row<DT_IN2>(a, t, kDtDelay[DT_IN2], i);
        const float d_in3 = *row<DT_IN3>(a, t, kDtDelay[DT_IN3], i);
        const float fb_b = *row<DT_DL2B>(a, t, kDtDelay[DT_DL2B], i);   // feeds half A
        const float fb_a = *row<DT_DL2A>(a, t, kDtDelay[DT_DL2A], i);   // feeds half B
        const float d_ap1a = *row<DT_AP1A>(a, t, kDtDelay[DT_AP1A] + ex, i);
        const float d_ap1b = *row<DT_AP1B>(a, t, kDtDelay[DT_AP1B] + ex, i);
        const float d_dl1a = *row<DT_DL1A>(a, t, kDtDelay[DT_DL1A], i);
        const float d_dl1b = *row<DT_DL1B>(a, t, kDtDelay[DT_DL1B], i);
        const float d_ap2a = *row<DT_AP2A>(a, t, kDtDelay[DT_AP2A], i);
        const float d_ap2b = *row<DT_AP2B>(a, t, kDtDelay[DT_AP2B], i);

        // ---- input section: predelay -> 1-pole LPF -> 4 all-passes (verb.cpp:273-282) ----
        *row<DT_PRE>(a, t, 0, i) = xin;
        lp_pre += (d_pre - lp_pre) * g_pre;
        float x = lp_pre;
        x += d_in0 * -g_in1; *row<DT_IN0>(a, t, 0, i) = x; x = d_in0 + x * g_in1;
        x += d_in1 * -g_in1; *row<DT_IN1>(a, t, 0, i) = x; x = d_in1 + x * g_in1;
        x += d_in2 * -g_in2; *row<DT_IN2>(a, t, 0, i) = x; x = d_in2 + x * g_in2;
        x += d_in3 * -g_in2; *row<DT_IN3>(a, t, 0, i) = x; x = d_in3 + x * g_in2;

        // ---- tank half A (verb.cpp:284-295, i = 0); the APF gain is -dd1 ----
        {
            float y = x + fb_b * g_decay;
            y += d_ap1a * g_dd1;                 // in += delayed * -(-dd1)
            *row<DT_AP1A>(a, t, 0, i) = y;
            y = d_ap1a + y * -g_dd1;
            *row<DT_DL1A>(a, t, 0, i) = y;
            lp_a += (d_dl1a - lp_a) * g_damp;
            y = lp_a * g_decay;
            y += d_ap2a * -g_dd2;
            *row<DT_AP2A>(a, t, 0, i) = y;
            y = d_ap2a + y * g_dd2;
            *row<DT_DL2A>(a, t, 0, i) = y;
        }
        // ---- tank half B (i = 1) ----
        {
            float y = x + fb_a * g_decay;
            y += d_ap1b * g_dd1;
            *row<DT_AP1B>(a, t, 0, i) = y;
            y = d_ap1b + y * -g_dd1;
            *row<DT_DL1B>(a, t, 0, i) = y;
            lp_b += (d_dl1b - lp_b) * g_damp;
            y = lp_b * g_decay;
            y += d_ap2b * -g_dd2;
            *row<DT_AP2B>(a, t, 0, i) = y;
            y = d_ap2b + y * g_dd2;
            *row<DT_DL2B>(a, t, 0, i) = y;
        }

        // ---- stereo taps at t+1 (verb.cpp:298-325) ----
        const uint32_t tn = t + 1u;
        float l = *row<DT_DL1B>(a, tn, kDl1B_o1, i);
        l += *row<DT_DL1B>(a, tn, kDl1B_o2, i);
        l -= *row<DT_AP2B>(a, tn, kAp2B_o2, i);
        l += *row<DT_DL2B>(a, tn, kDl2B_o2, i);
        l -= *row<DT_DL1A>(a, tn, kDl1A_o3, i);
        l -= *row<DT_AP2A>(a, tn, kAp2A_o1, i);
        l += *row<DT_DL2A>(a, tn, kDl2A_o1, i);
        float r = *row<DT_DL1A>(a, tn, kDl1A_o1, i);
        r += *row<DT_DL1A>(a, tn, kDl1A_o2, i);
        r -= *row<DT_AP2A>(a, tn, kAp2A_o2, i);
        r += *row<DT_DL2A>(a, tn, kDl2A_o2, i);
        r -= *row<DT_DL1B>(a, tn, kDl1B_o3, i);
        r -= *row<DT_AP2B>(a, tn, kAp2B_o1, i);
        r += *row<DT_DL2B>(a, tn, kDl2B_o1, i);
        a.out[(size_t)f * n + i] = l;
        a.out[plane + (size_t)f * n + i] = r;
    }

    a.state[DTS_LP_PRE * n + i] = lp_pre;
    a.state[DTS_LP_DAMP_A * n + i] = lp_a;
    a.state[DTS_LP_DAMP_B * n + i] = lp_b;
}

hipError_t launch_dattorro(const DattorroArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t threads = 256;
    const uint32_t blocks = (a.n + threads - 1) / threads;
    hipLaunchKernelGGL(dattorro_block_v1, dim3(blocks), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
