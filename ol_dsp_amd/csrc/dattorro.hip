// ol_dsp_amd/csrc/dattorro.hip -- Dattorro plate reverb kernels: one wavefront lane per instance.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
// The network, its ring layout and the step carry/prefetch scheme are in dattorro_stage.h.
//
// Two networks ("Which network"):
//   dattorro_block_v4: one wave per 64 instances carries all 27 taps (one wave per SIMD); the
//     pre-delay ring position-major like every other ring, one pre-delay for all instances (PreTap).
//     Taken for uniform pre-delays once v4 has at least two waves per CU (32,768 instances and up
//     on 256 CUs), where the memory system is the limit and v4 keeps the most loads in flight.
//   dattorro_block_v5: the split network (DI, TA, TB: three waves per 64 instances) with the
//     pre-delay ring in ROWS of 16 positions ([512][n][16], dt::PreRow): any mix of per-instance
//     pre-delays (verb.cpp:137-139) costs one 64-B row per instance and 16 frames.  Taken below
//     that size (v4 would leave SIMDs idle) and for per-instance pre-delays at every size.
// The engine keeps the pre-delay ring in the layout of the network it runs and converts it when
// the choice changes (dattorro_pre_layout; the pre-delays became equal or differ).
#include <cstdlib>

#include "dattorro_stage.h"
#include "lds_flags.h"

namespace olfx {

// IN1 (the second input diffuser, 128 positions, verb.cpp:180) is read and written in LDS for the
// launch (LdsTap): its 8 B/frame of ring traffic become 512 B in and out per instance and launch.
__global__ __launch_bounds__(64, 1) void dattorro_block_v4(DattorroArgs a) {
    __shared__ float4 in1_ring[kDtSize[DT_IN1] / 4u * 64u];      // 32 KB: [group][lane]
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;

    DT_STAGE_X(a, i, olfx::dt::PreTap, (olfx::dt::LdsTap<DT_IN1, 107>));
    in1.lds = in1_ring + threadIdx.x;
    in1.lds_in(a, i);
    dt_prime(a.t0);

    // raw input frames are prefetched one step ahead like the taps
    float in_l[4], in_r[4], nx_l[4], nx_r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        in_l[k] = a.in[(size_t)k * n + i];
        in_r[k] = stereo ? a.in[plane + (size_t)k * n + i] : 0.f;
    }
    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        const bool has_next = f0 + 4 < a.n_frames;
        // this step's input: (l + r) / 2, ReverbFx.cpp:13-16
        float xin[4], o_l[4], o_r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xin[k] = stereo ? (in_l[k] + in_r[k]) / 2 : in_l[k];
        // next step's inputs, loaded unconditionally (clamped to the last frame in the last step)
        const uint32_t fn = has_next ? f0 + 4 : f0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            nx_l[k] = a.in[(size_t)(fn + k) * n + i];
            nx_r[k] = stereo ? a.in[plane + (size_t)(fn + k) * n + i] : 0.f;
        }
        dt_step(a.t0 + f0, has_next, xin, o_l, o_r);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a.out[(size_t)(f0 + k) * n + i] = o_l[k];
            a.out[plane + (size_t)(f0 + k) * n + i] = o_r[k];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) { in_l[k] = nx_l[k]; in_r[k] = nx_r[k]; }
    }
    dt_finish();
    in1.lds_out(a, i);
}

// dattorro_block_v5 (round 6): the split network of dattorro_stage.h -- DI, TA and TB, one wave
// each per 64 instances -- so each wave carries only its own taps (DI 5, each half 11, where v4's
// one wave carries all 27): 16,384 instances run 768 waves instead of 256.  DI takes its input 16
// frames ahead, keeps IN1's ring in LDS for the launch and the pre-delay ring in rows
// (dt::split_di_rows).  LDS: IN1 32 KB + the row staging 25 KB + the queues 12 KB: two workgroups
// per CU.  Launches of at most kSplitMaxFrames frames.
__global__ __launch_bounds__(192) void dattorro_block_v5(DattorroArgs a) {
    __shared__ float4 in1_ring[kDtSize[DT_IN1] / 4u * 64u];     // DI's IN1 ring (32 KB)
    __shared__ float4 stage[25 * 64];                           // DI's pre-delay row staging (25 KB)
    __shared__ float4 qx[dt::kSplitDepth * 64u], q0[dt::kSplitDepth * 64u], q1[dt::kSplitDepth * 64u];
    __shared__ uint32_t flags[dt::SPF_N];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t role = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t n = a.n, nf = a.n_frames;
    const uint32_t i0 = blockIdx.x * 64u + lane;
    const bool live = i0 < n;
    const uint32_t i = live ? i0 : n - 1u;             // dead lanes mirror instance n - 1 (same bits)
    if (tid < dt::SPF_N) flags[tid] = 0;
    __syncthreads();
    const uint32_t steps = nf / 4u;
    if (role == 1) {
        dt::split_tank<0>(a, i, lane, live, a.t0, steps, 0, a.out, n, {qx, q0, q1, flags});
        return;
    }
    if (role == 2) {
        dt::split_tank<1>(a, i, lane, live, a.t0, steps, 0, a.out + a.plane, n, {qx, q1, q0, flags});
        return;
    }
    // ---- DI: the input (l + r) / 2 (ReverbFx.cpp:13-16), 16 frames ahead; the network's front ----
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;
    olfx::dt::LdsTap<DT_IN1, 107> in1;
    in1.lds = in1_ring + lane;
    in1.lds_in(a, i);
    float nl[16], nr[16];
    auto load = [&](uint32_t f0) {                    // frames f0 .. f0 + 15, clamped to the block
#pragma unroll
        for (int k = 0; k < 16; ++k) {
            const uint32_t f = min(f0 + (uint32_t)k, nf - 1u);
            nl[k] = a.in[(size_t)f * n + i];
            nr[k] = stereo ? a.in[plane + (size_t)f * n + i] : 0.f;
        }
    };
    load(0);
    dt::split_di_rows(a, blockIdx.x, lane, nf, 0, stage, qx, flags, in1,
                      [&](uint32_t, uint32_t f0, uint32_t, float (&xm)[16]) {
#pragma unroll
                          for (int k = 0; k < 16; ++k) xm[k] = stereo ? (nl[k] + nr[k]) / 2 : nl[k];
                          load(f0 + 16u);
                      });
    in1.lds_out(a, i);
}

// The pre-delay ring between layouts, through a copy of it (src): position-major groups
// [8192/4][n][4] (v4's PreTap) <-> rows [8192/16][n][16] (v5's PreRow).  One thread per (row,
// instance): 4 groups of one side, one 64-B row of the other; the position-major side coalesced.
__global__ __launch_bounds__(256) void dattorro_pre_layout(const float4 *__restrict__ src, float4 *__restrict__ dst,
                                                           uint32_t n, int to_rows) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x, r = blockIdx.y;
    if (i >= n) return;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const size_t pos = (size_t)(4u * r + q) * n + i, row = ((size_t)r * n + i) * 4u + q;
        if (to_rows) dst[row] = src[pos];
        else dst[pos] = src[row];
    }
}

// The network for these pre-delays ("Which network"): v4 for one pre-delay
// once v4 has two waves per CU, else v5 (same box, profiles/r6/NOTES.md: 16,384 instances v5 0.138
// against v4 0.166 ms; 32,768 v4 0.2764 against v5 0.2797; 65,536 v4 0.5551 against v5 0.5736).
// OLFX_DT_V4=1 / =0 forces v4 / v5 for uniform pre-delays (A/B timing).
int dattorro_network(uint32_t n, uint32_t cus, bool uniform) {
    static const int force = [] {
        const char *e = std::getenv("OLFX_DT_V4");
        return e && e[0] ? (e[0] == '1' ? 1 : 0) : -1;
    }();
    if (!uniform) return DT_NET_V5;
    if (force >= 0) return force ? DT_NET_V4 : DT_NET_V5;
    return (uint64_t)(n + 63u) / 64u >= 2ull * (cus ? cus : 256u) ? DT_NET_V4 : DT_NET_V5;
}

const char *dattorro_network_name(int net) { return net == DT_NET_V4 ? "dattorro_block_v4" : "dattorro_block_v5"; }

hipError_t launch_dattorro(const DattorroArgs &a, int net, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.t0 & 3u) || (a.n_frames & 3u)) return hipErrorInvalidValue;   // 4-frame steps
    // the modulated taps' buffer loads take 32-bit offsets into their (1024-position) rings
    if ((uint64_t)kDtSize[DT_AP1A] * a.n * 4u >= (1ull << 32) || (uint64_t)kDtSize[DT_AP1B] * a.n * 4u >= (1ull << 32))
        return hipErrorInvalidValue;
    const uint32_t blocks = (a.n + 63u) / 64u;   // one 64-instance group per workgroup
    if (net == DT_NET_V4) {
        hipLaunchKernelGGL(dattorro_block_v4, dim3(blocks), dim3(64), 0, s, a);
        return hipGetLastError();
    }
    // pieces of at most kSplitMaxFrames (the halves' cross taps then read earlier launches only)
    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += dt::kSplitMaxFrames) {
        DattorroArgs p = a;
        p.n_frames = min(dt::kSplitMaxFrames, a.n_frames - f0);
        p.t0 = (a.t0 + f0) & 0xFFFFu;
        p.in = a.in + (size_t)f0 * a.n;
        p.out = a.out + (size_t)f0 * a.n;
        hipLaunchKernelGGL(dattorro_block_v5, dim3(blocks), dim3(192), 0, s, p);
    }
    return hipGetLastError();
}

hipError_t launch_dattorro_pre_layout(const DattorroArgs &a, float *tmp, bool to_rows, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    const size_t bytes = (size_t)kDtSize[DT_PRE] * a.n * 4u;
    hipError_t r = hipMemcpyAsync(tmp, a.ring[DT_PRE], bytes, hipMemcpyDeviceToDevice, s);
    if (r != hipSuccess) return r;
    hipLaunchKernelGGL(dattorro_pre_layout, dim3((a.n + 255) / 256, kDtSize[DT_PRE] / 16), dim3(256), 0, s,
                       (const float4 *)tmp, (float4 *)a.ring[DT_PRE], a.n, to_rows ? 1 : 0);
    return hipGetLastError();
}

}  // namespace olfx
