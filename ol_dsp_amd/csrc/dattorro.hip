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
// pre-delays differ) keeps that ring instance-major and runs dattorro_predelay_v1 ahead of the
// block: one lane per instance walks its own ring in stream order (whole lines, in order) and
// hands the network its pre-delayed block as a coalesced stream (PreBlock).  The network itself
// then reads no input and writes no pre-delay ring.
#include "dattorro_stage.h"

namespace olfx {

template <bool GATHER>
__global__ __launch_bounds__(64, 1) void dattorro_block_v4(DattorroArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;

    using Pre = typename std::conditional<GATHER, olfx::dt::PreBlock, olfx::dt::PreTap>::type;
    DT_STAGE_PRE(a, i, Pre);
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
}

// Gather mode's pre-pass: one lane per instance, chunk by chunk in stream order as
// DelayBuffer_process (verb.cpp:107-110: write position t, then read t - d): the chunk's
// pre-delayed samples are read first -- the positions before the chunk from the instance's own
// ring (two aligned 16-B pieces: consecutive chunks hit the same line back to back, one fetch per
// line), those inside it (d < 4) from the chunk's input -- then the chunk's mono input (l + r) / 2
// is written (a lane's pieces of one line leave back to back: the L2 merges them into whole lines).
// The pre-delayed block goes out as [F/4][n][4] (coalesced) for the network.
constexpr uint32_t kPreSize = kDtSize[DT_PRE];
__global__ __launch_bounds__(256) void dattorro_predelay_v1(DattorroArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;
    const uint32_t d = (uint32_t)a.coef[DTC_PREDELAY * n + i];         // exact integer 0..8191
    const float *ring_r = a.pre_im + (size_t)i * kPreSize;
    float *ring = a.pre_im + (size_t)i * kPreSize;
    float4 *blk = (float4 *)a.pre_block;
    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        float x[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float l = a.in[(size_t)(f0 + k) * n + i];
            x[k] = stereo ? (l + a.in[plane + (size_t)(f0 + k) * n + i]) / 2 : l;
        }
        const uint32_t t = a.t0 + f0, q = t - d, g = q & ~3u;
        const float4 pa = *(const float4 *)(ring_r + (g & (kPreSize - 1u)));
        const float4 pb = *(const float4 *)(ring_r + ((g + 4u) & (kPreSize - 1u)));
        float v[4];
        olfx::dt::shift4(q & 3u, pa, pb, v);
        // positions inside this chunk (d <= k): x[k - d], by selects (no indexed register access)
        v[0] = d == 0u ? x[0] : v[0];
        v[1] = d == 0u ? x[1] : (d == 1u ? x[0] : v[1]);
        v[2] = d == 0u ? x[2] : (d == 1u ? x[1] : (d == 2u ? x[0] : v[2]));
        v[3] = d == 0u ? x[3] : (d == 1u ? x[2] : (d == 2u ? x[1] : (d == 3u ? x[0] : v[3])));
        blk[(size_t)(f0 >> 2) * n + i] = make_float4(v[0], v[1], v[2], v[3]);
        *(float4 *)(ring + (t & (kPreSize - 1u))) = make_float4(x[0], x[1], x[2], x[3]);
    }
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

hipError_t launch_dattorro(const DattorroArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.t0 & 3u) || (a.n_frames & 3u)) return hipErrorInvalidValue;   // 4-frame chunks
    // the modulated taps' buffer loads take 32-bit offsets into their (1024-position) rings
    if ((uint64_t)kDtSize[DT_AP1A] * a.n * 4u >= (1ull << 32) || (uint64_t)kDtSize[DT_AP1B] * a.n * 4u >= (1ull << 32))
        return hipErrorInvalidValue;
    const uint32_t threads = 64;      // one wave per workgroup: spreads small engines over all CUs
    const uint32_t blocks = (a.n + threads - 1) / threads;
    if (a.pre_im) {
        hipLaunchKernelGGL(dattorro_predelay_v1, dim3((a.n + 255) / 256), dim3(256), 0, s, a);
        hipLaunchKernelGGL(dattorro_block_v4<true>, dim3(blocks), dim3(threads), 0, s, a);
    } else {
        hipLaunchKernelGGL(dattorro_block_v4<false>, dim3(blocks), dim3(threads), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_dattorro_pre_convert(const DattorroArgs &a, bool to_im, hipStream_t s) {
    if (a.n == 0) return hipSuccess;
    hipLaunchKernelGGL(dattorro_pre_convert, dim3((a.n + 255) / 256, kPreSize / 4), dim3(256), 0, s, a, to_im ? 1 : 0);
    return hipGetLastError();
}

}  // namespace olfx
