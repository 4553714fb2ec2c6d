// ol_dsp_amd/csrc/dattorro.hip -- Dattorro plate reverb kernel: one wavefront lane per instance.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
// The network, its ring layout and the chunked carry/prefetch scheme are in dattorro_stage.h.
#include "dattorro_stage.h"

namespace olfx {

__global__ __launch_bounds__(64, 1) void dattorro_block_v4(DattorroArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;

    DT_STAGE(a, i);
    dt_prime(a.t0);

    // raw input frames are prefetched one chunk ahead like the taps
    float in_l[4], in_r[4], nx_l[4], nx_r[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        in_l[k] = a.in[(size_t)k * n + i];
        in_r[k] = stereo ? a.in[plane + (size_t)k * n + i] : 0.f;
    }
    for (uint32_t f0 = 0; f0 < a.n_frames; f0 += 4) {
        const bool has_next = f0 + 4 < a.n_frames;
        // this chunk's input: (l + r) / 2, ReverbFx.cpp:13-16
        float xin[4], o_l[4], o_r[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) xin[k] = stereo ? (in_l[k] + in_r[k]) / 2 : in_l[k];
        // next chunk's inputs, loaded unconditionally (clamped to the last frame in the last chunk)
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
}

hipError_t launch_dattorro(const DattorroArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.t0 & 3u) || (a.n_frames & 3u)) return hipErrorInvalidValue;   // 4-frame chunks
    // the modulated taps' buffer loads take 32-bit offsets into their (1024-position) rings
    if ((uint64_t)kDtSize[DT_AP1A] * a.n * 4u >= (1ull << 32) || (uint64_t)kDtSize[DT_AP1B] * a.n * 4u >= (1ull << 32))
        return hipErrorInvalidValue;
    const uint32_t threads = 64;      // one wave per workgroup: spreads small engines over all CUs
    const uint32_t blocks = (a.n + threads - 1) / threads;
    hipLaunchKernelGGL(dattorro_block_v4, dim3(blocks), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
