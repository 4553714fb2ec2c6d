// ol_dsp_amd/csrc/mix.hip -- voice buses: the Polyvoice / VoiceMap sums.
//
// Reference (modules/synthlib): Polyvoice::Process (Polyvoice.h:28-33) runs each of its voices into
// a one-sample buffer and adds it to the caller's frame, `*frame_out += frame_buffer`, voice by
// voice in vector order; VoiceMap::Process (VoiceMap.h:64-73) does the same over its note slots
// 0..127.  Per frame and bus that is the float sequence (((out + v0) + v1) + ...): one IEEE add per
// voice, in order.  A bus here is that list of voices (CSR: order[off[b] .. off[b+1])), and the
// kernel performs exactly those adds, so a bus is bit-identical to the reference's sum of the same
// voice samples.
//
// HBM-bound and small beside the voice kernel: one 4-B read per voice sample, one 4-B read and one
// 4-B write per bus sample.  Buses run fastest across lanes: the lanes of a wave read the voices of
// neighbouring buses in one frame row, so the lines one add step touches are the lines the next
// step reuses (from the L1).
#include "olfx_internal.h"

namespace olfx {

// One lane = (bus, four frames).  A bus's voice indices are read once per four frames instead of
// once per frame, and the four frames' loads of one voice are independent, so eight loads are in
// flight per unrolled step.  Every frame's adds still run voice by voice in list order.  A block
// row loops over frame tiles (grid.y is capped), so any frame count launches.
constexpr uint32_t kMixFr = 4;
constexpr uint32_t kMixMaxRows = 4096;

__global__ __launch_bounds__(256) void voice_mix_v2(MixArgs a) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= a.n_buses) return;
    for (uint32_t f0 = blockIdx.y * kMixFr; f0 < a.n_frames; f0 += gridDim.y * kMixFr) {
        const uint32_t nfr = a.n_frames - f0 < kMixFr ? a.n_frames - f0 : kMixFr;   // uniform per block
        const float *row = a.in + (size_t)f0 * a.n;
        float *dst = a.out + (size_t)f0 * a.n_buses + b;
        const uint32_t k1 = a.off[b + 1];
        uint32_t k = a.off[b];
        if (nfr == kMixFr) {
            float acc[kMixFr];
#pragma unroll
            for (uint32_t j = 0; j < kMixFr; ++j) acc[j] = dst[(size_t)j * a.n_buses];
            for (; k + 2 <= k1; k += 2) {
                const uint32_t i0 = a.order[k], i1 = a.order[k + 1];
                float v0[kMixFr], v1[kMixFr];
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j) {
                    v0[j] = row[(size_t)j * a.n + i0];
                    v1[j] = row[(size_t)j * a.n + i1];
                }
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j) acc[j] = (acc[j] + v0[j]) + v1[j];
            }
            if (k < k1) {
                const uint32_t i0 = a.order[k];
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j) acc[j] = acc[j] + row[(size_t)j * a.n + i0];
            }
#pragma unroll
            for (uint32_t j = 0; j < kMixFr; ++j) dst[(size_t)j * a.n_buses] = acc[j];
        } else {
            for (uint32_t j = 0; j < nfr; ++j) {
                float acc = dst[(size_t)j * a.n_buses];
                for (uint32_t q = k; q < k1; ++q) acc = acc + row[(size_t)j * a.n + a.order[q]];
                dst[(size_t)j * a.n_buses] = acc;
            }
        }
    }
}

// voice_mix_v4: buses that are contiguous runs of voices in voice order (order[k] == k, the layout
// Polyvoice groups get when voices are allotted in order -- the bench's buses of 8) starting and
// ending on multiples of 4 voices, with 16-B aligned frame rows.  A lane reads its bus's voices as
// float4 runs (buses of 8: two 16-B loads per frame instead of v2's eight 4-B gathers at the bus
// stride, 16 lines per instruction) and adds them in list order -- the same adds as v2, bit for bit.
__global__ __launch_bounds__(256) void voice_mix_v4(MixArgs a) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= a.n_buses) return;
    const uint32_t k0 = a.off[b], k1 = a.off[b + 1];
    for (uint32_t f0 = blockIdx.y * kMixFr; f0 < a.n_frames; f0 += gridDim.y * kMixFr) {
        const uint32_t nfr = a.n_frames - f0 < kMixFr ? a.n_frames - f0 : kMixFr;   // uniform per block
        const float *row = a.in + (size_t)f0 * a.n;
        float *dst = a.out + (size_t)f0 * a.n_buses + b;
        if (nfr == kMixFr) {
            float acc[kMixFr];
#pragma unroll
            for (uint32_t j = 0; j < kMixFr; ++j) acc[j] = dst[(size_t)j * a.n_buses];
            uint32_t k = k0;
            for (; k + 8 <= k1; k += 8) {                 // two runs of 4 per frame in flight
                float4 v0[kMixFr], v1[kMixFr];
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j) {
                    v0[j] = *(const float4 *)(row + (size_t)j * a.n + k);
                    v1[j] = *(const float4 *)(row + (size_t)j * a.n + k + 4);
                }
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j)
                    acc[j] = (((((((acc[j] + v0[j].x) + v0[j].y) + v0[j].z) + v0[j].w) + v1[j].x) + v1[j].y) + v1[j].z) + v1[j].w;
            }
            if (k < k1) {
#pragma unroll
                for (uint32_t j = 0; j < kMixFr; ++j) {
                    const float4 v = *(const float4 *)(row + (size_t)j * a.n + k);
                    acc[j] = (((acc[j] + v.x) + v.y) + v.z) + v.w;
                }
            }
#pragma unroll
            for (uint32_t j = 0; j < kMixFr; ++j) dst[(size_t)j * a.n_buses] = acc[j];
        } else {
            for (uint32_t j = 0; j < nfr; ++j) {
                float acc = dst[(size_t)j * a.n_buses];
                for (uint32_t q = k0; q < k1; ++q) acc = acc + row[(size_t)j * a.n + q];
                dst[(size_t)j * a.n_buses] = acc;
            }
        }
    }
}

hipError_t launch_mix(const MixArgs &a, hipStream_t s) {
    if (a.n_buses == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t rows = (a.n_frames + kMixFr - 1) / kMixFr;
    const dim3 grid((a.n_buses + 255) / 256, rows < kMixMaxRows ? rows : kMixMaxRows);
    if (a.quad && (a.n & 3u) == 0 && ((uintptr_t)a.in & 15u) == 0) {
        hipLaunchKernelGGL(voice_mix_v4, grid, dim3(256), 0, s, a);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(voice_mix_v2, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
