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

// voice_mix_v3: buses that are contiguous runs of voices in voice order (order[k] == k, the layout
// Polyvoice groups get when voices are allotted in order -- the bench's buses of 8).  A block takes
// 256 buses; per 4 frames it stages the voice run those buses cover, [off[b0], off[b0 + 256)), from
// each frame row into LDS with coalesced loads (256 lanes x 4 B per instruction: one 1-KB run),
// then every lane adds its bus's voices from LDS in list order -- the same adds as v2, bit for bit.
// v2's lanes gathered 4 B each at the bus stride (32 B for buses of 8): 16 lines per load
// instruction for 256 B used ("Voice buses").
__global__ __launch_bounds__(256) void voice_mix_v3(MixArgs a, uint32_t span) {
    extern __shared__ float stage[];                  // [kMixFr][span]
    const uint32_t b0 = blockIdx.x * 256u, b = b0 + threadIdx.x;
    const uint32_t bl = b0 + 256u < a.n_buses ? b0 + 256u : a.n_buses;
    const uint32_t v0 = a.off[b0], len = a.off[bl] - v0;
    const bool live = b < a.n_buses;
    const uint32_t k0 = live ? a.off[b] - v0 : 0u, k1 = live ? a.off[b + 1] - v0 : 0u;
    for (uint32_t f0 = blockIdx.y * kMixFr; f0 < a.n_frames; f0 += gridDim.y * kMixFr) {
        const uint32_t nfr = a.n_frames - f0 < kMixFr ? a.n_frames - f0 : kMixFr;   // uniform per block
        __syncthreads();                              // the previous rows' readers are done
        for (uint32_t j = 0; j < nfr; ++j) {
            const float *row = a.in + (size_t)(f0 + j) * a.n + v0;
            for (uint32_t q = threadIdx.x; q < len; q += 256u) stage[j * span + q] = row[q];
        }
        __syncthreads();
        if (!live) continue;
        float *dst = a.out + (size_t)f0 * a.n_buses + b;
        for (uint32_t j = 0; j < nfr; ++j) {
            const float *v = stage + j * span;
            float acc = dst[(size_t)j * a.n_buses];
            for (uint32_t k = k0; k < k1; ++k) acc = acc + v[k];
            dst[(size_t)j * a.n_buses] = acc;
        }
    }
}

hipError_t launch_mix(const MixArgs &a, hipStream_t s) {
    if (a.n_buses == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t rows = (a.n_frames + kMixFr - 1) / kMixFr;
    const dim3 grid((a.n_buses + 255) / 256, rows < kMixMaxRows ? rows : kMixMaxRows);
    if (a.contig_span) {
        hipLaunchKernelGGL(voice_mix_v3, grid, dim3(256), (size_t)kMixFr * a.contig_span * sizeof(float), s, a,
                           a.contig_span);
        return hipGetLastError();
    }
    hipLaunchKernelGGL(voice_mix_v2, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
