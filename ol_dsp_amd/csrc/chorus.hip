// ol_dsp_amd/csrc/chorus.hip -- RNBO stereo chorus and gen~ pitch-shifter kernel on gfx950.
// The stage (spec, memory shape, line carry, software pipeline) is in chorus_stage_l.h, its
// helpers in chorus_stage.h.
#include "chorus_stage_l.h"

namespace olfx {

// chorus_block_v11: one wave = 32 instances x 2 channels over the line-carry stage
// (chorus_stage_l.h); chunks alternate the line set (PAR), so the chunk loop is unrolled by two.
template <bool FULL>
__global__ __launch_bounds__(ch::kThreads, 2) void chorus_block_v11(ChorusArgs a) {
    using Stage = ch::ChStageL<FULL>;
    constexpr int kChunk = Stage::kChunk;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t tid = threadIdx.x;
    const uint32_t wib = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t wave = blockIdx.x * (ch::kThreads / 64) + wib, lane = tid & 63u;
    const uint32_t inst0 = wave * 32u;
    if (inst0 >= a.n) return;
    Stage st;
    st.init(a, lds + wib * Stage::kRegion, lane, inst0);

    const uint32_t nf = a.n_frames, n = a.n;
    const ch::Rsrc rIn = ch::rsrc(a.in, (a.plane + (uint64_t)nf * n) * 4);
    const ch::Rsrc rOut = ch::rsrc(a.out, (a.plane + (uint64_t)nf * n) * 4);
    const uint32_t io_v = st.ch * (uint32_t)a.plane * 4u + st.i * 4u, frame_b = n * 4u;
    const uint32_t out_v = st.valid ? io_v : 0xFFFFFFF0u;

    float x[kChunk], xn[kChunk];
    int C = (int)min((uint32_t)kChunk, nf);
#pragma unroll
    for (int k = 0; k < kChunk; ++k) x[k] = k < C ? ch::ld1<ch::kStreamAux>(rIn, io_v, (uint32_t)k * frame_b) : 0.f;
    st.begin(x, C);
    auto step = [&](auto par, uint32_t f0) {
        C = (int)min((uint32_t)kChunk, nf - f0);
        const int Cn = f0 + kChunk < nf ? (int)min((uint32_t)kChunk, nf - f0 - kChunk) : 0;
        // the next chunk's input (unconditional loads, the frame clamped into the block; lanes
        // past Cn get 0), issued by the stage once this chunk's stores and staging are out
        auto prefetch = [&]() {
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                const float v = ch::ld1<ch::kStreamAux>(rIn, io_v, min(f0 + kChunk + (uint32_t)k, nf - 1u) * frame_b);
                xn[k] = k < Cn ? v : 0.f;
            }
        };
        st.template chunk<decltype(par)::value>(
            x, xn, C, Cn,
            [&](int k, float v) { ch::st1<ch::kStreamAux>(rOut, out_v, (f0 + (uint32_t)k) * frame_b, v); }, prefetch);
#pragma unroll
        for (int k = 0; k < kChunk; ++k) x[k] = xn[k];
    };
    for (uint32_t f0 = 0; f0 < nf; f0 += 2 * kChunk) {
        step(std::integral_constant<int, 0>{}, f0);
        if (f0 + kChunk < nf) step(std::integral_constant<int, 1>{}, f0 + kChunk);
    }
    st.finish(a);
}


hipError_t launch_chorus(const ChorusArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.n_frames & 3u) || (a.t0 & 3u)) return hipErrorInvalidValue;
    // 32-bit buffer offsets: the rings and the two audio planes must stay below 4 GiB
    if ((uint64_t)a.n * 2 * a.csize * 4 >= (1ull << 32) || (a.plane + (uint64_t)a.n_frames * a.n) * 4 >= (1ull << 32) ||
        a.plane < (uint64_t)a.n_frames * a.n)
        return hipErrorInvalidValue;
    const uint32_t waves = (a.n + 31) / 32;              // 32 instances x 2 channels per wave
    const uint32_t blocks = (waves + ch::kThreads / 64 - 1) / (ch::kThreads / 64);
    const size_t lds_c = (size_t)(ch::kThreads / 64) * ch::ChStageL<true>::kRegion * sizeof(float);
    const size_t lds_p = (size_t)(ch::kThreads / 64) * ch::ChStageL<false>::kRegion * sizeof(float);
    if (a.mode == 0) hipLaunchKernelGGL(chorus_block_v11<true>, dim3(blocks), dim3(ch::kThreads), lds_c, s, a);
    else hipLaunchKernelGGL(chorus_block_v11<false>, dim3(blocks), dim3(ch::kThreads), lds_p, s, a);
    return hipGetLastError();
}

}  // namespace olfx
