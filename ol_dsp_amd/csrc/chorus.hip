// ol_dsp_amd/csrc/chorus.hip -- RNBO stereo chorus and gen~ pitch-shifter kernel on gfx950.
// The stage (spec, memory shape, line carry, software pipeline) is in chorus_stage_l.h, its
// helpers in chorus_stage.h.
#include "chorus_stage_l.h"

namespace olfx {

// Round 4's block-at-once kernels (chorus_block_v13: frame-parallel pitch-shifter and chorus tap
// over a whole 256-frame block per 16 instances, lores~ serial; v14: lores~ on its own wave,
// overlapped with the next group) were bit-exact and slower (chorus 0.324-0.328 ms against v11's
// 0.234-0.241, pitch-shift 0.151-0.168 against 0.148-0.152) and are not kept.

// chorus_block_v11: one wave = 32 instances x 2 channels over the line-carry stage
// (chorus_stage_l.h); chunks alternate the line set (PAR), so the chunk loop is unrolled by two.
// COOP: cooperative input/output rows (4 + 4 dwordx4 per lane and chunk, transposed through LDS:
// ChStageL COOP), for n and the plane distance multiples of 4 (16-B aligned rows, no row split by
// the last instance); otherwise one float per lane, frame and direction.
template <bool FULL, bool COOP>
__global__ __launch_bounds__(ch::kThreads, 2) void chorus_block_v11(ChorusArgs a) {
    using Stage = ch::ChStageL<FULL, COOP>;
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
    // COOP rows: lane's piece of row r = (frame r / 2, channel r % 2): instances inst0 + 4 (lane % 8) ..
    const uint32_t pinst = inst0 + (lane & 7u) * 4u;
    auto row_v = [&](int q, uint32_t f0) {              // byte offset of the lane's piece, frame clamped
        const uint32_t r = Stage::coop_row(q, lane);
        return (r & 1u) * (uint32_t)a.plane * 4u + min(f0 + (r >> 1), nf - 1u) * frame_b + pinst * 4u;
    };

    float x[kChunk], xn[kChunk];
    float4 xq[4];
    int C = (int)min((uint32_t)kChunk, nf);
    if constexpr (COOP) {
#pragma unroll
        for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, 0));
        st.begin(x, C, xq);
    } else {
#pragma unroll
        for (int k = 0; k < kChunk; ++k) x[k] = k < C ? ch::ld1<ch::kStreamAux>(rIn, io_v, (uint32_t)k * frame_b) : 0.f;
        st.begin(x, C);
    }
    auto step = [&](auto par, uint32_t f0) {
        C = (int)min((uint32_t)kChunk, nf - f0);
        const int Cn = f0 + kChunk < nf ? (int)min((uint32_t)kChunk, nf - f0 - kChunk) : 0;
        // the next chunk's input (unconditional loads, the frame clamped into the block; lanes
        // past Cn get 0), issued by the stage once this chunk's stores and staging are out
        auto prefetch = [&]() {
            if constexpr (COOP) {
#pragma unroll
                for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, f0 + kChunk));
            } else {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    const float v = ch::ld1<ch::kStreamAux>(rIn, io_v, min(f0 + kChunk + (uint32_t)k, nf - 1u) * frame_b);
                    xn[k] = k < Cn ? v : 0.f;
                }
            }
        };
        if constexpr (COOP) {
            st.template chunk<decltype(par)::value>(
                x, xn, C, Cn, [&](int k, float v) { st.out_stage(k, v); }, prefetch, xq);
            // the chunk's outputs: rows of 32 instances, 16 B per lane (frames past C dropped)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t r = Stage::coop_row(q, lane), f = r >> 1;
                const bool ok = pinst < n && (int)f < C;
                ch::st4(rOut, ok ? (r & 1u) * (uint32_t)a.plane * 4u + (f0 + f) * frame_b + pinst * 4u : 0xFFFFFFF0u,
                        st.coop_out(q));
            }
        } else {
            st.template chunk<decltype(par)::value>(
                x, xn, C, Cn,
                [&](int k, float v) { ch::st1<ch::kStreamAux>(rOut, out_v, (f0 + (uint32_t)k) * frame_b, v); },
                prefetch, xq);
        }
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
    auto lds = [](auto full, auto coop) {
        return (size_t)(ch::kThreads / 64) * ch::ChStageL<decltype(full)::value, decltype(coop)::value>::kRegion *
               sizeof(float);
    };
    using T = std::true_type;
    using F = std::false_type;
    const size_t lds_c = lds(T{}, T{}), lds_cl = lds(T{}, F{}), lds_p = lds(F{}, T{}), lds_pl = lds(F{}, F{});
    // cooperative rows need 16-B aligned rows that never straddle the last instance
    const bool coop = (a.n & 3u) == 0 && (a.plane & 3u) == 0 && (((uintptr_t)a.in | (uintptr_t)a.out) & 15u) == 0;
    if (a.mode == 0) {
        if (coop) hipLaunchKernelGGL((chorus_block_v11<true, true>), dim3(blocks), dim3(ch::kThreads), lds_c, s, a);
        else hipLaunchKernelGGL((chorus_block_v11<true, false>), dim3(blocks), dim3(ch::kThreads), lds_cl, s, a);
    } else {
        if (coop) hipLaunchKernelGGL((chorus_block_v11<false, true>), dim3(blocks), dim3(ch::kThreads), lds_p, s, a);
        else hipLaunchKernelGGL((chorus_block_v11<false, false>), dim3(blocks), dim3(ch::kThreads), lds_pl, s, a);
    }
    return hipGetLastError();
}

}  // namespace olfx
