// ol_dsp_amd/csrc/chorus.hip -- RNBO stereo chorus and gen~ pitch-shifter kernel on gfx950.
// The stage (spec, memory shape, line carry, software pipeline) is in chorus_stage_l.h, its
// helpers in chorus_stage.h.
#include <cstdlib>

#include "chorus_block.h"
#include "chorus_pc.h"
#include "chorus_stage_l.h"

namespace olfx {

// chorus_block_v13 (chorus_block.h): one persistent workgroup per CU, 16 stereo instances per
// round, the next round's rings / window / input rows prefetched into registers.  Rounds are
// assigned XCD-aware: the groups of a workgroup's round sit next to those of the other workgroups
// of its XCD (workgroups are dispatched to the XCDs round-robin), so the two 16-instance halves
// of every 128-B input / output row line are fetched by one L2.
#ifndef OLFX_CB_STAMP
#define OLFX_CB_STAMP 0
#endif
#if OLFX_CB_STAMP
// diagnostic: workgroup 0's phase boundaries (s_memtime), read back by olfx_debug_stamps
__device__ uint64_t g_cb_stamps[512];
#define CB_STAMP(k)                                                                        \
    do {                                                                                   \
        if (blockIdx.x == 0 && threadIdx.x == 0 && ns < 500u) g_cb_stamps[ns] = __builtin_amdgcn_s_memtime(); \
        ++ns;                                                                              \
    } while (0)
#else
#define CB_STAMP(k) do { } while (0)
#endif

template <bool FULL>
__global__ __launch_bounds__(cb::kThreads, 1) void chorus_block_v13(ChorusArgs a) {
    uint32_t ns = 0;
    (void)ns;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    cb::Block<FULL> B(a, lds);
    const uint32_t ngroups = (a.n + cb::kG - 1) / cb::kG;
    const uint32_t grid = gridDim.x, b = blockIdx.x;
    uint32_t g = (grid & 7u) == 0 ? (b & 7u) * (grid >> 3) + (b >> 3) : b;
    if (g >= ngroups) return;
    int buf = 0;
    cb::Pre pre;
    CB_STAMP(0);
    B.store_scalar(buf, B.load_scalar(g));
    __syncthreads();
    B.issue(g, buf, pre);
    B.fill(buf, pre);
    __syncthreads();
    while (true) {
        CB_STAMP(1);
        const uint32_t gn = g + grid;
        const bool next = gn < ngroups;
        uint32_t sv = 0;
        if (next) sv = B.load_scalar(gn);
        B.phase1(g, buf);
        if (next) B.store_scalar(buf ^ 1, sv);
        __syncthreads();
        CB_STAMP(2);
        if (next) B.issue(gn, buf ^ 1, pre);        // in flight under phases 2, 3 and the outputs
        CB_STAMP(3);
        if (FULL) {
            B.phase2(buf);
            __syncthreads();
            CB_STAMP(4);
            B.phase3(g, buf);
        }
        B.phasors(g, buf);
        __syncthreads();
        CB_STAMP(5);
        B.out(g);
        if (!next) break;
        __syncthreads();
        CB_STAMP(6);
        B.fill(buf ^ 1, pre);
        buf ^= 1;
        g = gn;
        __syncthreads();
        CB_STAMP(7);
    }
}

// chorus_block_v14 (chorus_pc.h): v13 with lores~ on its own wave (wave 7), fed through its own
// LDS region and synchronised by LDS counters, so it overlaps the next group's loads and phases.
__global__ __launch_bounds__(pc::kThreads, 1) void chorus_block_v14(ChorusArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    pc::Block B(a, lds);
    const uint32_t ngroups = (a.n + pc::kG - 1) / pc::kG;
    const uint32_t grid = gridDim.x, b = blockIdx.x;
    const uint32_t g0 = (grid & 7u) == 0 ? (b & 7u) * (grid >> 3) + (b >> 3) : b;
    if (g0 >= ngroups) return;
    if (threadIdx.x < (uint32_t)pc::kFlags) B.flags[threadIdx.x] = 0u;
    __syncthreads();                                   // the only workgroup barrier
    if (B.wave == (uint32_t)pc::kProd) {               // the consumer: lores~, round by round
        uint32_t r = 0;
        for (uint32_t g = g0; g < ngroups; g += grid, ++r) {
            B.wait_flag(1, r + 1);
            B.phase3(g, (int)(r % pc::kNBuf));
            B.signal(2, r + 1);
        }
        return;
    }
    pc::Pre pre;
    uint32_t g = g0, r = 0;
    int buf = 0;
    B.store_scalar(buf, B.load_scalar(g));
    B.producer_barrier();
    B.issue(g, buf, pre);
    B.fill(buf, pre);
    B.producer_barrier();
    while (true) {
        const uint32_t gn = g + grid;
        const bool next = gn < ngroups;
        const int nb = buf == pc::kNBuf - 1 ? 0 : buf + 1;
        uint32_t sv = 0;
        if (next) sv = B.load_scalar(gn);
        B.phase1(g, buf);
        if (next) B.store_scalar(nb, sv);
        B.producer_barrier();
        if (next) B.issue(gn, nb, pre);               // in flight until the fill below
        B.wait_flag(2, r);                            // lores~ of the previous group done: W free
        B.out(g - grid, r > 0);
        B.producer_barrier();
        B.phase2(buf);
        B.producer_barrier();
        if (B.wave == 0) B.signal(1, r + 1);          // W holds this group's taps
        if (!next) break;
        B.fill(nb, pre);
        B.producer_barrier();
        g = gn;
        buf = nb;
        ++r;
    }
    B.wait_flag(2, r + 1);
    B.out(g, true);
}

namespace {
// OLFX_CHORUS_KERNEL=11 / 13 / 14 forces that chorus kernel (A/B diagnostic)
int forced_kernel() {
    static const int k = [] {
        const char *v = std::getenv("OLFX_CHORUS_KERNEL");
        return v ? std::atoi(v) : 0;
    }();
    return k;
}
// The block-at-once kernels run only when forced: measured on MI355X (65,536 instances, same box)
// the chorus v14 takes 0.324-0.328 ms against v11's 0.234-0.241.
bool v13_geometry(uint32_t n, uint32_t psize, uint32_t csize) {
    const int f = forced_kernel();
    return (f == 13 || f == 14) && (n & 3u) == 0 && psize == cb::kPsize && csize == cb::kCsize;
}
// the block-at-once kernel for a mode: the chorus v14 (v13 when forced), the pitch-shifter v13
int block_kernel(uint32_t mode) {
    if (mode == 0) return forced_kernel() == 13 ? 13 : 14;
    return 13;
}
}  // namespace

#if OLFX_CB_STAMP
extern "C" __attribute__((visibility("default"))) int olfx_debug_stamps(uint64_t *dst, uint32_t n) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_cb_stamps), (size_t)n * 8) == hipSuccess ? 0 : -1;
}
#endif

const char *chorus_kernel_name(uint32_t n, uint32_t psize, uint32_t csize, uint32_t mode) {
    if (!v13_geometry(n, psize, csize)) return "chorus_block_v11";
    return block_kernel(mode) == 14 ? "chorus_block_v14" : "chorus_block_v13";
}

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
    if (coop && v13_geometry(a.n, a.psize, a.csize)) {
        // at most kS frames per launch (the LDS holds one block per instance); longer calls run as
        // consecutive launches, whose boundaries order each launch's ring stores before the next
        // one's ring loads
        const bool v14 = block_kernel(a.mode) == 14;
        const uint32_t gsize = v14 ? (uint32_t)pc::kG : (uint32_t)cb::kG;
        const uint32_t ngroups = (a.n + gsize - 1) / gsize;
        const uint32_t grid = min(ngroups, a.cus ? a.cus : 256u);
        for (uint32_t f0 = 0; f0 < a.n_frames; f0 += (uint32_t)cb::kS) {
            ChorusArgs sub = a;
            sub.in = a.in + (size_t)f0 * a.n;
            sub.out = a.out + (size_t)f0 * a.n;
            sub.n_frames = min((uint32_t)cb::kS, a.n_frames - f0);
            sub.t0 = a.t0 + f0;
            if (v14)
                hipLaunchKernelGGL(chorus_block_v14, dim3(grid), dim3(pc::kThreads),
                                   (size_t)pc::kLdsFloats * sizeof(float), s, sub);
            else if (a.mode == 0)
                hipLaunchKernelGGL((chorus_block_v13<true>), dim3(grid), dim3(cb::kThreads),
                                   (size_t)cb::kLdsFloats * sizeof(float), s, sub);
            else
                hipLaunchKernelGGL((chorus_block_v13<false>), dim3(grid), dim3(cb::kThreads),
                                   (size_t)cb::kLdsFloats * sizeof(float), s, sub);
        }
        return hipGetLastError();
    }
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
