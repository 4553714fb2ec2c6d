// ol_dsp_amd/csrc/chain.hip -- chorus -> pitch-shift -> dattorro in one launch (BASELINE
// configs[4]: 16,384 chains per GPU; north_star: >= 64k chorus+reverb instances).
//
// A workgroup owns 64 instances and runs the three stages as a pipeline of four single-role waves,
// one per SIMD:
//   waves 0, 1 ("C"):  the chorus stage, 32 instances x 2 channels each, input from HBM;
//   wave 2     ("P"):  the pitch-shift stage for all 64 instances, lane = instance (both channels);
//   wave 3     ("DT"): the 64 reverbs, lane = instance, output to HBM.
// Stage outputs go through LDS queues (double-buffered, [ch][16 frames][64 instances]).  Barrier
// b ends step b: the C waves produce chunk b, P runs chunk b-1, DT runs chunk b-2; nchunks + 2
// steps.  Every stage still processes each instance's frames in order, so the output is the plain
// composition of the three stages (bit-exact with the oracle's chorus -> pitch-shift -> dattorro,
// tests/test_gpu_parity.py), and the intermediates never touch HBM.
//
// The chorus and pitch stages carry their windows' lines in registers (line carry): the chorus
// stage is chorus_block_v11's (chorus_stage_l.h), the pitch stage its stereo-lane form
// (pitch_stage_s.h): per tap and instance the two aligned 128-B lines of the window live in
// registers and a chunk loads only the new line, so every ring byte is read about once (v1
// re-fetched a fresh window per tap per chunk: 296 B/frame of HBM traffic against 228.6
// algorithmic; v3: 245).  The pitch stage's next input (the chorus output of the next chunk) does
// not exist while it runs a chunk, so it stores its own input and patches it in at the next chunk.
// The reverb's pre-delay ring is the one ring laid out differently from the standalone reverb's:
// rows of 16 positions per instance (dt::PreRow), so per-instance pre-delays cost one 64-B row per
// instance and chunk instead of a 64-B request per 16 B read.
// Why four roles (history in DESIGN.md section 4): every wave of the kernel gets the reverb's
// register allocation (256 VGPR + AGPRs), so a CU holds four waves; v2 ran chorus and pitch
// in the same two waves (12.6 us per step against the reverb's 8.1) and left one SIMD idle.
#include "chorus_stage_l.h"
#include "pitch_stage_s.h"
#include "dattorro_stage.h"
#include "lds_flags.h"

namespace olfx {

namespace {
constexpr int kChainThreads = 256;            // 4 waves
constexpr int kQCh = 16 * 64 + 16;            // floats per channel of one queue buffer, padded to 16 mod 32: the two channels of a lane pair sit 16 banks apart
constexpr int kQBuf = 2 * kQCh;               // one buffer: [ch][16 frames][64 instances]
constexpr int kDepth = 3;                     // buffers per queue: a role may run 2 chunks ahead
constexpr int kChainRegion = ch::ChStageL<true>::kRegion;
constexpr int kFlags = 8;                     // LDS progress counters
constexpr int kPreLds = (17 + 8) * 64 * 4;    // DT's pre-delay staging (dt::PreRow): far [17][64], near [8][64] float4
constexpr int kChainLds = 4 * kChainRegion + 2 * kDepth * kQBuf + kFlags + kPreLds;
enum { F_C0 = 0, F_C1, F_PIN, F_POUT, F_DIN };   // chunks published by C0 / C1, taken by P, published by P, taken by DT

}  // namespace

// COOP: the C role takes its input as cooperative rows (4 x 16 B per lane and chunk instead of 16
// single floats; ChStageL COOP, chorus.hip), for n and the plane distance multiples of 4
template <bool COOP>
__global__ __launch_bounds__(kChainThreads, 1) void chain_block_v5(ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int kChunk = 16;
    const uint32_t tid = threadIdx.x;
    const uint32_t wib = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t n = a.n, nf = a.n_frames;
    const uint32_t nchunks = (nf + kChunk - 1) / kChunk;
    const uint32_t ngroups = (n + 63u) / 64u;              // 64 instances per group
    float *q1 = lds + 4 * kChainRegion;                    // chorus -> pitch   [kDepth][2 ch][16][64]
    float *q2 = q1 + kDepth * kQBuf;                       // pitch -> reverb
    uint32_t *flags = (uint32_t *)(q2 + kDepth * kQBuf);
    if (tid < kFlags) flags[tid] = 0;
    __syncthreads();                                       // the only barrier
    // A workgroup runs the groups blockIdx.x, + gridDim.x, ... back to back; its queues and
    // counters run on across them (chunk number gc = group index in the workgroup x nchunks + c),
    // so the pipeline fills and drains once per launch, not once per group.

    if (wib < 2) {
        // ---------------- C: the chorus, per (instance, channel) lane ----------------
        using StageC = ch::ChStageL<true, COOP, false>;
        StageC s1;
        const ch::Rsrc rIn = ch::rsrc(a.in, (a.plane + (uint64_t)nf * n) * 4);
        const uint32_t frame_b = n * 4u;
        for (uint32_t g = blockIdx.x, gi = 0; g < ngroups; g += gridDim.x, ++gi) {
            const uint32_t base = g * 64u, gc0 = gi * nchunks;
            const uint32_t inst0 = base + 32u * wib;
            s1.init(a.c1, lds + wib * kChainRegion, lane, inst0);
            const uint32_t io_v = s1.ch * (uint32_t)a.plane * 4u + s1.i * 4u;
            const uint32_t qcol = s1.ch * kQCh + 32u * wib + s1.j;
            // COOP rows: (frame r / 2, channel r % 2) of instances inst0 + 4 (lane % 8) .. + 3
            const uint32_t pinst = inst0 + (lane & 7u) * 4u;
            auto row_v = [&](int q, uint32_t f0) {
                const uint32_t r = StageC::coop_row(q, lane);
                return (r & 1u) * (uint32_t)a.plane * 4u + min(f0 + (r >> 1), nf - 1u) * frame_b + pinst * 4u;
            };
            float x[kChunk], xn[kChunk];
            float4 xq[4];
            int C = (int)min((uint32_t)kChunk, nf);
            if constexpr (COOP) {
#pragma unroll
                for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, 0));
                s1.begin(x, C, xq);
            } else {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) x[k] = k < C ? ch::ld1(rIn, io_v, (uint32_t)k * frame_b) : 0.f;
                s1.begin(x, C);
            }
            auto step = [&](auto par, uint32_t f0, uint32_t c) {
                C = (int)min((uint32_t)kChunk, nf - f0);
                const int Cn = f0 + kChunk < nf ? (int)min((uint32_t)kChunk, nf - f0 - kChunk) : 0;
                auto prefetch = [&]() {                       // next chunk's input, clamped, unconditional
                    if constexpr (COOP) {
#pragma unroll
                        for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, f0 + kChunk));
                    } else {
#pragma unroll
                        for (int k = 0; k < kChunk; ++k) {
                            const float v = ch::ld1(rIn, io_v, min(f0 + kChunk + (uint32_t)k, nf - 1u) * frame_b);
                            xn[k] = k < Cn ? v : 0.f;
                        }
                    }
                };
                // outputs to registers first, then to the queue: a store through a generic
                // pointer inside the stage's sink may alias the stage object (scratch).  Frames
                // past a short chunk's C are never read downstream: no zero fill (16 moves)
                float y[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) y[k] = __builtin_nondeterministic_value(0.f);
                s1.template chunk<decltype(par)::value>(x, xn, C, Cn, [&](int k, float v) { y[k] = v; }, prefetch, xq);
                const uint32_t gc = gc0 + c;
                wait_for([&] { return flag_get(flags + F_PIN) + kDepth > gc; });   // buffer gc % kDepth free
                float *q = q1 + (gc % kDepth) * kQBuf + qcol;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) q[k * 64] = y[k];
                flag_put(flags + F_C0 + wib, gc + 1);
#pragma unroll
                for (int k = 0; k < kChunk; ++k) x[k] = xn[k];
            };
            for (uint32_t f0 = 0, c = 0; f0 < nf; f0 += 2 * kChunk, c += 2) {
                step(std::integral_constant<int, 0>{}, f0, c);
                if (f0 + kChunk < nf) step(std::integral_constant<int, 1>{}, f0 + kChunk, c + 1);
            }
            s1.finish(a.c1);
        }
    } else if (wib == 2) {
        // ---------------- P: the pitch-shifter, one lane per instance (pitch_stage_s.h) ----------------
        ch::PStageS sp;
        static_assert(ch::PStageS::kRegion <= 2 * kChainRegion, "P's LDS share");
        for (uint32_t g = blockIdx.x, gi = 0; g < ngroups; g += gridDim.x, ++gi) {
            const uint32_t gc0 = gi * nchunks;
            sp.init(a.c2, lds + 2 * kChainRegion, lane, g * 64u);
            int C = (int)min((uint32_t)kChunk, nf);
            sp.begin(C);
            auto step = [&](auto par, uint32_t f0, uint32_t c) {
                constexpr int P = decltype(par)::value;
                C = (int)min((uint32_t)kChunk, nf - f0);
                const int Cn = f0 + kChunk < nf ? (int)min((uint32_t)kChunk, nf - f0 - kChunk) : 0;
                const uint32_t gc = gc0 + c;
                wait_for([&] { return flag_get(flags + F_C0) > gc && flag_get(flags + F_C1) > gc; });
                const float *qi = q1 + (gc % kDepth) * kQBuf + lane;
                float2 x[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) x[k] = make_float2(qi[k * 64], qi[kQCh + k * 64]);
                flag_put(flags + F_PIN, gc + 1);              // (the release waits for these reads)
                // (frames past a short chunk's C are never read downstream: no zero fill)
                float2 y[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) y[k] = make_float2(__builtin_nondeterministic_value(0.f), __builtin_nondeterministic_value(0.f));
                sp.template chunk<P>(x, C, Cn, [&](int k, float2 v) { y[k] = v; });
                wait_for([&] { return flag_get(flags + F_DIN) + kDepth > gc; });
                float *qo = q2 + (gc % kDepth) * kQBuf + lane;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) { qo[k * 64] = y[k].x; qo[kQCh + k * 64] = y[k].y; }
                flag_put(flags + F_POUT, gc + 1);
            };
            for (uint32_t f0 = 0, c = 0; f0 < nf; f0 += 2 * kChunk, c += 2) {
                step(std::integral_constant<int, 0>{}, f0, c);
                if (f0 + kChunk < nf) step(std::integral_constant<int, 1>{}, f0 + kChunk, c + 1);
            }
            sp.finish(a.c2);
        }
    } else {
        // ---------------- DT: the reverb, lane = instance, input from the queue ----------------
        // the network in one wave over the pre-delay ring in rows (dt::rows_network, dt::PreRow)
        float4 *const stage = (float4 *)(flags + kFlags);
        for (uint32_t g = blockIdx.x, gi = 0; g < ngroups; g += gridDim.x, ++gi) {
            const uint32_t i = g * 64u + lane, gc0 = gi * nchunks;   // < d.n (padded to 64)
            const bool valid = i < n;
            dt::rows_network<false>(
                a.d, g, lane, nf, stage,
                [&](uint32_t c, uint32_t, uint32_t, float (&xm)[kChunk]) {   // the chunk's mono input, (l + r) / 2
                    const uint32_t gc = gc0 + c;
                    wait_for([&] { return flag_get(flags + F_POUT) > gc; });
                    const float *q = q2 + (gc % kDepth) * kQBuf + lane;
#pragma unroll
                    for (int k = 0; k < kChunk; ++k) xm[k] = (q[k * 64] + q[kQCh + k * 64]) / 2;
                    flag_put(flags + F_DIN, gc + 1);
                },
                [&](uint32_t f, const float (&o_l)[4], const float (&o_r)[4]) {
                    if (valid) {
#pragma unroll
                        for (int k = 0; k < 4; ++k) {
                            a.out[(size_t)(f + k) * n + i] = o_l[k];
                            a.out[a.plane + (size_t)(f + k) * n + i] = o_r[k];
                        }
                    }
                });
        }
    }
}

hipError_t launch_chain(const ChainArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.n_frames & 3u) || (a.c1.t0 & 3u) || (a.d.t0 & 3u) || a.d.n < ((a.n + 63u) & ~63u)) return hipErrorInvalidValue;
    if ((uint64_t)a.n * 2 * a.c1.csize * 4 >= (1ull << 32) || (a.plane + (uint64_t)a.n_frames * a.n) * 4 >= (1ull << 32))
        return hipErrorInvalidValue;
    // one workgroup per CU (LDS and registers allow no more), each running its groups back to back;
    // the CU count is the engine's (olfx_create), so concurrent engines share no launcher state
    if (a.cus == 0) return hipErrorInvalidValue;
    const uint32_t groups = (a.n + 63u) / 64u;
    const uint32_t blocks = groups < a.cus ? groups : a.cus;
    const bool coop = (a.n & 3u) == 0 && (a.plane & 3u) == 0 && (((uintptr_t)a.in | (uintptr_t)a.out) & 15u) == 0;
    if (coop) hipLaunchKernelGGL(chain_block_v5<true>, dim3(blocks), dim3(kChainThreads), (size_t)kChainLds * sizeof(float), s, a);
    else hipLaunchKernelGGL(chain_block_v5<false>, dim3(blocks), dim3(kChainThreads), (size_t)kChainLds * sizeof(float), s, a);
    return hipGetLastError();
}

}  // namespace olfx
