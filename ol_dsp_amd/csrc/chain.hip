// ol_dsp_amd/csrc/chain.hip -- chorus -> pitch-shift -> dattorro in one launch (BASELINE
// configs[4]: 16,384 chains per GPU).
//
// A workgroup owns 64 instances and runs the three stages as a pipeline of waves:
//   waves 0, 1 ("CP"): 32 instances x 2 channels each; every lane runs the chorus stage and then
//                      the pitch-shift stage on the chorus output, chunk by chunk (16 frames);
//   wave 2     ("DT"): the 64 reverbs, lane = instance, fed through LDS.
// Step s: the CP waves produce chunk s into queue buffer s & 1 while the DT wave consumes chunk
// s-1 from the other buffer; one workgroup barrier per step.  Every stage still processes each
// instance's frames in order, so the output is the plain composition of the three stages
// (bit-exact with the oracle's chorus -> pitch-shift -> dattorro, tests/test_gpu_parity.py).
// The intermediates never touch HBM, and the three stages run concurrently on different SIMDs,
// where three separate launches each filled only part of the chip at 16,384 instances.
#include "chorus_stage.h"
#include "dattorro_stage.h"

namespace olfx {

namespace {
constexpr int kChainThreads = 192;            // 3 waves
constexpr int kQCh = 16 * 64 + 32;            // floats per channel of one queue buffer (padded)
constexpr int kQBuf = 2 * kQCh;               // one buffer: [ch][16 frames][64 instances]
constexpr int kChainLds = 4 * ch::ChStage<true>::kRegion + 2 * kQBuf;   // 2 CP waves x 2 regions
}  // namespace

__global__ __launch_bounds__(kChainThreads, 1) void chain_block_v1(ChainArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    constexpr int kChunk = 16;
    const uint32_t tid = threadIdx.x;
    const uint32_t wib = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t lane = tid & 63u;
    const uint32_t base = blockIdx.x * 64u;               // first instance of the workgroup
    const uint32_t n = a.n, nf = a.n_frames;
    const uint32_t nchunks = (nf + kChunk - 1) / kChunk;
    float *queue = lds + 4 * ch::ChStage<true>::kRegion;   // [2 bufs][2 ch][16][64]

    if (wib < 2) {
        // ---------------- CP: chorus then pitch-shift, per (instance, channel) lane ----------------
        ch::ChStage<true> s1;
        ch::ChStage<false> s2;
        s1.init(a.c1, lds + (2 * wib) * ch::ChStage<true>::kRegion, lane, base + 32u * wib);
        s2.init(a.c2, lds + (2 * wib + 1) * ch::ChStage<true>::kRegion, lane, base + 32u * wib);
        const ch::Rsrc rIn = ch::rsrc(a.in, (a.plane + (uint64_t)nf * n) * 4);
        const uint32_t io_v = s1.ch * (uint32_t)a.plane * 4u + s1.i * 4u, frame_b = n * 4u;
        const uint32_t qcol = s1.ch * kQCh + 32u * wib + s1.j;   // this lane's queue column

        float x[kChunk], xn[kChunk], y1[kChunk];
        int C = (int)min((uint32_t)kChunk, nf);
#pragma unroll
        for (int k = 0; k < kChunk; ++k) x[k] = k < C ? ch::ld1(rIn, io_v, (uint32_t)k * frame_b) : 0.f;
        s1.begin(x, C);
        // chunk c: stage 1 on x, stage 2 on stage 1's output, published into queue buffer c & 1.
        // Chunk 0 is peeled: stage 2's begin() needs stage 1's first output (a begin() inside the
        // loop kept stage 2's state in scratch memory).
        auto step = [&](uint32_t c, auto first_tag) {
            constexpr bool FIRST = decltype(first_tag)::value;
            const uint32_t f0 = c * kChunk;
            C = (int)min((uint32_t)kChunk, nf - f0);
            const int Cn = f0 + kChunk < nf ? (int)min((uint32_t)kChunk, nf - f0 - kChunk) : 0;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {   // next chunk's input in flight (clamped, unconditional)
                const float v = ch::ld1(rIn, io_v, min(f0 + kChunk + (uint32_t)k, nf - 1u) * frame_b);
                xn[k] = k < Cn ? v : 0.f;
            }
#pragma unroll
            for (int k = 0; k < kChunk; ++k) y1[k] = 0.f;
            s1.chunk(x, C, Cn, [&](int k, float v) { y1[k] = v; });
            if (FIRST) s2.begin(y1, C);
            float *q = queue + (c & 1u) * kQBuf + qcol;
            // stage 2's output goes to registers first and then to the queue: a store through a
            // generic pointer inside the stage's sink may alias the stage object, which then
            // stays in scratch memory
            float y2[kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; ++k) y2[k] = 0.f;
            s2.chunk(y1, C, Cn, [&](int k, float v) { y2[k] = v; });
#pragma unroll
            for (int k = 0; k < kChunk; ++k) q[k * 64] = y2[k];
            __syncthreads();                                  // chunk c published to the DT wave
#pragma unroll
            for (int k = 0; k < kChunk; ++k) x[k] = xn[k];
        };
        step(0, std::true_type{});
        for (uint32_t c = 1; c < nchunks; ++c) step(c, std::false_type{});
        __syncthreads();                                      // the DT wave's last step
        s1.finish(a.c1);
        s2.finish(a.c2);
    } else {
        // ---------------- DT: the reverb, lane = instance, input from the queue ----------------
        const uint32_t i = base + lane;                       // < d.n (padded to 64)
        DT_STAGE(a.d, i);
        const uint32_t t0 = a.d.t0;
        dt_prime(t0);
        const bool valid = i < n;
        __syncthreads();                                      // chunk 0 published
        for (uint32_t c = 0; c < nchunks; ++c) {
            const uint32_t f0 = c * kChunk;
            const uint32_t C = min((uint32_t)kChunk, nf - f0);
            const float *q = queue + (c & 1u) * kQBuf + lane;
            for (uint32_t s = 0; s < C; s += 4) {
                float xin[4], o_l[4], o_r[4];
#pragma unroll
                for (int k = 0; k < 4; ++k) xin[k] = (q[(s + k) * 64] + q[kQCh + (s + k) * 64]) / 2;
                dt_step(t0 + f0 + s, f0 + s + 4 < nf, xin, o_l, o_r);
                if (valid) {
#pragma unroll
                    for (int k = 0; k < 4; ++k) {
                        a.out[(size_t)(f0 + s + k) * n + i] = o_l[k];
                        a.out[a.plane + (size_t)(f0 + s + k) * n + i] = o_r[k];
                    }
                }
            }
            __syncthreads();                                  // chunk c consumed; c + 1 published
        }
        dt_finish();
    }
}

hipError_t launch_chain(const ChainArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.n_frames & 3u) || (a.c1.t0 & 3u) || (a.d.t0 & 3u) || a.d.n < ((a.n + 63u) & ~63u)) return hipErrorInvalidValue;
    if ((uint64_t)a.n * 2 * a.c1.csize * 4 >= (1ull << 32) || (a.plane + (uint64_t)a.n_frames * a.n) * 4 >= (1ull << 32))
        return hipErrorInvalidValue;
    const uint32_t blocks = (a.n + 63u) / 64u;
    hipLaunchKernelGGL(chain_block_v1, dim3(blocks), dim3(kChainThreads), (size_t)kChainLds * sizeof(float), s, a);
    return hipGetLastError();
}

}  // namespace olfx
