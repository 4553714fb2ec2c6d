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
// pre-delays differ) keeps that ring instance-major and runs dattorro_predelay_v2 ahead of the
// block: each instance's ring is read and written in whole 128-B lines (below) and the network
// gets its pre-delayed block as a coalesced stream (PreBlock).  The network itself then reads no
// input and writes no pre-delay ring.  Measured (65,536 instances, random pre-delays): pre-pass
// 0.073 ms + network 0.479 ms = 0.552 ms against the uniform reverb's 0.514 ms (1.07x).
#include "dattorro_stage.h"
#include "chorus_stage.h"

namespace olfx {

// Uniform mode: IN1 (the second input diffuser, 128 positions, verb.cpp:180) is read and written
// in LDS for the launch (LdsTap): its 8 B/frame of ring traffic become 512 B in and out per
// instance and launch (rocprof, same box: 571 -> 557 us).  Gather mode keeps IN1 in HBM: with the
// LDS ring its network measured 527 -> 554 us.
template <bool GATHER>
__global__ __launch_bounds__(64, 1) void dattorro_block_v4(DattorroArgs a) {
    __shared__ float4 in1_ring[GATHER ? 1u : kDtSize[DT_IN1] / 4u * 64u];      // 32 KB: [group][lane]
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const size_t plane = a.plane;
    const bool stereo = a.in_ch == 2;

    using Pre = typename std::conditional<GATHER, olfx::dt::PreBlock, olfx::dt::PreTap>::type;
    using In1 = typename std::conditional<GATHER, olfx::dt::Tap<DT_IN1, 107, 0>, olfx::dt::LdsTap<DT_IN1, 107>>::type;
    DT_STAGE_X(a, i, Pre, (In1));
    if constexpr (!GATHER) {
        in1.lds = in1_ring + threadIdx.x;
        in1.lds_in(a, i);
    }
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
    if constexpr (!GATHER) in1.lds_out(a, i);
}

constexpr uint32_t kPreSize = kDtSize[DT_PRE];

// dattorro_predelay_v2: gather mode's pre-pass in whole 128-B lines (round 4's first form, one lane
// per instance in 4-frame chunks moving 16-B pieces -- 64 lines per instruction, each line touched
// by 8 chunks -- made the mode 0.78 ms against 0.54 uniform and is gone).  One wave per workgroup = 64 instances,
// 32-frame chunks aligned to the ring's lines (chunk positions [T, T + 32), T % 32 == 0):
//   - a chunk's ring write is exactly one line per instance, stored cooperatively (8 lanes x 16 B
//     per line, 8 lines per instruction) from the LDS history `hist`;
//   - its pre-delayed reads [T - d, T - d + 32) lie in two lines Lq = (T - d) / 32 and Lq + 1; the
//     window `win` holds both in LDS, and each chunk loads only the next one (Lq + 2, cooperatively,
//     one chunk ahead), since the window advances by exactly one line per chunk;
//   - positions >= T - 32 (d <= k + 32) come from `hist`, which holds the previous chunk's and this
//     chunk's inputs.  The line prefetched during chunk c was issued before chunk c's ring store:
//     every earlier chunk's store precedes it, so its only possibly stale positions are chunk c's
//     own line [T, T + 32) -- when it is that line, hist's copy replaces it.
// Frames outside [t0, t0 + n_frames) in the first and last chunks are neither stored nor output;
// the first chunk's history positions [T, t0) and [T - 32, T) are loaded into `hist` from the ring.
// The pre-delayed block goes out as [F/4][n][4] (coalesced).
namespace {
constexpr uint32_t kPdLine = 32;                   // positions per 128-B line
constexpr uint32_t kPdLines = kPreSize / kPdLine;   // 256
constexpr uint32_t kPdRow = 65;                    // LDS floats per instance row (odd: lanes spread over banks)
}

__global__ __launch_bounds__(64) void dattorro_predelay_v2(DattorroArgs a) {
    __shared__ float hist[64 * kPdRow];            // [instance][P & 63]: inputs of positions [T - 32, T + 32)
    __shared__ float win[64 * kPdRow];             // [instance][P & 63]: ring lines Lq, Lq + 1
    const uint32_t lane = threadIdx.x, n = a.n, F = a.n_frames, t0 = a.t0;
    const uint32_t i0 = blockIdx.x * 64u, i = i0 + lane, nv = min(n - i0, 64u);
    const bool live = i < n;
    const bool stereo = a.in_ch == 2;
    const uint32_t d = (uint32_t)a.coef[DTC_PREDELAY * n + min(i, n - 1u)];
    // cooperative line accesses: in instruction m, lane L serves instance 8 m + L / 8, piece L % 8
    const uint32_t pc = lane & 7u;
    uint32_t dj[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) dj[m] = (uint32_t)a.coef[DTC_PREDELAY * n + min(i0 + 8u * m + (lane >> 3), n - 1u)];
    const ch::Rsrc rRing = ch::rsrc(a.pre_im + (size_t)i0 * kPreSize, (uint64_t)nv * kPreSize * 4u);
    auto line_off = [&](int m, uint32_t line) {    // byte offset of piece pc of instance 8 m + L / 8's line
        const uint32_t j = 8u * (uint32_t)m + (lane >> 3);
        return j < nv ? j * kPreSize * 4u + (line & (kPdLines - 1u)) * 128u + pc * 16u : 0xFFFFFFF0u;
    };
    auto to_lds = [&](float *dst, int m, uint32_t line, float4 v) {   // piece -> row slot (line & 1) * 32 + 4 pc
        float *r = dst + (8u * (uint32_t)m + (lane >> 3)) * kPdRow + (line & 1u) * kPdLine + 4u * pc;
        r[0] = v.x; r[1] = v.y; r[2] = v.z; r[3] = v.w;
    };
    auto wave_sync = [] {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    // input frame rows: f = T + k - t0, loaded when 0 <= f < F (else 0 through an out-of-range offset)
    const ch::Rsrc rIn0 = ch::rsrc(a.in, ((uint64_t)F * n) * 4u);
    const ch::Rsrc rIn1 = ch::rsrc(stereo ? a.in + a.plane : a.in, ((uint64_t)F * n) * 4u);
    auto load_x = [&](uint32_t T, float (&x0)[kPdLine], float (&x1)[kPdLine]) {
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const uint32_t f = T + k - t0;                 // wraps above F when T + k < t0
            const uint32_t off = f < F && live ? (f * n + i) * 4u : 0xFFFFFFF0u;
            x0[k] = ch::ld1(rIn0, off, 0);
            x1[k] = ch::ld1(rIn1, off, 0);
        }
    };
    const uint32_t T0 = t0 & ~(kPdLine - 1u);
    const uint32_t nch = (t0 + F - T0 + kPdLine - 1u) / kPdLine;
    // history lines T0 / 32 - 1 and T0 / 32, window lines Lq and Lq + 1 of the first chunk
    {
        float4 h[2][8], w[2][8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            h[0][m] = ch::ld4(rRing, line_off(m, T0 / kPdLine - 1u));
            h[1][m] = ch::ld4(rRing, line_off(m, T0 / kPdLine));
            w[0][m] = ch::ld4(rRing, line_off(m, (T0 - dj[m]) / kPdLine));
            w[1][m] = ch::ld4(rRing, line_off(m, (T0 - dj[m]) / kPdLine + 1u));
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            to_lds(hist, m, T0 / kPdLine - 1u, h[0][m]);
            to_lds(hist, m, T0 / kPdLine, h[1][m]);
            to_lds(win, m, (T0 - dj[m]) / kPdLine, w[0][m]);
            to_lds(win, m, (T0 - dj[m]) / kPdLine + 1u, w[1][m]);
        }
    }
    float x0[kPdLine], x1[kPdLine];
    load_x(T0, x0, x1);
    const ch::Rsrc rBlk = ch::rsrc(a.pre_block, (uint64_t)F * n * 4u);
    float *hrow = hist + lane * kPdRow, *wrow = win + lane * kPdRow;
    for (uint32_t c = 0; c < nch; ++c) {
        const uint32_t T = T0 + c * kPdLine;
        // the next chunk's window line and inputs, issued before this chunk's ring store
        float4 nl[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) nl[m] = ch::ld4(rRing, line_off(m, (T - dj[m]) / kPdLine + 2u));
        float n0[kPdLine], n1[kPdLine];
        load_x(T + kPdLine, n0, n1);
        // this chunk's mono input (l + r) / 2 into the history (positions before t0 keep the ring's)
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const float xm = stereo ? (x0[k] + x1[k]) / 2 : x0[k];
            if (T + k - t0 < F) hrow[(T + k) & 63u] = xm;
        }
        wave_sync();
        // the pre-delayed samples: positions T + k - d, from the history when >= T - 32
        float v[kPdLine];
        const uint32_t q = T - d;
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) {
            const float *src = d <= k + kPdLine ? hrow + ((T + k - d) & 63u) : wrow + ((q + k) & 63u);
            v[k] = *src;
        }
#pragma unroll
        for (uint32_t g = 0; g < kPdLine / 4u; ++g) {
            const uint32_t f = T + 4u * g - t0;            // a group is wholly inside or outside (t0 % 4 == 0)
            ch::st4(rBlk, f < F && live ? ((f >> 2) * n + i) * 16u : 0xFFFFFFF0u,
                make_float4(v[4 * g], v[4 * g + 1], v[4 * g + 2], v[4 * g + 3]));
        }
        // the chunk's ring line, cooperatively from the history (pieces outside the block dropped)
        float4 hv[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const float *r = hist + (8u * (uint32_t)m + (lane >> 3)) * kPdRow + (T & 63u) + 4u * pc;
            hv[m] = make_float4(r[0], r[1], r[2], r[3]);
            const uint32_t f = T + 4u * pc - t0;
            ch::st4(rRing, f < F ? line_off(m, T / kPdLine) : 0xFFFFFFF0u, hv[m]);
        }
        wave_sync();
        // the window advances one line: Lq + 2 replaces Lq (its reads are done); if Lq + 2 is this
        // chunk's own line, its prefetch predates the store above: hist's copy instead
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t l2 = (T - dj[m]) / kPdLine + 2u;
            to_lds(win, m, l2, ((l2 ^ (T / kPdLine)) & (kPdLines - 1u)) == 0u ? hv[m] : nl[m]);
        }
#pragma unroll
        for (uint32_t k = 0; k < kPdLine; ++k) { x0[k] = n0[k]; x1[k] = n1[k]; }
        wave_sync();
    }
}

// dattorro_predelay_v3: the whole call's block (<= 256 frames) at once.  The pass has no serial
// dependence inside a block: every pre-delayed sample x[t - d] is either this block's own input
// (d <= f, from LDS) or a ring position written before the block (d > f), so v2's chunk-by-chunk
// chain of line loads becomes three phases per 32-instance workgroup (4 waves, 66 KB of LDS: two
// workgroups per CU):
//   1. the block's input rows (32 instances = 128 B per row and channel, 16-B pieces, all 16 loads
//      in flight at once), mono (l + r) / 2 transposed into `mono` [instance][frame];
//   2. per instance (wave-uniform), lanes = 64 consecutive frames: the ring reads t - d of one
//      instance are consecutive positions of its instance-major row (two or three 128-B lines per
//      instruction); d <= f reads `mono` instead; results into `outv` [instance][frame];
//   3. the pre-delayed block out of `outv` as [F/4][n][4] rows (512 B per frame group) and the
//      block's mono input into the ring (1 KB per instance), after every read of phase 2: a
//      pre-delay above 8192 - F reads a slot this block overwrites, and reads it first, as
//      DelayBuffer_process does (verb.cpp:107-110).
// Needs 16-B aligned input rows (n % 4 == 0, plane % 4 == 0, in 16-B aligned); v2 otherwise.
namespace {
constexpr uint32_t kPd3J = 32;                      // instances per workgroup
constexpr uint32_t kPd3F = 256;                     // frames per launch (the engine splits at 256)
constexpr uint32_t kPd3Row = kPd3F + 1;             // LDS floats per instance row (odd)
}

__global__ __launch_bounds__(256) void dattorro_predelay_v3(DattorroArgs a) {
    __shared__ float mono[kPd3J * kPd3Row];
    __shared__ float outv[kPd3J * kPd3Row];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const uint32_t n = a.n, F = a.n_frames, t0 = a.t0;
    const uint32_t i0 = blockIdx.x * kPd3J, nv = min(n - i0, kPd3J);
    const bool stereo = a.in_ch == 2;
    constexpr uint32_t kOob = 0xFFFFFFF0u;
    {   // 1. input rows: piece pc (instances 4 pc .. 4 pc + 3) of rows r0 + 32 m
        const ch::Rsrc rIn0 = ch::rsrc(a.in, (uint64_t)F * n * 4u);
        const ch::Rsrc rIn1 = ch::rsrc(stereo ? a.in + a.plane : a.in, (uint64_t)F * n * 4u);
        const uint32_t pc = tid & 7u, r0 = tid >> 3;
        float4 l[8], r[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t f = r0 + 32u * (uint32_t)m;
            const uint32_t off = f < F && 4u * pc < nv ? (f * n + i0 + 4u * pc) * 4u : kOob;
            l[m] = ch::ld4(rIn0, off);
            r[m] = stereo ? ch::ld4(rIn1, off) : l[m];
        }
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            float *dst = mono + 4u * pc * kPd3Row + r0 + 32u * (uint32_t)m;
            dst[0] = stereo ? (l[m].x + r[m].x) / 2 : l[m].x;
            dst[kPd3Row] = stereo ? (l[m].y + r[m].y) / 2 : l[m].y;
            dst[2 * kPd3Row] = stereo ? (l[m].z + r[m].z) / 2 : l[m].z;
            dst[3 * kPd3Row] = stereo ? (l[m].w + r[m].w) / 2 : l[m].w;
        }
    }
    __syncthreads();
    const ch::Rsrc rRing = ch::rsrc(a.pre_im + (size_t)i0 * kPreSize, (uint64_t)nv * kPreSize * 4u);
    {   // 2. wave w: instances 8 w .. 8 w + 7, lane = frame within each 64-frame group
        float rv[8][4];
        uint32_t dj[8];
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const uint32_t j = 8u * w + (uint32_t)jj;
            dj[jj] = (uint32_t)a.coef[DTC_PREDELAY * n + min(i0 + j, n - 1u)];   // exact integer 0..8191
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint32_t f = 64u * (uint32_t)g + lane;
                const uint32_t off = j < nv && f < F && dj[jj] > f
                                         ? (j * kPreSize + ((t0 + f - dj[jj]) & (kPreSize - 1u))) * 4u : kOob;
                rv[jj][g] = ch::ld1(rRing, off, 0);
            }
        }
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const uint32_t j = 8u * w + (uint32_t)jj;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const uint32_t f = 64u * (uint32_t)g + lane;
                outv[j * kPd3Row + f] = dj[jj] <= f ? mono[j * kPd3Row + f - dj[jj]] : rv[jj][g];
            }
        }
    }
    __syncthreads();
    {   // 3a. the pre-delayed block: frame groups gs + 8 m, instance j
        const ch::Rsrc rBlk = ch::rsrc(a.pre_block, (uint64_t)F * n * 4u);
        const uint32_t j = tid & 31u, gs = tid >> 5;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const uint32_t g = gs + 8u * (uint32_t)m;
            const float *src = outv + j * kPd3Row + 4u * g;
            ch::st4(rBlk, 4u * g < F && j < nv ? (g * n + i0 + j) * 16u : kOob,
                    make_float4(src[0], src[1], src[2], src[3]));
        }
    }
    {   // 3b. the block's mono input into the ring: wave w's instances, lane = 4-position piece
#pragma unroll
        for (int jj = 0; jj < 8; ++jj) {
            const uint32_t j = 8u * w + (uint32_t)jj;
            const float *src = mono + j * kPd3Row + 4u * lane;
            ch::st4(rRing, 4u * lane < F && j < nv ? (j * kPreSize + ((t0 + 4u * lane) & (kPreSize - 1u))) * 4u : kOob,
                    make_float4(src[0], src[1], src[2], src[3]));
        }
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

// v3 when the rows allow it (16-B aligned input rows), else v2
int predelay_kernel(uint32_t n, uint64_t plane, const float *in) {
    return n % 4u == 0u && plane % 4u == 0u && ((uintptr_t)in & 15u) == 0u ? 3 : 2;
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
        // per-workgroup ring resources: 64 instances x 32 KB; inputs and the block by 32-bit offsets
        if ((uint64_t)a.n_frames * a.n * 4u >= (1ull << 32)) return hipErrorInvalidValue;
        const int v = predelay_kernel(a.n, a.plane, a.in);
        if (v == 3 && a.n_frames > kPd3F) return hipErrorInvalidValue;   // the engine splits at 256
        if (v == 2)
            hipLaunchKernelGGL(dattorro_predelay_v2, dim3((a.n + 63) / 64), dim3(64), 0, s, a);
        else
            hipLaunchKernelGGL(dattorro_predelay_v3, dim3((a.n + kPd3J - 1) / kPd3J), dim3(256), 0, s, a);
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
