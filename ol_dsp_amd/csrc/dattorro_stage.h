// ol_dsp_amd/csrc/dattorro_stage.h -- the Dattorro plate reverb as a per-lane device stage.
//
// Reference: /root/reference/libs/dattorro-verb/verb.cpp:258-325 (DattorroVerb_process +
// getLeft/getRight) with the fxlib glue's (l+r)/2 input (modules/fxlib/ReverbFx.cpp:11-27).
//
// Layout: ring l is [kDtSize[l]/4][n][4] floats -- groups of 4 consecutive positions of one
// instance, instances fastest.  All instances of an engine share the stream time t and every tap
// delay, so a wave reading one tap for a 4-frame chunk issues ONE 16-B-per-lane load that covers
// 1 KB contiguous.  The block is processed in 4-frame chunks aligned to t % 4 == 0:
//   * a tap with delay d reads positions t0 - d + k (k = 0..3) = a window of 2 groups shifted by
//     s = (-d) & 3, a compile-time constant for the 24 fixed taps: each chunk loads ONE new group
//     per tap and carries the other from the previous chunk (every ring byte is read once);
//   * the group for the next chunk is prefetched before the current chunk's serial recurrence,
//     so ~30 x 1 KB loads per wave are in flight while it computes (1 wave per SIMD at 65,536
//     instances; latency hiding comes from this ILP, not occupancy);
//   * the 13 ring writes of a chunk leave as one 16-B store per line.
// Every fixed delay is >= 107 samples, so no chunk reads a group written by itself or by its
// predecessor.  The two modulated all-pass taps and the per-instance pre-delay tap are carried
// the same way (one new group per chunk; see ModTap / PreTap), so every ring byte is read once.
// Groups written by earlier chunks of this launch are read back by the lane that wrote them, in
// program order.  No MFMA: scalar recurrences.
// Bound: HBM.
#pragma once
#include <type_traits>

#include "olfx_internal.h"

namespace olfx {
namespace dt {

__device__ __forceinline__ float el(const float4 &v, int e) {
    return e == 0 ? v.x : (e == 1 ? v.y : (e == 2 ? v.z : v.w));
}

// v[k] = element s + k of the 8-float window (a0..a3, b0..b2), s in 0..3 (runtime, uniform or per
// lane): a shift by 2 on bit 1, then by 1 on bit 0 -- 9 v_cndmask.  The two bits pass through an
// empty asm: a chain of `s == 0 ? .. : s == 1 ? ..` selects was rebuilt by the compiler into a
// switch on s, i.e. an exec-mask branch tree per element (about 25 instructions each, every merge
// a loss of waitcnt precision for the prefetch in flight)
__device__ __forceinline__ void shift4(uint32_t s, float a0, float a1, float a2, float a3, float b0, float b1,
                                       float b2, float (&v)[4]) {
    uint32_t hi = s & 2u, lo = s & 1u;
    asm volatile("" : "+v"(hi), "+v"(lo));
    const float t0 = hi ? a2 : a0, t1 = hi ? a3 : a1, t2 = hi ? b0 : a2, t3 = hi ? b1 : a3, t4 = hi ? b2 : b0;
    v[0] = lo ? t1 : t0;
    v[1] = lo ? t2 : t1;
    v[2] = lo ? t3 : t2;
    v[3] = lo ? t4 : t3;
}
__device__ __forceinline__ void shift4(uint32_t s, const float4 &a, const float4 &b, float (&v)[4]) {
    shift4(s, a.x, a.y, a.z, a.w, b.x, b.y, b.z, v);
}

template <int L>
__device__ __forceinline__ float4 *grp(const DattorroArgs &a, uint32_t g, uint32_t i) {
    constexpr uint32_t gm = kDtSize[L] / 4u - 1u;
    return (float4 *)a.ring[L] + ((size_t)(g & gm) * a.n + i);
}
// The same for a wave-uniform g: the group's row start is uniform (scalar arithmetic) and the
// lane's 16 B an unsigned 32-bit offset from it, so the access is a global load/store with an SGPR
// base and a VGPR offset -- no 64-bit vector address add per access
template <int L>
__device__ __forceinline__ float4 *grpu(const DattorroArgs &a, uint32_t g, uint32_t i) {
    constexpr uint32_t gm = kDtSize[L] / 4u - 1u;
    char *row = (char *)a.ring[L] + (size_t)(g & gm) * a.n * 16u;
    return (float4 *)(row + (uint32_t)(i * 16u));
}

// A fixed tap: delay D, read at t + OFF (OFF = 1 for the output taps, verb.cpp:298,302-325).
template <int L, uint32_t D, uint32_t OFF>
struct Tap {
    static constexpr uint32_t S = (OFF - D) & 3u;     // shift of the window inside its groups
    float4 cur, nxt, pre;
    __device__ __forceinline__ static uint32_t g0(uint32_t t0) { return (t0 + OFF - D) >> 2; }
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        cur = *grpu<L>(a, g0(t0), i);
        if (S) nxt = *grpu<L>(a, g0(t0) + 1u, i);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        pre = *grpu<L>(a, g0(t0) + (S ? 2u : 1u), i);
    }
    __device__ __forceinline__ float get(int k) const {
        return (int)S + k < 4 ? el(cur, (int)S + k) : el(nxt, (int)S + k - 4);
    }
    __device__ __forceinline__ void advance() {
        if (S) { cur = nxt; nxt = pre; } else { cur = pre; }
    }
    // the ring's write, for a ring with this one tap (IN1)
    __device__ __forceinline__ void write(const DattorroArgs &a, uint32_t gw, uint32_t i, float4 v) { *grpu<L>(a, gw, i) = v; }
};

// A fixed tap whose whole ring lives in LDS for the launch (the standalone reverb's IN1, 128
// positions: 32 groups x 64 lanes x 16 B = 32 KB per wave): the kernel copies the ring in before the
// first chunk and back after the last (lds_in / lds_out), and the chunks read and write LDS only.
// The lane's groups sit at lds[(g & 31) * 64 + lane] (a wave's accesses: 1 KB contiguous).
template <int L, uint32_t D>
struct LdsTap {
    static constexpr uint32_t S = (0u - D) & 3u;
    static constexpr uint32_t kGroups = kDtSize[L] / 4u;
    float4 *lds;                                      // this lane's column: lds[g * 64]
    float4 cur, nxt, pre;
    __device__ __forceinline__ static uint32_t g0(uint32_t t0) { return (t0 - D) >> 2; }
    __device__ __forceinline__ float4 &at(uint32_t g) const { return lds[(g & (kGroups - 1u)) * 64u]; }
    __device__ __forceinline__ void lds_in(const DattorroArgs &a, uint32_t i) {
#pragma unroll
        for (uint32_t g = 0; g < kGroups; ++g) at(g) = *grpu<L>(a, g, i);
    }
    __device__ __forceinline__ void lds_out(const DattorroArgs &a, uint32_t i) const {
#pragma unroll
        for (uint32_t g = 0; g < kGroups; ++g) *grpu<L>(a, g, i) = at(g);
    }
    __device__ __forceinline__ void prime(const DattorroArgs &, uint32_t t0, uint32_t) {
        cur = at(g0(t0));
        if (S) nxt = at(g0(t0) + 1u);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &, uint32_t t0, uint32_t) {
        pre = at(g0(t0) + (S ? 2u : 1u));
    }
    __device__ __forceinline__ float get(int k) const {
        return (int)S + k < 4 ? el(cur, (int)S + k) : el(nxt, (int)S + k - 4);
    }
    __device__ __forceinline__ void advance() {
        if (S) { cur = nxt; nxt = pre; } else { cur = pre; }
    }
    __device__ __forceinline__ void write(const DattorroArgs &, uint32_t gw, uint32_t, float4 v) { at(gw) = v; }
};

// A modulated tank all-pass tap (verb.cpp:262-270): delay D + ex(t), with ex wave-uniform and
// constant for 512 chunks at a time.  The window of a chunk is 2 groups from its start q; while ex
// is constant the next window starts 4 later, so its first group is this chunk's second one and
// only one new group is loaded (as the fixed taps).  At a step of ex the first group is loaded
// too.  That load is never under a branch (a load under a branch made the compiler wait for every
// outstanding load, the whole prefetch, at the merge): it is a buffer load whose offset is past
// the end of the ring when the group is carried -- no memory access, the returned zeros unused.
template <int L, uint32_t D>
struct ModTap {
    float c0, c1, c2, c3, n0, n1, n2, n3;             // this chunk's window
    float p0, p1, p2, p3, r0, r1, r2, r3;             // the next chunk's groups, in flight
    float v[4];
    uint32_t q, qn;                                   // window start of this / the next chunk
    bool carry;                                       // next window's first group = n0..n3
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        q = t0 - (D + dt_ap1_extra(t0 & 0xFFFFu));
        const float4 g0 = *grpu<L>(a, q >> 2, i), g1 = *grpu<L>(a, (q >> 2) + 1u, i);
        c0 = g0.x; c1 = g0.y; c2 = g0.z; c3 = g0.w;
        n0 = g1.x; n1 = g1.y; n2 = g1.z; n3 = g1.w;
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        const uint32_t t0n = t0 + 4u;
        qn = t0n - (D + dt_ap1_extra(t0n & 0xFFFFu));
        const uint32_t gq = qn >> 2;
        carry = gq == (q >> 2) + 1u;
        const float4 g1 = *grpu<L>(a, gq + 1u, i);
        constexpr uint32_t gm = kDtSize[L] / 4u - 1u;
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            a.ring[L], (short)0, (int)(uint32_t)((uint64_t)kDtSize[L] * a.n * 4u), 0x00020000);
        const uint32_t off = carry ? 0xFFFFFFF0u : ((gq & gm) * a.n + i) * 16u;
        typedef unsigned int u4 __attribute__((ext_vector_type(4)));
        const u4 g0 = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
        p0 = __uint_as_float(g0.x); p1 = __uint_as_float(g0.y); p2 = __uint_as_float(g0.z); p3 = __uint_as_float(g0.w);
        r0 = g1.x; r1 = g1.y; r2 = g1.z; r3 = g1.w;
    }
    __device__ __forceinline__ void resolve() {       // shift q & 3 (wave-uniform) by selects
        // (shift4 keeps them v_cndmask: scalar or exec-mask branches cost precise waitcnt
        // tracking of the prefetch at every merge)
        shift4(q & 3u, c0, c1, c2, c3, n0, n1, n2, v);
    }
    __device__ __forceinline__ void advance() {
        uint32_t k;                                   // VGPR copy of the uniform flag, as in resolve()
        asm volatile("v_mov_b32 %0, %1" : "=v"(k) : "s"(carry ? 1u : 0u));
        c0 = k ? n0 : p0; c1 = k ? n1 : p1; c2 = k ? n2 : p2; c3 = k ? n3 : p3;
        n0 = r0; n1 = r1; n2 = r2; n3 = r3;
        q = qn;
    }
};

// The per-instance pre-delay tap (verb.cpp:137-139, :273).  Delay d is constant over a launch.
//   d >= 9 : carried ring window with a per-lane shift (t0 - d) & 3: the group prefetched during
//            chunk c (before chunk c's own store) is ((t0 - d) >> 2) + 2 <= chunk c-1's group;
//   d <= 8 : the frames come from registers: this chunk's input and the two previous chunks'.
// Both are evaluated and selected per lane, with no branch and no load that depends on d, so
// every chunk issues the same loads (a load under a branch made the compiler wait for ALL
// outstanding loads, the next chunk's prefetch included, at the merge).  Lanes of one wave
// that share d issue coalesced loads.
struct PreTap {
    float4 cur, nxt, pre;
    float x1[4], x2[4];                               // inputs of chunks c-1 and c-2
    uint32_t s;
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t d, uint32_t i) {
        const uint32_t q = t0 - d;
        s = q & 3u;
        cur = *grp<DT_PRE>(a, q >> 2, i);
        nxt = *grp<DT_PRE>(a, (q >> 2) + 1u, i);
        const float4 g1 = *grpu<DT_PRE>(a, (t0 >> 2) - 1u, i), g2 = *grpu<DT_PRE>(a, (t0 >> 2) - 2u, i);
        x1[0] = g1.x; x1[1] = g1.y; x1[2] = g1.z; x1[3] = g1.w;
        x2[0] = g2.x; x2[1] = g2.y; x2[2] = g2.z; x2[3] = g2.w;
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t d, uint32_t i) {
        pre = *grp<DT_PRE>(a, ((t0 - d) >> 2) + 2u, i);
    }
    // xpd[k] = mono input at t0 + k - d
    // d <= 8: xpd[k] = r[8 - d + k] of the history r = x2 | x1 | xin, i.e. groups g, g + 1 of r
    // (g = (8 - d) / 4) shifted by (8 - d) & 3 -- group selects and a shift4, no compare per d
    __device__ __forceinline__ void resolve(const float (&xin)[4], uint32_t d, float (&xpd)[4]) const {
        float ring[4], reg[4];
        shift4(s, cur, nxt, ring);
        const uint32_t idx = 8u - min(d, 8u);
        uint32_t g1 = idx & 4u, g2 = idx & 8u, near = d <= 8u ? 1u : 0u;
        asm volatile("" : "+v"(g1), "+v"(g2), "+v"(near));
        float a[4], b[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            a[k] = g2 ? xin[k] : (g1 ? x1[k] : x2[k]);
            b[k] = g1 ? xin[k] : x1[k];               // (g = 2 is d = 0: shift 0, b unused)
        }
        shift4(idx & 3u, a[0], a[1], a[2], a[3], b[0], b[1], b[2], reg);
#pragma unroll
        for (int k = 0; k < 4; ++k) xpd[k] = near ? reg[k] : ring[k];
    }
    __device__ __forceinline__ void advance(const float (&xin)[4]) {
        cur = nxt; nxt = pre;
#pragma unroll
        for (int k = 0; k < 4; ++k) { x2[k] = x1[k]; x1[k] = xin[k]; }
    }
    // the chunk's input into the ring: one 16-B group per lane, position-major (coalesced)
    __device__ __forceinline__ void write(const DattorroArgs &a, uint32_t gw, uint32_t i, const float (&xin)[4]) const {
        *grpu<DT_PRE>(a, gw, i) = make_float4(xin[0], xin[1], xin[2], xin[3]);
    }
};

// Gather mode with unaligned rows (per-instance pre-delays, verb.cpp:137-139): dattorro_predelay_v2 has already written
// the block's pre-delayed input, group by group, to a.pre_block ([n_frames/4][n][4]: 16 B per lane
// and chunk, coalesced) and kept the ring itself, instance-major.  The network reads that stream:
// no gather across lines here, and no ring write.
struct PreBlock {
    float4 cur, pre;
    uint32_t t0, last;
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0_, uint32_t d, uint32_t i) {
        (void)d;
        t0 = t0_;
        last = a.n_frames / 4u - 1u;
        cur = ((const float4 *)a.pre_block)[i];
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t, uint32_t d, uint32_t i) {
        (void)d;
        const uint32_t g = min(((t - t0) >> 2) + 1u, last);
        pre = ((const float4 *)a.pre_block)[(size_t)g * a.n + i];
    }
    __device__ __forceinline__ void resolve(const float (&xin)[4], uint32_t d, float (&xpd)[4]) const {
        (void)xin; (void)d;
        xpd[0] = cur.x; xpd[1] = cur.y; xpd[2] = cur.z; xpd[3] = cur.w;
    }
    __device__ __forceinline__ void advance(const float (&xin)[4]) { (void)xin; cur = pre; }
    __device__ __forceinline__ void write(const DattorroArgs &, uint32_t, uint32_t, const float (&)[4]) const {}
};

// Fused gather mode (dattorro_block_v4f, dattorro.hip): the kernel itself keeps, per 32-frame
// piece, the piece's mono input (M) and each instance's window of its pre-delay ring (W, the 36
// positions from (T - d) & ~3) in LDS, filled one piece ahead.  Frame t of the piece (t = T + f)
// reads x[t - d]: from M when t - d >= T (d <= f: this piece's own input), else from W.  The
// caller points m / w at the lane's rows and sets fc (the chunk's first frame within the piece)
// and off0 ((T - d) & 3) before each dt_step.
struct PreFused {
    const float *m, *w;
    int fc;
    uint32_t off0;
    __device__ __forceinline__ void prime(const DattorroArgs &, uint32_t, uint32_t, uint32_t) {}
    __device__ __forceinline__ void prefetch(const DattorroArgs &, uint32_t, uint32_t, uint32_t) {}
    __device__ __forceinline__ void resolve(const float (&)[4], uint32_t d, float (&xpd)[4]) const {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int q = fc + k - (int)d;
            const float *src = q >= 0 ? m + q : w + (off0 + (uint32_t)(fc + k));
            xpd[k] = *src;
        }
    }
    __device__ __forceinline__ void advance(const float (&)[4]) {}
    __device__ __forceinline__ void write(const DattorroArgs &, uint32_t, uint32_t, const float (&)[4]) const {}
};

// The fused chain's pre-delay tap (chain.hip, round 5).  The chain keeps its pre-delay ring in ROWS
// of 16 positions ([8192/16][n][16]: 64 B per instance and row, a workgroup's 64 rows one 4-KB
// run), so whatever the instances' pre-delays, a 16-frame chunk needs one new row per instance: 64 B
// that one HBM request serves whole (the position-major groups of PreTap, read at 64 different
// rows for 64 different delays, cost a 64-B request per 16 B read).  The chain's reverb wave stages
// in LDS ([slot][lane] float4 columns):
//   near (slot = group & 7): the inputs of this chunk and the one before (positions T - 16 .. T + 15);
//   far (slot = group & 15): rows r0 - 1 .. r0 + 2 (r0 = (T - d) >> 4), for the positions before
//        T - 16.  Row r0 + 2 is loaded during the chunk -- after the chunk's ring store, so it holds
//        every position before T, all that far serves up to two chunks later -- a group per step
//        (step m: group m, 16 B of the lane's 64-B row; the row's later groups hit the L2), and
//        staged one step later over row r0 - 2 (group 3 at the next chunk's first step: group m of
//        a row r0 + 1 is needed from step m on).  Load at one step, use at
//        the next: the taps' prefetch pattern, whose waits stay exact inside the step loop (a row
//        loaded before the loop and used after it cost a vmcnt(0) drain per chunk, +12 %).
// Groups are 4-aligned and T % 4 == 0, so a group lies wholly in near or in far.
struct PreRow {
    const float4 *near, *far;   // this lane's columns: near[slot * 64], far[slot * 64]
    float4 *farw;               // = far (written)
    const float4 *ring;         // group 0 of row 0 of this lane's instance
    uint32_t nd, T;             // nd: instances of the ring (a multiple of 64); T: the chunk's first position
    int fc;                     // the step's first frame within the chunk (0, 4, 8, 12)
    float4 pv;                  // the group loaded at the step before, for farw[pslot]
    uint32_t pslot;
    __device__ __forceinline__ void prime(const DattorroArgs &, uint32_t, uint32_t, uint32_t) {}
    // step m of the chunk: stage the group loaded at the step before, then load group m of this
    // lane's row r0 + 2
    __device__ __forceinline__ void prefetch(const DattorroArgs &, uint32_t, uint32_t d, uint32_t) {
        farw[pslot] = pv;
        const uint32_t m = (uint32_t)fc >> 2, row = ((T - d) >> 4) + 2u;
        pv = ring[(size_t)(row & (kDtSize[DT_PRE] / 16u - 1u)) * nd * 4u + m];
        pslot = ((row & 3u) * 4u + m) * 64u;
    }
    __device__ __forceinline__ void resolve(const float (&)[4], uint32_t d, float (&xpd)[4]) const {
        const uint32_t s = (0u - d) & 3u;            // (T + fc - d) & 3
        const int nr = fc - (int)(d + s);             // 4 x (first group - T / 4)
        const uint32_t g0 = (T + (uint32_t)fc - d) >> 2;
        const float4 *pa = nr >= -16 ? near + (g0 & 7u) * 64u : far + (g0 & 15u) * 64u;
        const float4 *pb = nr >= -20 ? near + ((g0 + 1u) & 7u) * 64u : far + ((g0 + 1u) & 15u) * 64u;
        shift4(s, *pa, *pb, xpd);                     // (s == 0: the second group is unused)
    }
    __device__ __forceinline__ void advance(const float (&)[4]) {}
    __device__ __forceinline__ void write(const DattorroArgs &, uint32_t, uint32_t, const float (&)[4]) const {}
};

// The body of one 4-frame chunk (verb.cpp:273-299, 302-325).  Taps come by reference, so after
// inlining every access is to the caller's locals.
#define DT_ALL_TAPS(OP) OP(in0) OP(in1) OP(in2) OP(in3) OP(fbA) OP(fbB) OP(dl1a) OP(dl1b) OP(ap2a) OP(ap2b) \
    OP(oL1) OP(oL2) OP(oL3) OP(oL4) OP(oL5) OP(oL6) OP(oL7) OP(oR1) OP(oR2) OP(oR3) OP(oR4) OP(oR5) OP(oR6) OP(oR7)

template <class TIN0, class TIN1, class TIN2, class TIN3, class TFBA, class TFBB, class TDL1A, class TDL1B,
          class TAP2A, class TAP2B, class TL1, class TL2, class TL3, class TL4, class TL5, class TL6, class TL7,
          class TR1, class TR2, class TR3, class TR4, class TR5, class TR6, class TR7, class TM1A, class TM1B,
          class TPRE>
__device__ __forceinline__ void step_body(
    const DattorroArgs &a, uint32_t i, uint32_t t0, bool has_next, const float (&xin)[4], float (&o_l)[4],
    float (&o_r)[4], uint32_t dpre, float g_pre, float g_in1, float g_in2, float g_dd1, float g_damp, float g_decay,
    float g_dd2, float &lp_pre, float &lp_a, float &lp_b, TIN0 &in0, TIN1 &in1, TIN2 &in2, TIN3 &in3, TFBA &fbA,
    TFBB &fbB, TDL1A &dl1a, TDL1B &dl1b, TAP2A &ap2a, TAP2B &ap2b, TL1 &oL1, TL2 &oL2, TL3 &oL3, TL4 &oL4,
    TL5 &oL5, TL6 &oL6, TL7 &oL7, TR1 &oR1, TR2 &oR2, TR3 &oR3, TR4 &oR4, TR5 &oR5, TR6 &oR6, TR7 &oR7,
    TM1A &ap1a, TM1B &ap1b, TPRE &pre) {
    // Prefetch unconditionally (the last chunk's prefetch reads valid ring memory and is
    // dropped): loads under a branch cost precise waitcnt tracking at the merge.
    (void)has_next;
#define DT_PREFETCH_OP(T) T.prefetch(a, t0, i);
    DT_ALL_TAPS(DT_PREFETCH_OP)
#undef DT_PREFETCH_OP
    ap1a.prefetch(a, t0, i);
    ap1b.prefetch(a, t0, i);
    pre.prefetch(a, t0, dpre, i);
    ap1a.resolve();
    ap1b.resolve();
    float xpd[4];
    pre.resolve(xin, dpre, xpd);

    float w_in0[4], w_in1[4], w_in2[4], w_in3[4], w_ap1a[4], w_dl1a[4], w_ap2a[4], w_dl2a[4];
    float w_ap1b[4], w_dl1b[4], w_ap2b[4], w_dl2b[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lp_pre += (xpd[k] - lp_pre) * g_pre;
        float x = lp_pre;
        float d = in0.get(k);
        x += d * -g_in1; w_in0[k] = x; x = d + x * g_in1;
        d = in1.get(k);
        x += d * -g_in1; w_in1[k] = x; x = d + x * g_in1;
        d = in2.get(k);
        x += d * -g_in2; w_in2[k] = x; x = d + x * g_in2;
        d = in3.get(k);
        x += d * -g_in2; w_in3[k] = x; x = d + x * g_in2;
        {   // tank half A; the APF gain is -dd1, so in += delayed * dd1
            float y = x + fbA.get(k) * g_decay;
            d = ap1a.v[k];
            y += d * g_dd1; w_ap1a[k] = y; y = d + y * -g_dd1;
            w_dl1a[k] = y;
            lp_a += (dl1a.get(k) - lp_a) * g_damp;
            y = lp_a * g_decay;
            d = ap2a.get(k);
            y += d * -g_dd2; w_ap2a[k] = y; y = d + y * g_dd2;
            w_dl2a[k] = y;
        }
        {   // tank half B
            float y = x + fbB.get(k) * g_decay;
            d = ap1b.v[k];
            y += d * g_dd1; w_ap1b[k] = y; y = d + y * -g_dd1;
            w_dl1b[k] = y;
            lp_b += (dl1b.get(k) - lp_b) * g_damp;
            y = lp_b * g_decay;
            d = ap2b.get(k);
            y += d * -g_dd2; w_ap2b[k] = y; y = d + y * g_dd2;
            w_dl2b[k] = y;
        }
        float l = oL1.get(k);
        l += oL2.get(k); l -= oL3.get(k); l += oL4.get(k); l -= oL5.get(k); l -= oL6.get(k); l += oL7.get(k);
        float r = oR1.get(k);
        r += oR2.get(k); r -= oR3.get(k); r += oR4.get(k); r -= oR5.get(k); r -= oR6.get(k); r += oR7.get(k);
        o_l[k] = l;
        o_r[k] = r;
    }

    // ---- writes: one 16-B group per line ----
    const uint32_t gw = t0 >> 2;
    pre.write(a, gw, i, xin);
    *grpu<DT_IN0>(a, gw, i) = make_float4(w_in0[0], w_in0[1], w_in0[2], w_in0[3]);
    in1.write(a, gw, i, make_float4(w_in1[0], w_in1[1], w_in1[2], w_in1[3]));
    *grpu<DT_IN2>(a, gw, i) = make_float4(w_in2[0], w_in2[1], w_in2[2], w_in2[3]);
    *grpu<DT_IN3>(a, gw, i) = make_float4(w_in3[0], w_in3[1], w_in3[2], w_in3[3]);
    *grpu<DT_AP1A>(a, gw, i) = make_float4(w_ap1a[0], w_ap1a[1], w_ap1a[2], w_ap1a[3]);
    *grpu<DT_DL1A>(a, gw, i) = make_float4(w_dl1a[0], w_dl1a[1], w_dl1a[2], w_dl1a[3]);
    *grpu<DT_AP2A>(a, gw, i) = make_float4(w_ap2a[0], w_ap2a[1], w_ap2a[2], w_ap2a[3]);
    *grpu<DT_DL2A>(a, gw, i) = make_float4(w_dl2a[0], w_dl2a[1], w_dl2a[2], w_dl2a[3]);
    *grpu<DT_AP1B>(a, gw, i) = make_float4(w_ap1b[0], w_ap1b[1], w_ap1b[2], w_ap1b[3]);
    *grpu<DT_DL1B>(a, gw, i) = make_float4(w_dl1b[0], w_dl1b[1], w_dl1b[2], w_dl1b[3]);
    *grpu<DT_AP2B>(a, gw, i) = make_float4(w_ap2b[0], w_ap2b[1], w_ap2b[2], w_ap2b[3]);
    *grpu<DT_DL2B>(a, gw, i) = make_float4(w_dl2b[0], w_dl2b[1], w_dl2b[2], w_dl2b[3]);

#define DT_ADVANCE_OP(T) T.advance();
    DT_ALL_TAPS(DT_ADVANCE_OP)
#undef DT_ADVANCE_OP
    ap1a.advance();
    ap1b.advance();
    pre.advance(xin);
}

}  // namespace dt
}  // namespace olfx

// One instance's reverb network as a resumable per-lane stage, used by dattorro_block (input from
// the audio buffer) and by the fused chain (input from the pitch-shift stage through LDS).
// DT_STAGE(A, I) declares the stage's locals and three lambdas over them in the caller's scope:
// one aggregate holding every tap would stay in scratch memory (SROA does not split it), while
// separate locals are promoted to registers exactly as in a hand-written kernel.
//   dt_prime(t0)                                   once per launch, t0 % 4 == 0
//   dt_step(t0, has_next, xin[4], o_l[4], o_r[4])  one 4-frame chunk, mono in -> L/R out
//   dt_finish()                                    writes the recursive scalars back
#define DT_PRIME_OP(T) T.prime(dt_args, t0, dt_i);
#define DT_STAGE(A, I) DT_STAGE_PRE(A, I, olfx::dt::PreTap)
#define DT_STAGE_PRE(A, I, PRE_T) DT_STAGE_X(A, I, PRE_T, (olfx::dt::Tap<DT_IN1, 107, 0>))
#define DT_UNPAREN(...) __VA_ARGS__
#define DT_STAGE_X(A, I, PRE_T, IN1_T)                                                                   \
    const DattorroArgs &dt_args = (A);                                                                   \
    const uint32_t dt_n = dt_args.n, dt_i = (I);                                                         \
    const float g_pre = dt_args.coef[DTC_PREFILTER * dt_n + dt_i];                                       \
    const float g_in1 = dt_args.coef[DTC_IN1 * dt_n + dt_i];                                             \
    const float g_in2 = dt_args.coef[DTC_IN2 * dt_n + dt_i];                                             \
    const float g_dd1 = dt_args.coef[DTC_DD1 * dt_n + dt_i];                                             \
    const float g_damp = dt_args.coef[DTC_DAMPING * dt_n + dt_i];                                        \
    const float g_decay = dt_args.coef[DTC_DECAY * dt_n + dt_i];                                         \
    const float g_dd2 = dt_args.coef[DTC_DD2 * dt_n + dt_i];                                             \
    const uint32_t dpre = (uint32_t)dt_args.coef[DTC_PREDELAY * dt_n + dt_i]; /* exact integer */        \
    float lp_pre = dt_args.state[DTS_LP_PRE * dt_n + dt_i];                                              \
    float lp_a = dt_args.state[DTS_LP_DAMP_A * dt_n + dt_i];                                             \
    float lp_b = dt_args.state[DTS_LP_DAMP_B * dt_n + dt_i];                                             \
    olfx::dt::Tap<DT_IN0, 142, 0> in0; DT_UNPAREN IN1_T in1;                                             \
    olfx::dt::Tap<DT_IN2, 379, 0> in2; olfx::dt::Tap<DT_IN3, 277, 0> in3;                               \
    olfx::dt::Tap<DT_DL2B, 3163, 0> fbA; olfx::dt::Tap<DT_DL2A, 3720, 0> fbB;                           \
    olfx::dt::Tap<DT_DL1A, 4453, 0> dl1a; olfx::dt::Tap<DT_DL1B, 4217, 0> dl1b;                         \
    olfx::dt::Tap<DT_AP2A, 1800, 0> ap2a; olfx::dt::Tap<DT_AP2B, 2656, 0> ap2b;                         \
    olfx::dt::Tap<DT_DL1B, kDl1B_o1, 1> oL1; olfx::dt::Tap<DT_DL1B, kDl1B_o2, 1> oL2;                   \
    olfx::dt::Tap<DT_AP2B, kAp2B_o2, 1> oL3; olfx::dt::Tap<DT_DL2B, kDl2B_o2, 1> oL4;                   \
    olfx::dt::Tap<DT_DL1A, kDl1A_o3, 1> oL5; olfx::dt::Tap<DT_AP2A, kAp2A_o1, 1> oL6;                   \
    olfx::dt::Tap<DT_DL2A, kDl2A_o1, 1> oL7;                                                             \
    olfx::dt::Tap<DT_DL1A, kDl1A_o1, 1> oR1; olfx::dt::Tap<DT_DL1A, kDl1A_o2, 1> oR2;                   \
    olfx::dt::Tap<DT_AP2A, kAp2A_o2, 1> oR3; olfx::dt::Tap<DT_DL2A, kDl2A_o2, 1> oR4;                   \
    olfx::dt::Tap<DT_DL1B, kDl1B_o3, 1> oR5; olfx::dt::Tap<DT_AP2B, kAp2B_o1, 1> oR6;                   \
    olfx::dt::Tap<DT_DL2B, kDl2B_o1, 1> oR7;                                                             \
    olfx::dt::ModTap<DT_AP1A, kDtDelay[DT_AP1A]> ap1a;                                                   \
    olfx::dt::ModTap<DT_AP1B, kDtDelay[DT_AP1B]> ap1b;                                                   \
    PRE_T pre;                                                                                           \
    auto dt_prime = [&](uint32_t t0) {                                                                   \
        DT_ALL_TAPS(DT_PRIME_OP)                                                                         \
        ap1a.prime(dt_args, t0, dt_i);                                                                   \
        ap1b.prime(dt_args, t0, dt_i);                                                                   \
        pre.prime(dt_args, t0, dpre, dt_i);                                                              \
    };                                                                                                   \
    auto dt_step = [&](uint32_t t0, bool has_next, const float(&xin)[4], float(&o_l)[4], float(&o_r)[4]) { \
        olfx::dt::step_body(dt_args, dt_i, t0, has_next, xin, o_l, o_r, dpre, g_pre, g_in1, g_in2, g_dd1, \
                            g_damp, g_decay, g_dd2, lp_pre, lp_a, lp_b, in0, in1, in2, in3, fbA, fbB, dl1a, \
                            dl1b, ap2a, ap2b, oL1, oL2, oL3, oL4, oL5, oL6, oL7, oR1, oR2, oR3, oR4, oR5,    \
                            oR6, oR7, ap1a, ap1b, pre);                                                  \
    };                                                                                                   \
    auto dt_finish = [&]() {                                                                             \
        dt_args.state[DTS_LP_PRE * dt_n + dt_i] = lp_pre;                                                \
        dt_args.state[DTS_LP_DAMP_A * dt_n + dt_i] = lp_a;                                               \
        dt_args.state[DTS_LP_DAMP_B * dt_n + dt_i] = lp_b;                                               \
    }
