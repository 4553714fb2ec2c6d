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
#include "lds_flags.h"

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

// A fixed tap prefetched TWO steps ahead (the split network's tank halves, whose register sets have
// room for it): p1 = the group step s + 1 needs, loaded a step ago; p2, loaded at step s for s + 2.
// Every fixed delay is >= 121 positions, so no prefetched group is written by the steps before it.
template <int L, uint32_t D, uint32_t OFF>
struct Tap2 {
    static constexpr uint32_t S = (OFF - D) & 3u;
    float4 cur, nxt, p1, p2;
    __device__ __forceinline__ static uint32_t g0(uint32_t t0) { return (t0 + OFF - D) >> 2; }
    __device__ __forceinline__ void prime(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        cur = *grpu<L>(a, g0(t0), i);
        if (S) nxt = *grpu<L>(a, g0(t0) + 1u, i);
        p1 = *grpu<L>(a, g0(t0) + (S ? 2u : 1u), i);
    }
    __device__ __forceinline__ void prefetch(const DattorroArgs &a, uint32_t t0, uint32_t i) {
        p2 = *grpu<L>(a, g0(t0) + (S ? 3u : 2u), i);
    }
    __device__ __forceinline__ float get(int k) const {
        return (int)S + k < 4 ? el(cur, (int)S + k) : el(nxt, (int)S + k - 4);
    }
    __device__ __forceinline__ void advance() {
        if (S) { cur = nxt; nxt = p1; } else { cur = p1; }
        p1 = p2;
    }
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

// The pre-delay tap over rows (round 5 in the fused chain; round 6 also dattorro_block_v5).  The chain keeps its pre-delay ring in ROWS
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

// ---------------------------------------------------------------------------------------------
// The split network (round 6): DI, TA and TB as three waves (dattorro_block_v5, the chain's reverb
// roles).  Within a launch of at most kSplitMaxFrames frames the network is three independent
// recurrences joined only by feed-forward values:
//   DI: pre-delay, pre-LPF and the 4 input all-passes (verb.cpp:273-282) -> x;
//   TA: tank half 0 (verb.cpp:284-295, i = 0): AP1A, DL1A, damping, AP2A, DL2A;
//   TB: tank half 1: AP1B, DL1B, damping, AP2B, DL2B.
// The halves exchange data only through postDampingDelay[1 - i]'s main tap (verb.cpp:286), 3163
// (TA reads DL2B) and 3720 (TB reads DL2A) samples back: within a launch shorter than that they
// read only what earlier launches wrote, and each wave reads back only rings it writes itself.  x
// goes to both halves through an LDS queue.  The stereo taps (verb.cpp:302-325) split at their sum
// order: L = pL - oL5 - oL6 + oL7 with pL = oL1 + oL2 - oL3 + oL4 on half 1's rings and oL5..7 on
// half 0's; R the mirror image.  So half 1 sends pL to half 0, which finishes L, and half 0 sends pR
// to half 1, which finishes R (one float per frame each way, through LDS, one step late so neither
// waits on the other's current step) -- the reference's additions in the reference's order.
// Per 4-frame step: DI 5 taps, each half 11 (3 network + 1 modulated + 7 output) and 4 ring writes.
// ---------------------------------------------------------------------------------------------
constexpr uint32_t kSplitDepth = 4;          // LDS queue slots (4-frame steps) per hand-off
constexpr uint32_t kSplitMaxFrames = 2048;   // < 3163 - queue skew: no cross-half read within a launch
// progress counters (lds_flags.h), in steps: SPF_X x published by DI; SPF_XT<h> x taken by half h;
// SPF_P<h> partial sums half h has published; SPF_PT<h> half h's partials the other half has taken
enum { SPF_X = 0, SPF_XT0, SPF_XT1, SPF_P0, SPF_P1, SPF_PT0, SPF_PT1, SPF_N };

struct SplitQ {
    const float4 *qx;   // [kSplitDepth][64]: x of a step per lane
    float4 *mine;       // this half's partial sums
    const float4 *other;
    uint32_t *flags;
};

__device__ __forceinline__ float4 f4(const float (&v)[4]) { return make_float4(v[0], v[1], v[2], v[3]); }

// The taps of tank half H.  P1..P4: the partial sum this half sends (half 0: pR = oR1 + oR2 - oR3 +
// oR4 on DL1A, DL1A, AP2A, DL2A; half 1: pL = oL1 + oL2 - oL3 + oL4 on DL1B, DL1B, AP2B, DL2B);
// T5..T7: the terms that finish the other half's sum into this half's channel (half 0, L: oL5 DL1A,
// oL6 AP2A, oL7 DL2A; half 1, R: oR5 DL1B, oR6 AP2B, oR7 DL2B).
template <int H> struct SplitHalf;
template <> struct SplitHalf<0> {
    static constexpr int kAP1 = DT_AP1A, kDL1 = DT_DL1A, kAP2 = DT_AP2A, kDL2 = DT_DL2A, kLp = DTS_LP_DAMP_A;
    using FB = Tap<DT_DL2B, 3163, 0>;
    using DL1 = Tap<DT_DL1A, 4453, 0>;
    using AP2 = Tap<DT_AP2A, 1800, 0>;
    using AP1 = ModTap<DT_AP1A, kDtDelay[DT_AP1A]>;
    using P1 = Tap<DT_DL1A, kDl1A_o1, 1>;
    using P2 = Tap<DT_DL1A, kDl1A_o2, 1>;
    using P3 = Tap<DT_AP2A, kAp2A_o2, 1>;
    using P4 = Tap<DT_DL2A, kDl2A_o2, 1>;
    using T5 = Tap<DT_DL1A, kDl1A_o3, 1>;
    using T6 = Tap<DT_AP2A, kAp2A_o1, 1>;
    using T7 = Tap<DT_DL2A, kDl2A_o1, 1>;
};
template <> struct SplitHalf<1> {
    static constexpr int kAP1 = DT_AP1B, kDL1 = DT_DL1B, kAP2 = DT_AP2B, kDL2 = DT_DL2B, kLp = DTS_LP_DAMP_B;
    using FB = Tap<DT_DL2A, 3720, 0>;
    using DL1 = Tap<DT_DL1B, 4217, 0>;
    using AP2 = Tap<DT_AP2B, 2656, 0>;
    using AP1 = ModTap<DT_AP1B, kDtDelay[DT_AP1B]>;
    using P1 = Tap<DT_DL1B, kDl1B_o1, 1>;
    using P2 = Tap<DT_DL1B, kDl1B_o2, 1>;
    using P3 = Tap<DT_AP2B, kAp2B_o2, 1>;
    using P4 = Tap<DT_DL2B, kDl2B_o2, 1>;
    using T5 = Tap<DT_DL1B, kDl1B_o3, 1>;
    using T6 = Tap<DT_AP2B, kAp2B_o1, 1>;
    using T7 = Tap<DT_DL2B, kDl2B_o1, 1>;
};

// DI's arithmetic for one 4-frame step (verb.cpp:275-282): the pre-delayed input xpd through the
// pre-LPF and the 4 input all-passes -> x (xo), and the groups the step writes to IN0..IN3
template <class T0, class T1, class T2, class T3>
__device__ __forceinline__ void di_compute(const float (&xpd)[4], float &lp_pre, float g_pre, float g_in1, float g_in2,
                                           T0 &in0, T1 &in1, T2 &in2, T3 &in3, float (&w0)[4], float (&w1)[4],
                                           float (&w2)[4], float (&w3)[4], float (&xo)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        lp_pre += (xpd[k] - lp_pre) * g_pre;
        float x = lp_pre;
        float d = in0.get(k);
        x += d * -g_in1; w0[k] = x; x = d + x * g_in1;
        d = in1.get(k);
        x += d * -g_in1; w1[k] = x; x = d + x * g_in1;
        d = in2.get(k);
        x += d * -g_in2; w2[k] = x; x = d + x * g_in2;
        d = in3.get(k);
        x += d * -g_in2; w3[k] = x; x = d + x * g_in2;
        xo[k] = x;
    }
}

// DI hands step gs's x to both halves (once both have taken step gs - kSplitDepth's)
__device__ __forceinline__ void split_publish_x(float4 *qx, uint32_t *flags, uint32_t lane, uint32_t gs,
                                                const float (&xo)[4]) {
    wait_for([&] {
        return flag_get(flags + SPF_XT0) + kSplitDepth > gs && flag_get(flags + SPF_XT1) + kSplitDepth > gs;
    });
    qx[(gs % kSplitDepth) * 64u + lane] = f4(xo);
    flag_put(flags + SPF_X, gs + 1);
}

__device__ __forceinline__ void wsync() {      // LDS written by some lanes, read by others
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// DI over the pre-delay ring in ROWS of 16 positions ([8192/16][n][16], PreRow above) for the
// instances 64 g .. 64 g + 63 (those >= d.n mirror instance d.n - 1 and store nothing): whatever
// the instances' pre-delays, a 16-frame chunk costs one 64-B row per instance (verb.cpp:137-139,
// :273).  stage: 25 x 64 float4 of LDS (far 17 x 64, near 8 x 64).  src(c, f0, C, xm) gives chunk c's
// mono input xm[16] (frames f0 .. f0 + 15 of the launch, C of them real).  in1: IN1's tap, an HBM Tap
// or an LdsTap (its write goes where it reads).  Each step's x goes to the tank halves through qx
// (step numbers from gs0).
template <class In1T, class Src>
__device__ __forceinline__ void split_di_rows(const DattorroArgs &d, uint32_t g, uint32_t lane, uint32_t nf,
                                              uint32_t gs0, float4 *stage, float4 *qx, uint32_t *flags,
                                              In1T &in1, Src &&src) {
    constexpr uint32_t kChunk = 16;
    constexpr uint32_t kRows = kDtSize[DT_PRE] / 16u;
    const uint32_t nd = d.n, base = g * 64u;
    const uint32_t i = min(base + lane, nd - 1u);
    const uint32_t cj = lane >> 2, cg = lane & 3u;
    float4 *const far = stage, *const near = stage + 17 * 64;
    const float g_pre = d.coef[DTC_PREFILTER * nd + i];
    const float g_in1 = d.coef[DTC_IN1 * nd + i];
    const float g_in2 = d.coef[DTC_IN2 * nd + i];
    const uint32_t dpre = (uint32_t)d.coef[DTC_PREDELAY * nd + i];
    float lp_pre = d.state[DTS_LP_PRE * nd + i];
    Tap<DT_IN0, 142, 0> in0; Tap<DT_IN2, 379, 0> in2; Tap<DT_IN3, 277, 0> in3;
    PreRow pre;
    const uint32_t t0 = d.t0;
    in0.prime(d, t0, i); in1.prime(d, t0, i); in2.prime(d, t0, i); in3.prime(d, t0, i);
    float4 *const ring = (float4 *)d.ring[DT_PRE];    // row r of instance j: ring + (r * nd + j) * 4
    uint32_t dj[4], jc[4];                            // cooperative instance 16 m + l / 4: its pre-delay, its index
    bool jl[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        dj[m] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((16u * m + cj) << 2), (int)dpre);
        jl[m] = base + 16u * m + cj < nd;
        jc[m] = min(base + 16u * m + cj, nd - 1u);
    }
    pre.near = near + lane;
    pre.far = far + lane;
    pre.farw = far + lane;
    pre.ring = ring + (size_t)i * 4u;
    pre.nd = nd;
    pre.pv = make_float4(0.f, 0.f, 0.f, 0.f);
    pre.pslot = 16u * 64u;                            // junk: nothing loaded yet
    auto row_ptr = [&](uint32_t row, int m) { return ring + ((size_t)(row & (kRows - 1u)) * nd + jc[m]) * 4u + cg; };
    auto put_row = [&](uint32_t T, uint32_t plus, int m) {   // group cg of row ((T - d) >> 4) + plus -> far
        const uint32_t row = ((T - dj[m]) >> 4) + plus;
        far[((row & 3u) * 4u + cg) * 64u + 16u * m + cj] = *row_ptr(row, m);
    };
    auto ring_at = [&](uint32_t T, int m) {           // group cg of positions T .. T + 15 in the ring
        const uint32_t P = T + 4u * cg;
        return ring + ((size_t)((P >> 4) & (kRows - 1u)) * nd + jc[m]) * 4u + ((P >> 2) & 3u);
    };
    auto near_at = [&](uint32_t T, int m) { return near + (((T >> 2) + cg) & 7u) * 64u + 16u * m + cj; };
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        put_row(t0, 0, m);
        put_row(t0, 1, m);
        *near_at(t0 - kChunk, m) = *ring_at(t0 - kChunk, m);
    }
    const uint32_t nchunks = (nf + kChunk - 1) / kChunk;
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t f0 = c * kChunk, T = t0 + f0;
        const uint32_t C = min(kChunk, nf - f0);
        float xm[kChunk];
        src(c, f0, C, xm);
        // the chunk's input -> near (over the chunk before the one before), then into the ring
        // cooperatively (groups past a short chunk's C frames stay); the next rows' loads, issued
        // during the steps below, see these stores (one wave, issue order)
#pragma unroll
        for (int m = 0; m < 4; ++m)
            near[(((T >> 2) + (uint32_t)m) & 7u) * 64u + lane] = make_float4(xm[4 * m], xm[4 * m + 1], xm[4 * m + 2], xm[4 * m + 3]);
        wsync();
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 v = *near_at(T, m);
            if (4u * cg < C && jl[m]) *ring_at(T, m) = v;
        }
        pre.T = T;
        for (uint32_t s = 0; s < C; s += 4) {
            const uint32_t t = T + s;
            float xin[4], xpd[4], w0[4], w1[4], w2[4], w3[4], xo[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) xin[k] = xm[s + k];
            pre.fc = (int)s;
            in0.prefetch(d, t, i); in1.prefetch(d, t, i); in2.prefetch(d, t, i); in3.prefetch(d, t, i);
            pre.prefetch(d, t, dpre, i);
            pre.resolve(xin, dpre, xpd);
            di_compute(xpd, lp_pre, g_pre, g_in1, g_in2, in0, in1, in2, in3, w0, w1, w2, w3, xo);
            const uint32_t gw = t >> 2;
            *grpu<DT_IN0>(d, gw, i) = f4(w0);
            in1.write(d, gw, i, f4(w1));
            *grpu<DT_IN2>(d, gw, i) = f4(w2);
            *grpu<DT_IN3>(d, gw, i) = f4(w3);
            split_publish_x(qx, flags, lane, gs0 + (f0 + s) / 4u, xo);
            in0.advance(); in1.advance(); in2.advance(); in3.advance();
        }
        wsync();                                      // this chunk's LDS reads before the next one's writes
    }
    if (base + lane < nd) d.state[DTS_LP_PRE * nd + i] = lp_pre;
}

// Tank half H of instance i over `steps` 4-frame steps from stream time t0; gs0 = the queues' step
// number of its first step (a workgroup's instance groups run back to back in the chain).  Channel
// H of frame f goes to out[f * out_n + i] for live lanes (out: the channel's plane).
template <int H>
__device__ __forceinline__ void split_tank(const DattorroArgs &a, uint32_t i, uint32_t lane, bool live, uint32_t t0,
                                           uint32_t steps, uint32_t gs0, float *out, uint32_t out_n,
                                           const SplitQ &q) {
    using Hf = SplitHalf<H>;
    const uint32_t n = a.n;
    const float g_dd1 = a.coef[DTC_DD1 * n + i];
    const float g_damp = a.coef[DTC_DAMPING * n + i];
    const float g_decay = a.coef[DTC_DECAY * n + i];
    const float g_dd2 = a.coef[DTC_DD2 * n + i];
    float lp = a.state[Hf::kLp * n + i];
    typename Hf::FB fb; typename Hf::DL1 dl1; typename Hf::AP2 ap2; typename Hf::AP1 ap1;
    typename Hf::P1 p1; typename Hf::P2 p2; typename Hf::P3 p3; typename Hf::P4 p4;
    typename Hf::T5 t5; typename Hf::T6 t6; typename Hf::T7 t7;
#define SPLIT_TAPS(OP) OP(fb) OP(dl1) OP(ap2) OP(p1) OP(p2) OP(p3) OP(p4) OP(t5) OP(t6) OP(t7)
#define SPLIT_PRIME(T) T.prime(a, t0, i);
#define SPLIT_PREFETCH(T) T.prefetch(a, t, i);
#define SPLIT_ADVANCE(T) T.advance();
    SPLIT_TAPS(SPLIT_PRIME)
    ap1.prime(a, t0, i);
    uint32_t *const flags = q.flags;
    float q5[4], q6[4], q7[4];                        // the previous step's finishing terms
    auto finish = [&](uint32_t s) {                   // channel H of step s: the other half's partial + q5..q7
        const uint32_t gs = gs0 + s;
        wait_for([&] { return flag_get(flags + SPF_P0 + (1 - H)) > gs; });
        const float4 po = q.other[(gs % kSplitDepth) * 64u + lane];
        flag_put(flags + SPF_PT0 + (1 - H), gs + 1);
        const float pv[4] = {po.x, po.y, po.z, po.w};
        if (live) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float o = pv[k];
                o -= q5[k]; o -= q6[k]; o += q7[k];
                out[(size_t)(4u * s + (uint32_t)k) * out_n + i] = o;
            }
        }
    };
    for (uint32_t s = 0; s < steps; ++s) {
        const uint32_t t = t0 + 4u * s, gs = gs0 + s, slot = gs % kSplitDepth;
        SPLIT_TAPS(SPLIT_PREFETCH)
        ap1.prefetch(a, t, i);
        ap1.resolve();
        wait_for([&] { return flag_get(flags + SPF_X) > gs; });
        const float4 xv = q.qx[slot * 64u + lane];
        flag_put(flags + SPF_XT0 + H, gs + 1);
        const float x[4] = {xv.x, xv.y, xv.z, xv.w};
        float w_ap1[4], w_dl1[4], w_ap2[4], w_dl2[4], pm[4], n5[4], n6[4], n7[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {                 // verb.cpp:286-294; the APF gain is -dd1
            float y = x[k] + fb.get(k) * g_decay;
            float d = ap1.v[k];
            y += d * g_dd1; w_ap1[k] = y; y = d + y * -g_dd1;
            w_dl1[k] = y;
            lp += (dl1.get(k) - lp) * g_damp;
            y = lp * g_decay;
            d = ap2.get(k);
            y += d * -g_dd2; w_ap2[k] = y; y = d + y * g_dd2;
            w_dl2[k] = y;
            float p = p1.get(k);
            p += p2.get(k); p -= p3.get(k); p += p4.get(k);
            pm[k] = p;
            n5[k] = t5.get(k); n6[k] = t6.get(k); n7[k] = t7.get(k);
        }
        const uint32_t gw = t >> 2;
        *grpu<Hf::kAP1>(a, gw, i) = f4(w_ap1);
        *grpu<Hf::kDL1>(a, gw, i) = f4(w_dl1);
        *grpu<Hf::kAP2>(a, gw, i) = f4(w_ap2);
        *grpu<Hf::kDL2>(a, gw, i) = f4(w_dl2);
        // this step's partial out, then the previous step's channel
        wait_for([&] { return flag_get(flags + SPF_PT0 + H) + kSplitDepth > gs; });
        q.mine[slot * 64u + lane] = f4(pm);
        flag_put(flags + SPF_P0 + H, gs + 1);
        if (s > 0) finish(s - 1);
#pragma unroll
        for (int k = 0; k < 4; ++k) { q5[k] = n5[k]; q6[k] = n6[k]; q7[k] = n7[k]; }
        SPLIT_TAPS(SPLIT_ADVANCE)
        ap1.advance();
    }
    if (steps) finish(steps - 1);
    if (live) a.state[Hf::kLp * n + i] = lp;
#undef SPLIT_TAPS
#undef SPLIT_PRIME
#undef SPLIT_PREFETCH
#undef SPLIT_ADVANCE
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

namespace olfx {
namespace dt {

// The whole network in one wave (DT_STAGE_X, all 27 taps) over the pre-delay ring in ROWS (PreRow),
// for the instances 64 g .. 64 g + 63: the fused chain's reverb role.
// CLAMP: instances >= d.n mirror instance d.n - 1 and store nothing (the chain pads d.n to 64).
// src(c, f0, C, xm) gives chunk c's mono input (16 frames from f0, C real); out(f, o_l, o_r) takes
// the 4 frames from f.  stage: 25 x 64 float4 of LDS (far 17 x 64, near 8 x 64).
template <bool CLAMP, class Src, class Out>
__device__ __forceinline__ void rows_network(const DattorroArgs &d, uint32_t g, uint32_t lane, uint32_t nf,
                                             float4 *stage, Src &&src, Out &&out) {
    constexpr uint32_t kChunk = 16;
    constexpr uint32_t kRows = kDtSize[DT_PRE] / 16u;
    const uint32_t nd = d.n, base = g * 64u;
    const uint32_t cj = lane >> 2, cg = lane & 3u;
    float4 *const far = stage, *const near = stage + 17 * 64;
    DT_STAGE_PRE(d, (CLAMP ? min(base + lane, nd - 1u) : base + lane), olfx::dt::PreRow);
    const uint32_t t0 = d.t0;
    dt_prime(t0);
    float4 *const ring = (float4 *)d.ring[DT_PRE];    // row r of instance j: ring + (r * nd + j) * 4
    uint32_t dj[4], jc[4];                            // cooperative instance 16 m + l / 4: its pre-delay, its index
    bool jl[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        dj[m] = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((16u * m + cj) << 2), (int)dpre);
        jl[m] = !CLAMP || base + 16u * m + cj < nd;
        jc[m] = CLAMP ? min(base + 16u * m + cj, nd - 1u) : base + 16u * m + cj;
    }
    pre.near = near + lane;
    pre.far = far + lane;
    pre.farw = far + lane;
    pre.ring = ring + (size_t)dt_i * 4u;
    pre.nd = nd;
    pre.pv = make_float4(0.f, 0.f, 0.f, 0.f);
    pre.pslot = 16u * 64u;                            // junk: nothing loaded yet
    auto row_ptr = [&](uint32_t row, int m) { return ring + ((size_t)(row & (kRows - 1u)) * nd + jc[m]) * 4u + cg; };
    auto put_row = [&](uint32_t T, uint32_t plus, int m) {   // group cg of row ((T - d) >> 4) + plus -> far
        const uint32_t row = ((T - dj[m]) >> 4) + plus;
        far[((row & 3u) * 4u + cg) * 64u + 16u * m + cj] = *row_ptr(row, m);
    };
    auto ring_at = [&](uint32_t T, int m) {           // group cg of positions T .. T + 15 in the ring
        const uint32_t P = T + 4u * cg;
        return ring + ((size_t)((P >> 4) & (kRows - 1u)) * nd + jc[m]) * 4u + ((P >> 2) & 3u);
    };
    auto near_at = [&](uint32_t T, int m) { return near + (((T >> 2) + cg) & 7u) * 64u + 16u * m + cj; };
#pragma unroll
    for (int m = 0; m < 4; ++m) {                     // the first chunk's rows r0, r0 + 1 and the chunk before
        put_row(t0, 0, m);
        put_row(t0, 1, m);
        *near_at(t0 - kChunk, m) = *ring_at(t0 - kChunk, m);
    }
    const uint32_t nchunks = (nf + kChunk - 1) / kChunk;
    for (uint32_t c = 0; c < nchunks; ++c) {
        const uint32_t f0 = c * kChunk, T = t0 + f0;
        const uint32_t C = min(kChunk, nf - f0);
        float xm[kChunk];
        src(c, f0, C, xm);
        // the chunk's input -> near (over the chunk before the one before), then into the ring
        // cooperatively (groups past a short chunk's C frames stay); the next rows' loads, issued
        // during the steps below (PreRow::prefetch), see these stores (one wave, issue order)
#pragma unroll
        for (int m = 0; m < 4; ++m)
            near[(((T >> 2) + (uint32_t)m) & 7u) * 64u + lane] = make_float4(xm[4 * m], xm[4 * m + 1], xm[4 * m + 2], xm[4 * m + 3]);
        wsync();
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 v = *near_at(T, m);
            if (4u * cg < C && jl[m]) *ring_at(T, m) = v;
        }
        pre.T = T;
        auto step = [&](uint32_t s) {
            float xin[4], o_l[4], o_r[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) xin[k] = xm[s + k];
            pre.fc = (int)s;
            dt_step(T + s, f0 + s + 4 < nf, xin, o_l, o_r);
            out(f0 + s, o_l, o_r);
        };
        for (uint32_t s = 0; s < C; s += 4) step(s);
        wsync();                                      // this chunk's LDS reads before the next one's writes
    }
    if (!CLAMP || base + lane < nd) dt_finish();
}

}  // namespace dt
}  // namespace olfx
