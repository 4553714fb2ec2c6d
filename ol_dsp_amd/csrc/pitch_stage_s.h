// ol_dsp_amd/csrc/pitch_stage_s.h -- the fused chain's pitch-shift stage with STEREO LANES.
//
// The chain's P role runs the gen~ pitch-shifter (pitchshift.gendsp / gencode at
// mono-chorus.rnbopat:962; spec in DESIGN.md section 3) on the chorus output of 64 instances.
// Rounds 1-3 ran it as two ChStageL<false, true> stages (chorus_stage_l.h), one lane per
// (instance, channel) of 32 instances each.  Here one lane is one instance and carries both
// channels: L and R share the phasor, so every frame's window gains and delay splits are computed
// once per instance instead of once per lane pair plus DPP exchanges, the stereo-interleaved ring
// positions are read as one 8-B (L, R) LDS read, and the per-chunk work of the line carry (plan,
// ownership exchange, line loads, staging, patches) is done once for 64 instances instead of twice
// for 32.  A wave alone on its SIMD issues every one of those instructions serially (DESIGN.md
// section 4), so the role's instruction count is its time.
//
// Everything else follows the per-lane stage it replaced (ChStageL's former XPREV form, which took
// its input one chunk late; removed from chorus_stage_l.h with this file), operation for operation
// (bit-exact):
//   * per tap and instance the two aligned 128-B lines L', L'+1 of the window are carried in
//     registers, spread over the wave (8 lanes x 16 B per line; 8 parts of 8 instances);
//   * the stage stores its own input x_c (staged in LDS, cooperative 128-B runs) before the next
//     chunk's line loads, so a carried line lacks x_c (patched from the staging at chunk c+1) and
//     x_{c+1} (patched from registers); out-of-window frames land in junk slots (clamped slots);
//   * a chunk whose pitch window the lines cannot cover (a phasor wrap, a short chunk) runs the
//     generic per-frame path with direct ring reads.
#pragma once
#include "chorus_stage_l.h"

namespace olfx {
namespace ch {

__device__ __forceinline__ float2 ld2(Rsrc r, uint32_t voff) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    const u2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, 0, 0);
    return make_float2(__uint_as_float(v.x), __uint_as_float(v.y));
}
__device__ __forceinline__ void st2(Rsrc r, uint32_t voff, float2 v) {
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    u2 u;
    u.x = __float_as_uint(v.x);
    u.y = __float_as_uint(v.y);
    __builtin_amdgcn_raw_buffer_store_b64(u, r, voff, 0, 0);
}
__device__ __forceinline__ float2 lerp2(float2 x0, float2 x1, float fr) {
    return make_float2(lerp_pair(x0.x, x1.x, fr), lerp_pair(x0.y, x1.y, fr));
}

struct PStageS {
    static constexpr int kChunk = 16, kWin = 24, kSlots = kWin + 2;   // slots kWin, kWin + 1: junk
    static constexpr int kRow2 = 128;                // floats per slot row: 64 instances x (L, R)
    static constexpr int kStride = 36;               // input staging per instance: 16 x (L, R) + pad
    static constexpr int kWinFloats = 2 * kSlots * kRow2;
    static constexpr int kRegion = kWinFloats + 64 * kStride;   // the windows, then the staging

    uint32_t lane, inst0, n;
    bool valid;
    uint32_t i;
    uint64_t lfo_inc, ps_inc, lfo_acc, ps_acc;
    uint32_t wi, wf, pmaxu;   // pitch window W in 32.32 fixed point; delay clamp psize - 2
    uint32_t pmask, pshift;
    Rsrc rP;
    float *region;
    float4 ln[2][2][8];       // [tap][line set][part]: piece lane/8 of a line of instance part*8 + (lane & 7)
    uint32_t s15;             // window start & 15 per (tap, part), 2 bits each (starts are 4-aligned)
    uint32_t lcur[2];         // line L' of the current chunk's window, per tap (this lane's instance)
    PlanL pl;
    uint32_t wpos;
    bool started;

    __device__ __forceinline__ static uint64_t word64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }

    __device__ __forceinline__ void init(const ChorusArgs &a, float *lds_region, uint32_t lane_, uint32_t inst0_) {
        lane = lane_; inst0 = inst0_; n = a.n;
        const uint32_t i_raw = inst0 + lane;
        valid = i_raw < n;
        i = valid ? i_raw : n - 1;
        lfo_inc = word64(a.coef[CHC_LFO_INC * n + i], a.coef[CHC_LFO_INC_LO * n + i]);
        ps_inc = word64(a.coef[CHC_PS_INC * n + i], a.coef[CHC_PS_INC_LO * n + i]);
        wi = a.coef[CHC_WINDOW * n + i];
        wf = a.coef[CHC_WINDOW_LO * n + i];
        lfo_acc = word64(a.state[CHS_LFO_ACC * n + i], a.state[CHS_LFO_LO * n + i]);
        ps_acc = word64(a.state[CHS_PS_ACC * n + i], a.state[CHS_PS_LO * n + i]);
        pmask = a.psize - 1u;
        pmaxu = a.psize - 2u;
        rP = rsrc(a.pitch_ring, (uint64_t)n * 2 * a.psize * 4);
        pshift = (uint32_t)__builtin_ctz(a.psize) + 3u;
        region = lds_region;
        wpos = a.t0;
        started = false;
        s15 = 0;
    }

    // this lane's instance (clamped), recomputed where used (see ChStageL::own_i)
    __device__ __forceinline__ uint32_t own_pb() const {
        uint32_t l = lane;
        asm volatile("" : "+v"(l));
        return min(inst0 + l, n - 1u) << pshift;
    }
    __device__ __forceinline__ uint32_t pjj(int r) const { return (uint32_t)r * 8u + (lane & 7u); }
    __device__ __forceinline__ uint32_t pm() const { return lane >> 3; }
    __device__ __forceinline__ uint32_t line_off(uint32_t oi, uint32_t q) const {
        return (oi << pshift) + ((q * 16u + 2u * pm()) & pmask) * 8u;
    }
    __device__ __forceinline__ float *staging() const { return region + kWinFloats; }

    // the next chunk's line loads (ChStageL::load_lines): each lane decides carry / fresh for its
    // own instance and publishes (window start relative to w) * 2 | fresh through ds_bpermute
    template <int HI>
    __device__ __forceinline__ void load_lines(const PlanL &p, uint32_t w, bool first) {
        constexpr int LO = HI ^ 1;
        const int s[2] = {p.sA, p.sB};
        int pk[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const uint32_t lnext = (w + (uint32_t)s[t]) >> 4;
            const bool carry = !first && lnext == lcur[t] + 1u;
            lcur[t] = lnext;
            pk[t] = (int)((uint32_t)s[t] << 1) | (carry ? 0 : 1);
        }
        int v[2][8];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 8; ++r) v[t][r] = __builtin_amdgcn_ds_bpermute((int)(pjj(r) << 2), pk[t]);
        uint32_t s15n = 0;
#pragma unroll
        for (int t = 0; t < 2; ++t) {
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const uint32_t sabs = w + (uint32_t)(v[t][r] >> 1);
                const uint32_t q = sabs >> 4;
                const uint32_t oi = min(inst0 + pjj(r), n - 1);
                s15n |= ((sabs & 15u) >> 2) << (2 * (t * 8 + r));
                ln[t][HI][r] = ld4(rP, line_off(oi, q + 1u));
                if (v[t][r] & 1) ln[t][LO][r] = ld4(rP, line_off(oi, q));
            }
        }
        s15 = s15n;
    }

    // lines of tap t -> its LDS window [slot][instance](L, R); pieces outside the window go to the
    // junk slots (a piece is wholly inside or outside: its first slot is even)
    template <int HI, int t>
    __device__ __forceinline__ void stage_tap() {
        constexpr int LO = HI ^ 1;
        float *base = region + t * kSlots * kRow2;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t jj = pjj(r);
            const int st = (int)(((s15 >> (2 * (t * 8 + r))) & 3u) << 2);
            const int slo = 2 * (int)pm() - st, shi = slo + 16;
            const float4 a = ln[t][LO][r], b = ln[t][HI][r];
            float *plo = base + min((uint32_t)slo, (uint32_t)kWin) * kRow2 + 2 * jj;
            float *phi = base + min((uint32_t)shi, (uint32_t)kWin) * kRow2 + 2 * jj;
            *(float2 *)plo = make_float2(a.x, a.y);
            *(float2 *)(plo + kRow2) = make_float2(a.z, a.w);
            *(float2 *)phi = make_float2(b.x, b.y);
            *(float2 *)(phi + kRow2) = make_float2(b.z, b.w);
        }
    }

    __device__ __forceinline__ void begin(int C) {
        pl = plan_chunk_l<kWin>(0ull, 0ull, 0ull, ps_acc, ps_inc, C, 0.0, wi, wf, pmaxu, 0.0, false);
        load_lines<0>(pl, wpos, true);
    }

    // One chunk of C frames (a multiple of 4) with input x (L, R); PAR = chunk parity.  sink(k, y)
    // receives output frame k (k < C).
    template <int PAR, class Sink>
    __device__ __forceinline__ void chunk(const float2 (&x)[kChunk], int C, int Cn, Sink &&sink) {
        asm volatile("" : "+v"(lane));
        const uint32_t w0 = wpos;
        const uint64_t ps0 = ps_acc;
        const PlanL cur = pl;
        float *wP0 = region + 2u * lane;
        float *wP1 = region + kSlots * kRow2 + 2u * lane;
        float *stg = staging() + lane * kStride;
        stage_tap<PAR, 0>();
        stage_tap<PAR, 1>();
        if (started) {
            // x_{c-1} (still in the input staging) is not in a carried line: frame k -> slot
            // k - 16 - s, or a junk slot outside the window
            float2 xq[kChunk];
#pragma unroll
            for (int k = 0; k < kChunk; k += 2) {
                const float4 v = *(const float4 *)(stg + 2 * k);
                xq[k] = make_float2(v.x, v.y);
                xq[k + 1] = make_float2(v.z, v.w);
            }
            const uint32_t nA = (uint32_t)(-(kChunk + cur.sA)), nB = (uint32_t)(-(kChunk + cur.sB));
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                *(float2 *)(wP0 + min((uint32_t)k + nA, (uint32_t)kWin) * kRow2) = xq[k];
                *(float2 *)(wP1 + min((uint32_t)k + nB, (uint32_t)kWin) * kRow2) = xq[k];
            }
        }
        {
            // x_c is not in a carried line either: slot k - s (>= 2), the top clamped into the junk
            // slot; past a short chunk's C frames, slot C - s, a position no frame of it reads
            const int mA = min(kWin + cur.sA, C), mB = min(kWin + cur.sB, C);
            float *pA = wP0 - cur.sA * kRow2, *pB = wP1 - cur.sB * kRow2;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                *(float2 *)(pA + min(k, mA) * kRow2) = x[k];
                *(float2 *)(pB + min(k, mB) * kRow2) = x[k];
            }
            // and into the input staging, for the ring store and the next chunk's patch
#pragma unroll
            for (int k = 0; k < kChunk; k += 2) *(float4 *)(stg + 2 * k) = make_float4(x[k].x, x[k].y, x[k + 1].x, x[k + 1].y);
        }
        started = true;

        float2 psv[kChunk];
        const bool fast = C == kChunk && __all(cur.okA && cur.okB);
        if (fast) {
            // the tap delays of spec v2 (pitch_split: 32.32 fixed point)
            const int rA = -cur.sA, rB = -cur.sB;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                const uint32_t ph = hi32(ps_acc);
                float gA, gB;
                win_gains(unit24(ph), gA, gB);
                uint32_t di;
                float fr;
                pitch_split(ph, wi, wf, pmaxu, di, fr);
                const float *qA = wP0 + (k + rA - (int)di) * kRow2;
                const float2 tA = lerp2(*(const float2 *)qA, *(const float2 *)(qA - kRow2), fr);
                pitch_split(ph + 0x80000000u, wi, wf, pmaxu, di, fr);     // p1 = (p0 + 1/2) % 1
                const float *qB = wP1 + (k + rB - (int)di) * kRow2;
                const float2 tB = lerp2(*(const float2 *)qB, *(const float2 *)(qB - kRow2), fr);
                psv[k] = make_float2(xfade(tB.x, gB, tA.x, gA), xfade(tB.y, gB, tA.y, gA));
                ps_acc += ps_inc;
            }
            lfo_acc += (uint64_t)kChunk * lfo_inc;
        } else {
            // generic chunk: per frame, direct ring reads for an uncovered tap.  Such a read can reach
            // this chunk's own input (a delay below 16 right after a phasor wrap): store it first, per
            // lane (the cooperative store follows as usual); the reads are this lane's own, in order
            const uint32_t pb = own_pb();
#pragma unroll
            for (int k = 0; k < kChunk; ++k) st2(rP, valid && k < C ? pb + ((w0 + (uint32_t)k) & pmask) * 8u : 0xFFFFFFF0u, x[k]);
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                if (k >= C) { psv[k] = make_float2(0.f, 0.f); continue; }
                float gA, gB;
                win_gains(unit24h(ps_acc), gA, gB);
                const uint32_t ph = hi32(ps_acc);
                lfo_acc += lfo_inc;
                ps_acc += ps_inc;
                uint32_t di;
                float fr;
                float2 tA, tB;
                pitch_split(ph, wi, wf, pmaxu, di, fr);
                if (!cur.okA) {
                    const uint32_t q = w0 + k - di;
                    tA = lerp2(ld2(rP, own_pb() + (q & pmask) * 8u), ld2(rP, own_pb() + ((q - 1u) & pmask) * 8u), fr);
                } else {
                    const int jw = k - (int)di - cur.sA;
                    tA = lerp2(*(const float2 *)(wP0 + jw * kRow2), *(const float2 *)(wP0 + (jw - 1) * kRow2), fr);
                }
                pitch_split(ph + 0x80000000u, wi, wf, pmaxu, di, fr);
                if (!cur.okB) {
                    const uint32_t q = w0 + k - di;
                    tB = lerp2(ld2(rP, own_pb() + (q & pmask) * 8u), ld2(rP, own_pb() + ((q - 1u) & pmask) * 8u), fr);
                } else {
                    const int jw = k - (int)di - cur.sB;
                    tB = lerp2(*(const float2 *)(wP1 + jw * kRow2), *(const float2 *)(wP1 + (jw - 1) * kRow2), fr);
                }
                psv[k] = make_float2(xfade(tB.x, gB, tA.x, gA), xfade(tB.y, gB, tA.y, gA));
            }
        }
        // x_c into the ring: 8 lanes per instance write its 128-B stereo run from the staging
#pragma unroll
        for (int r = 0; r < 8; ++r) {
            const uint32_t q = (uint32_t)r * 64u + lane, o = q >> 3, f2 = 2u * (q & 7u);
            const float4 v = *(const float4 *)(staging() + o * kStride + 2u * f2);
            const uint32_t oi = inst0 + o;
            const bool ok = oi < n && (int)f2 < C;
            st4<kStreamAux>(rP, ok ? (oi << pshift) + ((w0 + f2) & pmask) * 8u : 0xFFFFFFF0u, v);
        }
        // chunk c+1's plan and line loads (they see the store above: a wave's vector memory
        // operations reach the caches in issue order)
        pl = plan_chunk_l<kWin>(0ull, 0ull, 0ull, ps0 + (uint64_t)C * ps_inc, ps_inc, Cn > 0 ? Cn : 4, 0.0, wi, wf,
                                pmaxu, 0.0, false);
        load_lines<PAR ^ 1>(pl, w0 + (uint32_t)C, false);
#pragma unroll
        for (int k = 0; k < kChunk; ++k)
            if (fast || k < C) sink(k, psv[k]);
        wpos = w0 + (uint32_t)C;
    }

    __device__ __forceinline__ void finish(const ChorusArgs &a) const {
        if (!valid) return;
        a.state[CHS_LFO_ACC * n + i] = (uint32_t)(lfo_acc >> 32);
        a.state[CHS_LFO_LO * n + i] = (uint32_t)lfo_acc;
        a.state[CHS_PS_ACC * n + i] = (uint32_t)(ps_acc >> 32);
        a.state[CHS_PS_LO * n + i] = (uint32_t)ps_acc;
    }
};

}  // namespace ch
}  // namespace olfx
