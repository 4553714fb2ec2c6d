// ol_dsp_amd/csrc/chorus_stage_l.h -- the chorus / pitch-shifter stage with LINE CARRY (v11).
//
// Same spec, lane mapping, LDS window layout and per-frame recurrence as chorus_stage.h (v10); what
// changes is how the windows get from HBM into LDS.  v10 fetched, for every tap of every chunk, a
// fresh 24-position window (192 B at a 32-B aligned start: 2.25 128-B lines on average).  Each
// 128-B line was therefore fetched by two consecutive chunks, and the L2 cannot keep it between
// them (about 10 MB of other traffic passes through an XCD's 4 MB L2 in one chunk time), so the
// taps cost 18 B/frame each against the 8 B/frame they read (profiles/traffic_chorus.json).
//
// v11 holds, per tap and instance, the two aligned lines L', L'+1 (L' = line of the window start)
// in REGISTERS, cooperatively spread over the wave (8 lanes x 16 B per line, 4 parts of 8
// instances): 3 taps x 2 lines x 4 float4 = 96 VGPRs.  A tap's window advances about one line per
// chunk, so the line L'+1 of chunk c is the line L' of chunk c+1: each chunk loads only the new
// line (the "hi" load, unconditional) and carries the other.  The two line sets alternate roles by
// chunk parity (template PAR), so every register index is static.
//
// A carried line was loaded during the chunk before the previous one; positions written since are
// stale in it.  Each chunk therefore writes its pitch-shifter outputs (psv_c) and the NEXT chunk's
// inputs (x_{c+1}, prefetched) to the rings BEFORE it issues the next chunk's line loads, so a
// freshly loaded line holds everything up to the next chunk's own frames, and a carried line
// lacks only x_c and psv_{c-1}: both are still at hand (x_c in registers, psv_{c-1} in its LDS
// staging) and are patched into the windows, for every delay.  The chunk's pitch-shifter runs
// before those stores and line loads, the chorus tap after them, as the loads' cover.  A window
// that did not advance by exactly one line (or the first chunk of a launch) is FRESH: it also
// reloads L' (the "lo" load, exec-masked, so a carried line is never clobbered).
//
// The fused chain's pitch-shift stage, whose next input is not known while a chunk runs, is the
// stereo-lane variant of this scheme in pitch_stage_s.h (it stores its OWN input before the next
// chunk's line loads and patches it in at the next chunk).
//
// The chorus tap can span 18 positions (its delay may fall by one inside a chunk); when such a
// window starts at the last position of a line, its highest position lies in line L'+2: that one
// position per lane ("straggler") is loaded directly (4 B, own channel, exec-masked) and staged.
#pragma once
#include "chorus_stage.h"


namespace olfx {
namespace ch {

struct PlanL {
    int sA, sB, sC;           // window starts relative to the chunk's first write position (4-aligned)
    int hiC;                  // highest chorus-window position (relative)
    bool okA, okB;
};

// 64-bit phasors (2^64 = one cycle): the float phase is the top 24 bits of the high word, exact.
// The empty asm hides that the high word came from a 64-bit value: otherwise the compiler folds
// (float)(hi >> 8) into a 64-bit integer -> float conversion (five extra instructions each).
__device__ __forceinline__ uint32_t hi32(uint64_t acc) {
    uint32_t h = (uint32_t)(acc >> 32);
    asm("" : "+v"(h));
    return h;
}
__device__ __forceinline__ float unit24h(uint64_t acc) { return unit24(hi32(acc)); }
constexpr uint64_t kHalfCycle = 0x8000000000000000ull;

template <int kWin>
__device__ __forceinline__ PlanL plan_chunk_l(uint64_t lfo_acc, uint64_t lfo_inc, uint64_t lfo_off, uint64_t ps_acc,
                                              uint64_t ps_inc, int C, double D, uint32_t wi, uint32_t wf,
                                              uint32_t pmaxu, double cmaxd, bool full) {
    PlanL p;
    const uint32_t last = (uint32_t)(C - 1);
    // pitch taps: the floor delay is non-decreasing over the chunk unless the phasor wraps (the
    // delays are the frames' own: pitch_split, spec v2)
    uint32_t d0, d1;
    float fr;
    {
        const uint64_t a0 = ps_acc, a1 = ps_acc + last * ps_inc;
        pitch_split(hi32(a0), wi, wf, pmaxu, d0, fr);
        pitch_split(hi32(a1), wi, wf, pmaxu, d1, fr);
        const int lo = -(int)d1 - 1, hi = (int)last - (int)d0;
        p.sA = lo & ~3;
        p.okA = a1 >= a0 && hi - p.sA < kWin;
    }
    {
        const uint64_t a0 = ps_acc + kHalfCycle, a1 = a0 + last * ps_inc;
        pitch_split(hi32(a0), wi, wf, pmaxu, d0, fr);
        pitch_split(hi32(a1), wi, wf, pmaxu, d1, fr);
        const int lo = -(int)d1 - 1, hi = (int)last - (int)d0;
        p.sB = lo & ~3;
        p.okB = a1 >= a0 && hi - p.sB < kWin;
    }
    // chorus tap: the endpoint delays in fp32 (the 24-bit phase, cos2pi to 3e-7, D rounded: within
    // 5e-4 sample of the frames' own double delays, spec v2); in between the delay stays within
    // [min, max] of them up to the curvature of the LFO over 16 frames (< 1e-3 for every legal depth
    // and rate), so floor(min - .01) .. floor(max + .01) bounds every frame's floor delay, and those
    // two differ by at most one (|d'| <= 0.038 frame/frame).  (Round 4: the endpoints in double cost
    // two of the ten double cosines per lane and chunk; only the window bound depends on them.)
    p.sC = 0; p.hiC = 0;
    if (full) {
        const float Df = (float)D, cm = (float)cmaxd;
        const float e0 = fminf(fmaxf(cos2pi(unit24h(lfo_acc + lfo_off)) * Df + Df, 0.0f), cm);
        const float e1 = fminf(fmaxf(cos2pi(unit24h(lfo_acc + last * lfo_inc + lfo_off)) * Df + Df, 0.0f), cm);
        const int dhi = min((int)(fmaxf(e0, e1) + 0.01f), (int)cmaxd);
        const int dlo = (int)fmaxf(fminf(e0, e1) - 0.01f, 0.0f);
        p.sC = (-dhi - 1) & ~3;
        p.hiC = (int)last - dlo;
    }
    return p;
}

// COOP: the driver loads the block's input cooperatively -- per chunk 4 x 16 B per
// lane, rows (frame, channel) of the wave's 32 instances (coop_row below) -- and the stage
// transposes them through its LDS staging into the lanes' own frames; outputs go the same way
// (out_stage / coop_out below).  4 + 4 wide vector-memory instructions per chunk instead of
// 16 + 16 single-float ones (the per-CU vector-memory pipeline, TA/TD, is the busiest unit).
// OUT_LDS (default COOP): the sink writes the stage's LDS (out_stage), so a generic chunk emits its
// outputs only after stores_and_next has finished with the pitch windows (the fused chain's C role
// takes cooperative input but sinks into registers: OUT_LDS = false)
template <bool FULL, bool COOP = false, bool OUT_LDS = COOP>
struct ChStageL {
    // window slots: kWin, then two junk slots (patches, the straggler, clamped staging)
    static constexpr int kChunk = 16, kWin = 24, kSlots = kWin + 2;
    // floats of LDS per wave: one window per tap (chorus 3 x 26 x 64 = 4,992 = 19.5 KB: 2 waves/SIMD,
    // 156 KB per CU; pitch-shift alone 3,328 + its output staging)
    // COOP output staging [ch][frame][instance] (kOutCh below): in the chorus it overlays the pitch
    // windows' staging area (LDS is at its 2-waves/SIMD limit); the pitch-shifter has room for its own
    static constexpr uint32_t kOutCh = 544, kOutFloats = kOutCh + 16 * 32;
    static constexpr uint32_t kOutBase = FULL ? 0u : (uint32_t)(2 * kSlots * kRow);
    static constexpr int kRegion = (FULL ? 3 : 2) * kSlots * kRow + (OUT_LDS && !FULL ? (int)kOutFloats : 0);
    static constexpr int kStride = 36;
    static constexpr uint32_t kPsvBase = 32u * kStride;
    // (the channel planes 544 floats apart: conflict-free per-frame writes; in the chorus below the
    // psv staging, which must survive into the next chunk)
    static_assert(!FULL || kOutFloats <= kPsvBase, "output staging must not reach the psv staging");
    static constexpr int kTaps = FULL ? 3 : 2;
    static_assert(2 * 32 * kStride <= kRegion, "staging must fit in the window region");

    uint32_t lane, j, ch, inst0, n, i;
    bool valid;
    uint64_t lfo_inc, lfo_off, ps_inc;
    double D;                 // chorus depth in samples (spec v2: the delay is formed in double)
    uint32_t wi, wf;          // pitch window W in 32.32 fixed point
    float b0, b1, b2, a1, a2, mix, dry;
    uint64_t lfo_acc, ps_acc;
    float z1, z2;
    uint32_t pmask, cmask, pshift, cshift;   // ring sizes are powers of two: instance offset = i << shift
    uint32_t pmaxu;                          // delay clamps: psize - 2, csize - 2
    double cmaxd;
    Rsrc rP, rC;
    float *region;
    float4 ln[3][2][4];       // [tap][line set][part]: piece lane/8 of a line of instance part*8 + (lane & 7)
    uint32_t s15;             // window start & 15 per (tap, part), 2 bits each (start is 4-aligned)
    float strag;              // chorus straggler (own channel)
    uint32_t strag_slot;      // its LDS slot (kWin = junk)
    uint32_t lcur[3];         // owner: line L' of the current chunk's window, per tap
    PlanL pl;
    uint32_t wpos;
    bool started;

    __device__ __forceinline__ void init(const ChorusArgs &a, float *lds_region, uint32_t lane_, uint32_t inst0_) {
        lane = lane_; j = lane >> 1; ch = lane & 1u; inst0 = inst0_; n = a.n;
        const uint32_t i_raw = inst0 + j;
        valid = i_raw < n;
        i = valid ? i_raw : n - 1;
        lfo_inc = word64(a.coef[CHC_LFO_INC * n + i], a.coef[CHC_LFO_INC_LO * n + i]);
        lfo_off = word64(a.coef[CHC_LFO_OFF * n + i], a.coef[CHC_LFO_OFF_LO * n + i]);
        ps_inc = word64(a.coef[CHC_PS_INC * n + i], a.coef[CHC_PS_INC_LO * n + i]);
        D = __longlong_as_double((long long)word64(a.coef[CHC_DEPTH * n + i], a.coef[CHC_DEPTH_LO * n + i]));
        wi = a.coef[CHC_WINDOW * n + i];
        wf = a.coef[CHC_WINDOW_LO * n + i];
        b0 = __uint_as_float(a.coef[CHC_B0 * n + i]);
        b1 = __uint_as_float(a.coef[CHC_B1 * n + i]);
        b2 = __uint_as_float(a.coef[CHC_B2 * n + i]);
        a1 = __uint_as_float(a.coef[CHC_A1 * n + i]);
        a2 = __uint_as_float(a.coef[CHC_A2 * n + i]);
        mix = __uint_as_float(a.coef[CHC_MIX * n + i]);
        dry = __uint_as_float(a.coef[CHC_DRY * n + i]);
        lfo_acc = word64(a.state[CHS_LFO_ACC * n + i], a.state[CHS_LFO_LO * n + i]);
        ps_acc = word64(a.state[CHS_PS_ACC * n + i], a.state[CHS_PS_LO * n + i]);
        z1 = __uint_as_float(a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i]);
        z2 = __uint_as_float(a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i]);
        pmask = a.psize - 1u; cmask = a.csize - 1u;
        pmaxu = a.psize - 2u; cmaxd = (double)(a.csize - 2u);
        rP = rsrc(a.pitch_ring, (uint64_t)n * 2 * a.psize * 4);
        rC = rsrc(a.chorus_ring, (uint64_t)n * 2 * a.csize * 4);
        pshift = (uint32_t)__builtin_ctz(a.psize) + 3u; cshift = (uint32_t)__builtin_ctz(a.csize) + 3u;
        region = lds_region;
        wpos = a.t0;
        started = false;
        s15 = 0;
        strag = 0.f;
        strag_slot = kWin;
    }

    __device__ __forceinline__ static uint64_t word64(uint32_t hi, uint32_t lo) { return ((uint64_t)hi << 32) | lo; }

    // a window slot, or the junk slot kWin when the position lies outside the window: patches
    // write unconditionally (a select, no exec-masked block and branch per position)
    __device__ __forceinline__ static int junk_or(int jw) { return (uint32_t)jw < (uint32_t)kWin ? jw : kWin; }

    // this lane's samples in its rings, recomputed where used.  The empty asm makes the lane index
    // look loop-variant: otherwise the loop-invariant products are hoisted, spilled under the
    // register pressure of the carried lines, and every reload (a scratch load) costs a
    // vmcnt(0) drain of the whole prefetch.
    __device__ __forceinline__ uint32_t own_i() const {
        uint32_t l = lane;
        asm volatile("" : "+v"(l));
        return min(inst0 + (l >> 1), n - 1u);
    }
    __device__ __forceinline__ uint32_t own_pb() const { return (own_i() << pshift) + (lane & 1u) * 4u; }
    __device__ __forceinline__ uint32_t own_cb() const { return (own_i() << cshift) + (lane & 1u) * 4u; }

    // cooperative line geometry: part r (0..3) -> instance r*8 + (lane & 7), piece lane / 8.
    // Pieces outermost: a ds_write_b64 lane group (16 contiguous lanes) then stages two pieces of
    // eight instances (eight bank pairs, 2-way) instead of eight pieces of two instances (the
    // same bank pair in eight rows, 8-way); the line loads still cover 8 whole lines per wave.
    __device__ __forceinline__ uint32_t pjj(int r) const { return (uint32_t)r * 8u + (lane & 7u); }
    __device__ __forceinline__ uint32_t pm() const { return lane >> 3; }

    __device__ __forceinline__ uint32_t line_off(int t, uint32_t oi, uint32_t q) const {
        const uint32_t pos = q * 16u + 2u * pm();
        return t < 2 ? (oi << pshift) + (pos & pmask) * 8u : (oi << cshift) + (pos & cmask) * 8u;
    }
    __device__ __forceinline__ float4 ld_line(int t, uint32_t off) const { return ld4(t < 2 ? rP : rC, off); }

    // Issue the line loads for the chunk whose plan is p and first write position w.  Owner lanes
    // decide (carry / fresh) and publish per instance, through ds_bpermute, the packed value
    // (window start relative to w) * 2 | fresh.  Lines go into set HI (the new line L'+1) and, for
    // fresh instances only, set LO (L').
    template <int HI>
    __device__ __forceinline__ void load_lines(const PlanL &p, uint32_t w, bool first) {
        constexpr int LO = HI ^ 1;
        __builtin_amdgcn_s_setprio(kLoadPrio);      // the line loads ahead of the other wave's arithmetic
        const int s[3] = {p.sA, p.sB, p.sC};
        uint32_t s15n = 0;
        int pk[3];
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
            const uint32_t lnext = (w + (uint32_t)s[t]) >> 4;
            const bool carry = !first && lnext == lcur[t] + 1u;
            lcur[t] = lnext;
            pk[t] = (int)((uint32_t)s[t] << 1) | (carry ? 0 : 1);
        }
        // all exchanges first (one LDS round trip), then the loads
        int v[3][4];
#pragma unroll
        for (int t = 0; t < kTaps; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) v[t][r] = __builtin_amdgcn_ds_bpermute((int)(pjj(r) << 3), pk[t]);
#pragma unroll
        for (int t = 0; t < kTaps; ++t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const uint32_t jj = pjj(r);
                const uint32_t sabs = w + (uint32_t)(v[t][r] >> 1);
                const uint32_t q = sabs >> 4;
                const uint32_t oi = min(inst0 + jj, n - 1);
                s15n |= ((sabs & 15u) >> 2) << (2 * (t * 4 + r));
                ln[t][HI][r] = ld_line(t, line_off(t, oi, q + 1u));
                if (v[t][r] & 1) ln[t][LO][r] = ld_line(t, line_off(t, oi, q));
            }
        }
        s15 = s15n;
        // chorus straggler: a window of 18 positions starting at a line's last position
        strag_slot = kWin;
        if (FULL) {
            const uint32_t top = (lcur[2] << 4) + 32u;           // first position past the two lines
            const bool need = (w + (uint32_t)p.hiC) == top;
            strag_slot = need ? top - ((w + (uint32_t)p.sC)) : (uint32_t)kWin;
            if (need) strag = ld1(rC, own_cb() + (top & cmask) * 8u, 0);
        }
        __builtin_amdgcn_s_setprio(0);
    }

    // lines of tap t -> the chunk's LDS window ([tap][slot][lane], slot = position - window start)
    template <int HI, int t>
    __device__ __forceinline__ void stage_tap() {
        constexpr int LO = HI ^ 1;
        float *base = region + t * kSlots * kRow;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t jj = pjj(r);
            const int st = (int)(((s15 >> (2 * (t * 4 + r))) & 3u) << 2);
            const int slo = 2 * (int)pm() - st;          // line L' piece -> slots slo, slo + 1
            const int shi = slo + 16;                     // line L'+1 piece
            const float4 a = ln[t][LO][r], b = ln[t][HI][r];
            // pieces outside the window go to the junk slots kWin, kWin + 1 (slo is even, so a piece
            // is wholly inside or outside; slo < 0 wraps to a large unsigned value)
            float *plo = base + min((uint32_t)slo, (uint32_t)kWin) * kRow + 2 * jj;
            float *phi = base + min((uint32_t)shi, (uint32_t)kWin) * kRow + 2 * jj;
            *(float2 *)plo = make_float2(a.x, a.y);
            *(float2 *)(plo + kRow) = make_float2(a.z, a.w);
            *(float2 *)phi = make_float2(b.x, b.y);
            *(float2 *)(phi + kRow) = make_float2(b.z, b.w);
        }
        if (t == 2) base[strag_slot * kRow + lane] = strag;
    }

    __device__ __forceinline__ void stage_run(const float (&v)[kChunk], uint32_t base) {
        float *st = region + base + j * kStride + ch;
#pragma unroll
        for (int k = 0; k < kChunk; ++k) st[2 * k] = v[k];
    }
    __device__ __forceinline__ void coop_store(bool pitch, uint32_t base, uint32_t w, int C) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = (uint32_t)r * 64u + lane, o = q >> 3, f2 = 2u * (q & 7u);
            const float4 v = *(const float4 *)(region + base + o * kStride + 2u * f2);
            const uint32_t oi = inst0 + o;
            const bool ok = oi < n && (int)f2 < C;      // else an offset past the buffer: dropped
            if (pitch) st4<kStreamAux>(rP, ok ? (oi << pshift) + ((w + f2) & pmask) * 8u : 0xFFFFFFF0u, v);
            else st4<kStreamAux>(rC, ok ? (oi << cshift) + ((w + f2) & cmask) * 8u : 0xFFFFFFF0u, v);
        }
    }

    // COOP input: row r = 8 q + lane / 8 of instruction q is (frame r / 2, channel r % 2) of
    // instances 4 (lane % 8) .. + 3 -> the staging [j][2 frame + ch]; then each lane reads its own
    __device__ __forceinline__ static uint32_t coop_row(int q, uint32_t lane_) { return (uint32_t)q * 8u + (lane_ >> 3); }
    __device__ __forceinline__ void stage_rows(const float4 (&xq)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float *st = region + (lane & 7u) * 4u * kStride + coop_row(q, lane);
            st[0] = xq[q].x;
            st[kStride] = xq[q].y;
            st[2 * kStride] = xq[q].z;
            st[3 * kStride] = xq[q].w;
        }
    }
    __device__ __forceinline__ void read_own(float (&v)[kChunk], int Cv) const {
        const float *st = region + j * kStride + ch;
#pragma unroll
        for (int k = 0; k < kChunk; ++k) v[k] = k < Cv ? st[2 * k] : 0.f;
    }
    // COOP output: frame k of this lane -> [ch][k][j]; coop_out(q) = row 8 q + lane / 8 (frame,
    // channel) of instances 4 (lane % 8) .. + 3, after the chunk
    __device__ __forceinline__ void out_stage(int k, float v) { region[kOutBase + ch * kOutCh + (uint32_t)k * 32u + j] = v; }
    __device__ __forceinline__ float4 coop_out(int q) const {
        const uint32_t r = coop_row(q, lane);
        return *(const float4 *)(region + kOutBase + (r & 1u) * kOutCh + (r >> 1) * 32u + (lane & 7u) * 4u);
    }

    // first chunk of the launch: store its inputs, then load both lines of every window (fresh).
    // COOP: x is read from xq.
    __device__ __forceinline__ void begin(float (&x)[kChunk], int C, const float4 (&xq)[4]) {
        if (COOP) {
            stage_rows(xq);
            coop_store(true, 0, wpos, C);
            read_own(x, C);
        } else {
            stage_run(x, 0);
            coop_store(true, 0, wpos, C);
        }
        pl = plan_chunk_l<kWin>(lfo_acc, lfo_inc, lfo_off, ps_acc, ps_inc, C, D, wi, wf, pmaxu, cmaxd, FULL);
        load_lines<0>(pl, wpos, true);
    }
    __device__ __forceinline__ void begin(float (&x)[kChunk], int C) {
        static_assert(!COOP, "COOP stages begin with the cooperative rows");
        const float4 none[4] = {};
        begin(x, C, none);
    }

    // One chunk; PAR = chunk parity (the line set holding this chunk's line L'+1).
    // psv_c and x_{c+1} into the rings (the pitch windows are dead: their LDS is staging), then
    // chunk c+1's plan and line loads
    template <int PAR>
    __device__ __forceinline__ void stores_and_next(const float (&psv)[kChunk], const float (&x)[kChunk],
                                                    float (&xn)[kChunk], const float4 (&xq)[4], uint32_t w0,
                                                    int C, int Cn, uint64_t lfo0, uint64_t ps0) {
        if (FULL) {
            stage_run(psv, kPsvBase);
            coop_store(false, kPsvBase, w0, C);
        }
        if (COOP) {                              // x_{c+1}: rows -> staging -> ring and lanes
            if (Cn > 0) {
                stage_rows(xq);
                coop_store(true, 0, w0 + (uint32_t)C, Cn);
            }
            read_own(xn, Cn);
        } else if (Cn > 0) {
            stage_run(xn, 0);
            coop_store(true, 0, w0 + (uint32_t)C, Cn);
        }
        pl = plan_chunk_l<kWin>(lfo0 + (uint64_t)C * lfo_inc, lfo_inc, lfo_off, ps0 + (uint64_t)C * ps_inc,
                                ps_inc, Cn > 0 ? Cn : 4, D, wi, wf, pmaxu, cmaxd, FULL);
        // the line loads below read positions the stores above just wrote (other lanes of this
        // wave): vector memory operations of a wave reach the L1/L2 in issue order, as for the
        // v10 chunk-start input store and the loads after it
        load_lines<PAR ^ 1>(pl, w0 + (uint32_t)C, false);
    }

    // One chunk of C frames (multiple of 4) with input x; xn = the next chunk's input (Cn frames,
    // 0 = none), whose loads prefetch() issues.  PAR = chunk parity (the line set holding this
    // chunk's line L'+1).  Order (the staleness argument in the header):
    //   stage this chunk's windows, patch in x_c and psv_{c-1} (not in carried lines)
    //   A  pitch-shifter over the chunk -> psv_c; psv_c -> chorus window and chorus ring
    //      x_{c+1} (= xn) -> pitch ring
    //      plan chunk c+1, issue its line loads (they see both stores)
    //   C  chorus tap + lores~ + outputs (the cover for those loads)
    template <int PAR, class Sink, class Prefetch>
    __device__ __forceinline__ void chunk(const float (&x)[kChunk], float (&xn)[kChunk], int C, int Cn,
                                          Sink &&sink, Prefetch &&prefetch, const float4 (&xq)[4]) {
        // Everything lane-dependent is recomputed per chunk from a lane index the compiler must
        // treat as new: hoisted loop invariants (ring and LDS addresses) were spilled under the
        // pressure of the 96 line registers, and each scratch reload is a vmcnt(0) drain.
        asm volatile("" : "+v"(lane));
        j = lane >> 1;
        ch = lane & 1u;
        const uint32_t w0 = wpos;
        const uint64_t lfo0 = lfo_acc, ps0 = ps_acc;     // the phasors at the chunk's first frame
        const PlanL cur = pl;
        float psv[kChunk], yo[kChunk];
        float *wP0 = region + 0 * kSlots * kRow + lane;
        float *wP1 = region + 1 * kSlots * kRow + lane;
        float *wC = region + 2 * kSlots * kRow + lane;

        // tap C first: psv_{c-1}, still in its LDS staging (region + kPsvBase, under taps A/B),
        // is not in a carried line -- patch it in, then stage taps A and B over the staging
        if (FULL) {
            // psv_{c-1}'s frame k goes to slot k - 16 - sC when that lies in the window: all 16 read
            // first (a read after a store that may alias it would wait for the store, slot by slot),
            // then stored
            // branch-free: a slot outside the window becomes the junk slot kWin (unsigned min), so
            // no exec-mask region per store (each cost a compare, a saveexec, an exec restore and a
            // skip branch: instructions that a wave alone on its SIMD issues one by one)
            if (started) {
                const float *prev = region + kPsvBase + j * kStride + ch;
                float pv[kChunk];
#pragma unroll
                for (int k = 0; k < kChunk; ++k) pv[k] = prev[2 * k];
                stage_tap<PAR, 2>();
                const uint32_t nlo = (uint32_t)(-(kChunk + cur.sC));   // slot of frame k = k + nlo
#pragma unroll
                for (int k = 0; k < kChunk; ++k) wC[min((uint32_t)k + nlo, (uint32_t)kWin) * kRow] = pv[k];
            } else {
                stage_tap<PAR, 2>();
            }
        }
        stage_tap<PAR, 0>();
        stage_tap<PAR, 1>();
        // x_c is not in a carried line either.  Its slot k - s is >= 2 (a pitch window starts at
        // s <= -4: delays are >= 1), so only the top can leave the window
        {
            const int limA = kWin + cur.sA, limB = kWin + cur.sB;
            float *pA = wP0 - cur.sA * kRow, *pB = wP1 - cur.sB * kRow;
            // frame k -> slot min(k, lim) - s: past the window that is the junk slot kWin; past a
            // short chunk's C frames, slot C - s, a position no frame of this chunk reads
            const int mA = min(limA, C), mB = min(limB, C);
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                pA[min(k, mA) * kRow] = x[k];
                pB[min(k, mB) * kRow] = x[k];
            }
        }
        started = true;
        __builtin_amdgcn_s_setprio(kLoadPrio);      // the next chunk's input loads too
        prefetch();
        __builtin_amdgcn_s_setprio(0);

        const bool fast = C == kChunk && __all(cur.okA && cur.okB);
        if (fast) {
            // fast path, in phases with the per-frame arithmetic of frame() below:
            //  A. the pitch-shifter for all 16 frames (reads only the pitch windows, no LDS store:
            //     every frame's reads can be in flight together);
            //  B. its outputs into the chorus window -- delay~ writes before it reads, and a frame
            //     never reads a position newer than its own, so writing them all first is the same
            //     as writing each just before its frame;
            //  (C, the chorus tap, follows the ring stores and chunk c+1's line loads below)
            // the tap delays of spec v2 (pitch_split: 32.32 fixed point, olfx_internal.h).  L and R
            // lanes share every tap delay: per pair of frames each lane computes its own frame's
            // (k + ch) gains and delay splits once, and DPP hands both frames' values to both lanes;
            // slot offsets are kept relative to the pair's first frame, whose part of the address
            // is an immediate offset
            const int chA = (int)ch - cur.sA, chB = (int)ch - cur.sB;
            float gA0 = 0.f, gA1 = 0.f, gB0 = 0.f, gB1 = 0.f, fA0 = 0.f, fA1 = 0.f, fB0 = 0.f, fB1 = 0.f;
            int rA0 = 0, rA1 = 0, rB0 = 0, rB1 = 0;
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                if ((k & 1) == 0) {
                    const uint64_t pa = ps_acc + (ch ? ps_inc : 0ull);
                    const uint32_t ph = hi32(pa);
                    float m_gA, m_gB;
                    win_gains(unit24(ph), m_gA, m_gB);
                    gA0 = pair_even(m_gA); gA1 = pair_odd(m_gA);
                    gB0 = pair_even(m_gB); gB1 = pair_odd(m_gB);
                    uint32_t di; float fr;
                    pitch_split(ph, wi, wf, pmaxu, di, fr);
                    const int ra = chA - (int)di;
                    rA0 = pair_even_i(ra); rA1 = pair_odd_i(ra);
                    fA0 = pair_even(fr); fA1 = pair_odd(fr);
                    pitch_split(ph + 0x80000000u, wi, wf, pmaxu, di, fr);   // p1 = (p0 + 1/2) % 1
                    const int rb = chB - (int)di;
                    rB0 = pair_even_i(rb); rB1 = pair_odd_i(rb);
                    fB0 = pair_even(fr); fB1 = pair_odd(fr);
                }
                ps_acc += ps_inc;
                const bool odd = k & 1;
                const float *qA = wP0 + (k & ~1) * kRow + (odd ? rA1 : rA0) * kRow;
                const float *qB = wP1 + (k & ~1) * kRow + (odd ? rB1 : rB0) * kRow;
                const float tA = lerp_pair(qA[0], qA[-kRow], odd ? fA1 : fA0);
                const float tB = lerp_pair(qB[0], qB[-kRow], odd ? fB1 : fB0);
                psv[k] = xfade(tB, odd ? gB1 : gB0, tA, odd ? gA1 : gA0);
            }
            if (FULL) {
#pragma unroll
                for (int k = 0; k < kChunk; ++k) wC[min(k - cur.sC, kWin) * kRow] = psv[k];
            }
        } else {
            // generic chunk (partial, or a pitch window the lines cannot cover): per frame, with
            // per-frame guards and direct ring reads for the uncovered pitch taps
            float pl_gA[2], pl_gB[2];
#pragma unroll
            for (int k = 0; k < kChunk; ++k) {
                if (OUT_LDS && FULL) yo[k] = 0.f;
                if ((k & 1) == 0) {
                    const uint64_t pa = ps_acc + (ch ? ps_inc : 0ull);
                    float m_gA, m_gB;
                    win_gains(unit24h(pa), m_gA, m_gB);
                    const float o_gA = swap_pair(m_gA), o_gB = swap_pair(m_gB);
                    pl_gA[0] = ch ? o_gA : m_gA;    pl_gA[1] = ch ? m_gA : o_gA;
                    pl_gB[0] = ch ? o_gB : m_gB;    pl_gB[1] = ch ? m_gB : o_gB;
                }
                if (k >= C) { psv[k] = 0.f; continue; }
                const uint64_t lfo_k = lfo_acc + lfo_off;
                const uint32_t ph = hi32(ps_acc);
                const float gA = pl_gA[k & 1];
                const float gB = pl_gB[k & 1];
                lfo_acc += lfo_inc;
                ps_acc += ps_inc;
                uint32_t di; float fr;
                float tA, tB;
                pitch_split(ph, wi, wf, pmaxu, di, fr);
                if (!cur.okA) {
                    const uint32_t q = w0 + k - di;
                    tA = lerp_pair(ld1(rP, own_pb() + (q & pmask) * 8u, 0), ld1(rP, own_pb() + ((q - 1u) & pmask) * 8u, 0), fr);
                } else {
                    const int jw = k - (int)di - cur.sA;
                    tA = lerp_pair(wP0[jw * kRow], wP0[(jw - 1) * kRow], fr);
                }
                pitch_split(ph + 0x80000000u, wi, wf, pmaxu, di, fr);
                if (!cur.okB) {
                    const uint32_t q = w0 + k - di;
                    tB = lerp_pair(ld1(rP, own_pb() + (q & pmask) * 8u, 0), ld1(rP, own_pb() + ((q - 1u) & pmask) * 8u, 0), fr);
                } else {
                    const int jw = k - (int)di - cur.sB;
                    tB = lerp_pair(wP1[jw * kRow], wP1[(jw - 1) * kRow], fr);
                }
                const float p = xfade(tB, gB, tA, gA);
                psv[k] = p;
                float out = p;
                if (FULL) {
                    wC[min(k - cur.sC, kWin) * kRow] = p;
                    chorus_split(lfo_k, D, cmaxd, di, fr);
                    const int jw = k - (int)di - cur.sC;
                    const float wet = lerp_pair(wC[jw * kRow], wC[(jw - 1) * kRow], fr);
                    const float lp = lores_step(wet, b0, b1, b2, a1, a2, z1, z2);
                    out = dry_wet(x[k], dry, lp, mix);
                }
                if (OUT_LDS && FULL) yo[k] = out;
                else sink(k, out);
            }
        }
        // one call site: line registers loaded on two paths meet in a phi, and the copies it needs
        // pushed the kernel from 211 VGPRs to 256 + spills
        stores_and_next<PAR>(psv, x, xn, xq, w0, C, Cn, lfo0, ps0);
        if (OUT_LDS && FULL && !fast) {
            // the generic chunk's outputs leave after the stores and staging above (a COOP sink
            // writes LDS that was the pitch windows until then)
#pragma unroll
            for (int k = 0; k < kChunk; ++k)
                if (k < C) sink(k, yo[k]);
        }
        if (fast) {
            // C. the chorus tap + lores~ (reads independent of each other; only the biquad is serial),
            //    the cover for chunk c+1's line loads
            if (FULL) {
                // the tap delay shared by L and R as in phase A: each lane splits its own frame's
                // (k + ch) delay, DPP hands both frames' slot offsets and fractions to both lanes
                const int chC = (int)ch - cur.sC;
                int r0 = 0, r1 = 0;
                float f0 = 0.f, f1 = 0.f;
                uint32_t dn = 0;                      // the next pair's split, computed with this one's
                float fn = 0.f;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) {
                    if ((k & 1) == 0) {
                        uint32_t di; float fr;
                        if ((k & 3) == 0) {
                            const uint64_t p = lfo_acc + (ch ? lfo_inc : 0ull) + lfo_off;
                            chorus_split2(p, p + 2ull * lfo_inc, D, cmaxd, di, fr, dn, fn);
                        } else {
                            di = dn;
                            fr = fn;
                        }
                        const int rc = chC - (int)di;
                        r0 = pair_even_i(rc); r1 = pair_odd_i(rc);
                        f0 = pair_even(fr); f1 = pair_odd(fr);
                    }
                    lfo_acc += lfo_inc;
                    const bool odd = k & 1;
                    const float *qC = wC + (k & ~1) * kRow + (odd ? r1 : r0) * kRow;
                    const float wet = lerp_pair(qC[0], qC[-kRow], odd ? f1 : f0);
                    const float lp = lores_step(wet, b0, b1, b2, a1, a2, z1, z2);
                    sink(k, dry_wet(x[k], dry, lp, mix));
                }
            } else {
                lfo_acc += (uint64_t)kChunk * lfo_inc;
#pragma unroll
                for (int k = 0; k < kChunk; ++k) sink(k, psv[k]);
            }
        }
        wpos = w0 + (uint32_t)C;
    }

    __device__ __forceinline__ void finish(const ChorusArgs &a) const {
        if (!valid) return;
        if (ch == 0) {
            a.state[CHS_LFO_ACC * n + i] = (uint32_t)(lfo_acc >> 32);
            a.state[CHS_LFO_LO * n + i] = (uint32_t)lfo_acc;
            a.state[CHS_PS_ACC * n + i] = (uint32_t)(ps_acc >> 32);
            a.state[CHS_PS_LO * n + i] = (uint32_t)ps_acc;
        }
        a.state[(ch ? CHS_Z1R : CHS_Z1L) * n + i] = __float_as_uint(z1);
        a.state[(ch ? CHS_Z2R : CHS_Z2L) * n + i] = __float_as_uint(z2);
    }
};

}  // namespace ch
}  // namespace olfx
