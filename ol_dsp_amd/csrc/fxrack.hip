// ol_dsp_amd/csrc/fxrack.hip -- the fxlib effect rack ol::fx::FxRack<2> on gfx950.
//
// Reference (modules/fxlib/Fx.h:398-492; oracle/fxrack_ref.c restates it):
//   DelayFx<2>   per channel: r = DelayLine.Read(); DelayLine.Write(in + feedback r);
//                filter_ (Svf LowPass) on channel 0 in place; a = r bal + in (1 - bal)   Fx.h:193-206
//   ReverbFx<2>  over the in-tree ReverbSc stub (Reverb.h:26-31): b = 0.8 a rbal + a (1 - rbal)
//   FilterFx<2>  filter1 (Svf, selected output) on channel 0 only; channel 1 is never written
//                and FxRack's buf_c starts at 0 (Fx.h:408), so output 1 is 0   Fx.h:88-108
//   out = buf_c * master_volume
// Topology 1 (OLFX_FR_TOPOLOGY, the Daisy synth firmware's callback, ol_daisy/app/synth/main.cpp:
// 78-86): DelayFx<1> is the rack's channel-0 delay with its filter; stereo[0] = stereo[1] makes the
// reverb's two outputs equal, FilterFx<2> in place leaves channel 1 at the reverb output, and there
// is no master volume (x 1.0f).  Topologies 2 / 3 / 4 are DelayFx<2>, ReverbFx<2> and FilterFx<2> on
// their own (the firmware's objects outside a rack; the COMP instantiation below).
// DelayLine<float, 48000> (DaisySP, restated): read at delay D and D + 1, linear interpolation,
// read before write.  Here the ring is time-forward (position = t mod 48000) and stereo-
// interleaved [n][48000][2]: both channels share the delay, so one window load serves both.
//
// Mapping (as chorus_stage.h): lane = (instance j of the wave, channel), a wave = 32 instances x
// 2 channels.  The block runs in 16-frame chunks.  A chunk's reads (frame k at t + k - D and one
// below) fall in a window of 18 positions from s = (t - D - 1) rounded down to even, de-interleaved
// into LDS as [slot][lane] (conflict-free per-frame reads).  LINE CARRY (v3): s is even, so the
// window lies in the two 128-B stereo lines L = s / 16 and L + 1 (s mod 16 <= 14); D is fixed
// within a block, so the next chunk's window is lines L + 1 and L + 2.  Each chunk loads only its
// successor's new line (cooperatively, one chunk ahead) and carries the other in registers:
// 8 B read per stereo frame, the algorithmic figure (v2 loaded 10 overlapping 16-B pieces per
// chunk: 23.8 B/frame measured).  The chunk's writes leave as one 128-B stereo run per instance
// (8 lanes x 16 B) from LDS staging.  Delays shorter than a chunk read positions the chunk itself
// writes: every written sample also goes into the window (a junk slot when it falls outside).  A
// carried line was loaded two chunks back, a new one a chunk back, each after the stores of the
// chunks before it: the last two chunks' writes are patched in from registers -- so every delay
// 0..47999 takes the same branch-free path.
// Bound: HBM (32 B per stereo frame: ring write 8 + ring read 8 + I/O 16).
#include <type_traits>
#include <utility>

#include "chorus_stage.h"

namespace olfx {

namespace {

constexpr int kFrThreads = 256;
constexpr int kFrChunk = 16;
constexpr int kFrWin = 20;                          // window slots (18 read) staged from two lines
constexpr int kFrSlots = kFrWin + 1;                // + junk slot
constexpr int kFrStride = 36;                       // staging floats per instance (32 + pad)
constexpr int kFrOutCh = 16 * 32 + 32;              // output staging [ch][frame][instance], per channel
// floats of LDS per wave: the window, the ring-run staging (which also transposes the cooperative
// input rows) and, with cooperative I/O, the output staging
constexpr int kFrRegion = kFrSlots * 64 + 32 * kFrStride + 2 * kFrOutCh;
__device__ __forceinline__ void wave_lds_order() {   // one wave's LDS writes before its other lanes' reads
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Svf::Process (DaisySP, double-sampled Chamberlin) returning the selected output
// (0 low, 1 band, 2 high, 3 notch, 4 peak), as oracle/fxrack_ref.c.  Each output is the mean of its
// two passes' values, 0.5 x1 + 0.5 x2: the pass's value is selected first and only the selected
// output is formed (the same operations for it; the reference forms all five)
__device__ __forceinline__ float svf_pick(uint32_t type, float low, float band, float high, float notch) {
    float peak = low - high;
    asm volatile("" : "+v"(peak));                  // computed for every lane: selects, not branches
    float r = type == 4 ? peak : low;
    r = type == 3 ? notch : r;
    r = type == 2 ? high : r;
    return type == 1 ? band : r;
}
__device__ __forceinline__ float svf_tick(float in, float freq, float damp, float drive, uint32_t type,
                                          float &low, float &band) {
    float notch = in - damp * band;
    low = low + freq * band;
    float high = notch - low;
    band = freq * high + band - drive * band * band * band;
    const float x1 = svf_pick(type, low, band, high, notch);
    notch = in - damp * band;
    low = low + freq * band;
    high = notch - low;
    band = freq * high + band - drive * band * band * band;
    const float x2 = svf_pick(type, low, band, high, notch);
    return 0.5f * x1 + 0.5f * x2;
}

// f(integral_constant<int, 0>) ... f(integral_constant<int, N-1>), unrolled at compile time
template <class F, int... K>
__device__ __forceinline__ void static_for_impl(F &&f, std::integer_sequence<int, K...>) {
    (f(std::integral_constant<int, K>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F &&f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ uint32_t wrap48k(int64_t p) {
    const int64_t m = p % (int64_t)kFrMaxDelay;
    return (uint32_t)(m < 0 ? m + kFrMaxDelay : m);
}

}  // namespace

// COMP = some instance of the engine is a standalone component (OLFX_FR_TOPOLOGY 2 DelayFx<2>,
// 3 ReverbFx<2>, 4 FilterFx<2>; the firmware's objects, ol_daisy/app/synth/main.cpp:82-85): the
// same lanes and ticks, with per-instance selects of what each lane outputs.  Engines of racks only
// (topologies 0 / 1) run COMP = false, the rack's own instruction stream.
// COOP (round 3): the block's audio moves as cooperative (frame, channel) rows of the wave's 32
// instances (4 x 16 B per lane and chunk each way, transposed through LDS, as the chorus) instead of
// 16 + 16 single floats per lane; for n and the plane distance multiples of 4 and 16-B aligned
// buffers.
template <bool COMP, bool COOP>
__global__ __launch_bounds__(kFrThreads) void fxrack_block_v3(FxRackArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    const uint32_t tid = threadIdx.x;
    const uint32_t wib = (uint32_t)__builtin_amdgcn_readfirstlane((int)(tid >> 6));
    const uint32_t wave = blockIdx.x * (kFrThreads / 64) + wib, lane = tid & 63u;
    const uint32_t j = lane >> 1, ch = lane & 1u;
    const uint32_t inst0 = wave * 32u;
    const uint32_t n = a.n, nf = a.n_frames;
    if (inst0 >= n) return;
    const uint32_t i_raw = inst0 + j;
    const bool valid = i_raw < n;
    const uint32_t i = valid ? i_raw : n - 1;

    const uint32_t D = a.coef[FRC_DELAY * n + i];
    const float frac = __uint_as_float(a.coef[FRC_FRAC * n + i]);
    const float feedback = __uint_as_float(a.coef[FRC_FEEDBACK * n + i]);
    const float dbal = __uint_as_float(a.coef[FRC_DBAL * n + i]);
    const float dfreq = __uint_as_float(a.coef[FRC_DFREQ * n + i]);
    const float ddamp = __uint_as_float(a.coef[FRC_DDAMP * n + i]);
    const float ddrive = __uint_as_float(a.coef[FRC_DDRIVE * n + i]);
    const float rbal = __uint_as_float(a.coef[FRC_RBAL * n + i]);
    const float ffreq = __uint_as_float(a.coef[FRC_FFREQ * n + i]);
    const float fdamp = __uint_as_float(a.coef[FRC_FDAMP * n + i]);
    const float fdrive = __uint_as_float(a.coef[FRC_FDRIVE * n + i]);
    const uint32_t ftype = a.coef[FRC_FTYPE * n + i];
    const float master = __uint_as_float(a.coef[FRC_MASTER * n + i]);
    // topology 1 (the synth firmware's callback): lane D's output is channel 1 = the reverb
    // output of the mono delay's stereo copy, which equals channel 0's reverb output b0
    const uint32_t topo = a.coef[FRC_TOPO * n + i];
    const bool fw = topo == 1u;
    // components: lane F's channel-0 output is D's value of the previous frame for DelayFx and
    // ReverbFx (no filter1); lane D's channel-1 output is F's value of the previous frame for all
    // three.  filter1 (lane F's Svf) keeps its state only where it runs: racks and FilterFx.
    const bool comp = COMP && topo >= 2u;
    const bool pass0 = COMP && (topo == 2u || topo == 3u);
    const bool filt_on = !COMP || !pass0;
    // Lane roles (v2): both filters act on channel 0 only (Fx.h:88-108, DelayFx filter_), so the
    // lane pair of an instance splits them: lane ch 0 ("D") runs DelayFx's filter_, lane ch 1 ("F")
    // runs FxRack's filter1 one tick behind, on D's reverb output of the previous frame (a DPP
    // broadcast).  A chunk of C frames is C + 1 ticks of ONE svf_tick per lane instead of two.
    const float sfreq = ch ? ffreq : dfreq, sdamp = ch ? fdamp : ddamp, sdrive = ch ? fdrive : ddrive;
    const uint32_t stype = ch ? ftype : 0u;
    float slow = __uint_as_float(a.state[(ch ? FRS_FLOW : FRS_DLOW) * n + i]);
    float sband = __uint_as_float(a.state[(ch ? FRS_FBAND : FRS_DBAND) * n + i]);

    // the wave's 32 rings (12.3 MB) get their own descriptor, so 32-bit offsets cover any n
    const ch::Rsrc rR = ch::rsrc(a.ring + (size_t)inst0 * kFrMaxDelay * 2, (uint64_t)min(32u, n - inst0) * kFrMaxDelay * 8);
    const ch::Rsrc rIn = ch::rsrc(a.in, (a.plane + (uint64_t)nf * n) * 4);
    const ch::Rsrc rOut = ch::rsrc(a.out, (a.plane + (uint64_t)nf * n) * 4);
    const uint32_t io_v = ch * (uint32_t)a.plane * 4u + i * 4u, frame_b = n * 4u;
    // lane F holds channel 0's output, lane D channel 1's (0): each stores the other plane
    const uint32_t out_v = valid ? (1u - ch) * (uint32_t)a.plane * 4u + i * 4u : 0xFFFFFFF0u;
    constexpr uint32_t kRing = kFrMaxDelay * 8u;        // bytes per instance ring

    float *win = lds + wib * kFrRegion;                 // [kFrSlots][64]
    float *wcol = win + lane;
    float *stage = win + kFrSlots * 64;                 // [32][kFrStride]
    float *ostage = stage + 32 * kFrStride;             // COOP: [ch][frame][instance]
    // COOP rows: row r = 8 q + lane / 8 of instruction q is (frame r / 2, channel r % 2) of
    // instances pinst .. + 3
    const uint32_t pinst = inst0 + (lane & 7u) * 4u;
    auto row_r = [&](int q) { return (uint32_t)q * 8u + (lane >> 3); };
    auto row_v = [&](int q, uint32_t f) {
        const uint32_t r = row_r(q);
        return (r & 1u) * (uint32_t)a.plane * 4u + min(f + (r >> 1), nf - 1u) * frame_b + pinst * 4u;
    };
    float4 xq[4];
    // the rows -> the staging [instance][2 frame + ch] -> this lane's frames (k < Cx; else 0)
    auto rows_to_lanes = [&](float (&xv)[kFrChunk], int Cx) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float *st = stage + (lane & 7u) * 4u * kFrStride + row_r(q);
            st[0] = xq[q].x;
            st[kFrStride] = xq[q].y;
            st[2 * kFrStride] = xq[q].z;
            st[3 * kFrStride] = xq[q].w;
        }
        wave_lds_order();
        const float *own = stage + j * kFrStride + ch;
#pragma unroll
        for (int k = 0; k < kFrChunk; ++k) xv[k] = k < Cx ? own[2 * k] : 0.f;
        wave_lds_order();
    };

    // window of the chunk starting at t: first position (t - D - 1) rounded down to even, as an
    // offset from t -- the same for every chunk (t is even)
    auto rel_of = [&](uint32_t t) { return (int)(((int64_t)t - (int64_t)D - 1) & ~(int64_t)1) - (int)t; };
    // Cooperative line loads: piece P = r * 64 + lane of 256 -> piece m = 2 r + lane / 32 (16 B:
    // positions 2m, 2m + 1 of the line) of instance jj = lane % 32 (instances innermost: a
    // ds_write_b64 lane group of 16 contiguous lanes stages one piece of 16 instances, 16 distinct
    // bank pairs, conflict-free).  Every part of a lane serves the same instance jj, whose window
    // start (ring position, wrapped) comes from lane 2 jj once per launch.
    const uint32_t jj = lane & 31u;
    const uint32_t oj = min(inst0 + jj, n - 1) - inst0;      // ring within the wave's descriptor
    const uint32_t spos = (uint32_t)__builtin_amdgcn_ds_bpermute(
        (int)(jj << 3), (int)wrap48k(((int64_t)a.t0 - (int64_t)D - 1) & ~(int64_t)1));
    const uint32_t so15 = spos & 15u;                   // window start within its line (even)
    uint32_t lcur = spos >> 4;                          // line L of the current chunk (instance jj)
    constexpr uint32_t kLines = kFrMaxDelay / 16u;      // 3000 lines per ring: wraps at a line edge
    float4 lo[4], nx[4];                                // lines L (carried) and L + 1 (loaded a chunk back)
    auto load_line = [&](float4 (&dst)[4], uint32_t line) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
            dst[r] = ch::ld4(rR, oj * kRing + line * 128u + ((uint32_t)r * 2u + (lane >> 5)) * 16u);
    };
    auto next_line = [&](uint32_t l) { return l + 1u == kLines ? 0u : l + 1u; };
    auto stage_lines = [&]() {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = r * 2 + (int)(lane >> 5);
            const int slo = 2 * m - (int)so15, shi = slo + 16;   // slots of the piece in L, L + 1
            if (slo >= 0) {
                float *p = win + (uint32_t)slo * 64u + 2u * jj;
                *(float2 *)p = make_float2(lo[r].x, lo[r].y);
                *(float2 *)(p + 64) = make_float2(lo[r].z, lo[r].w);
            }
            if (shi < kFrWin) {                         // shi + 1 <= kFrWin: the junk slot at most
                float *p = win + (uint32_t)shi * 64u + 2u * jj;
                *(float2 *)p = make_float2(nx[r].x, nx[r].y);
                *(float2 *)(p + 64) = make_float2(nx[r].z, nx[r].w);
            }
        }
    };

    float x[kFrChunk], xn[kFrChunk], y[kFrChunk], y2[kFrChunk];
    const uint32_t t00 = a.t0;                          // ring position of frame 0
    int C = (int)min((uint32_t)kFrChunk, nf);
    if constexpr (COOP) {
#pragma unroll
        for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, 0));
        rows_to_lanes(x, C);
    } else {
#pragma unroll
        for (int k = 0; k < kFrChunk; ++k) x[k] = k < C ? ch::ld1(rIn, io_v, (uint32_t)k * frame_b) : 0.f;
    }
    load_line(lo, lcur);
    load_line(nx, next_line(lcur));
    // A chunk's stores (ring run and outputs) are issued at the start of the NEXT chunk, ahead of
    // that chunk's loads: the compiler drains vmcnt to 0 at the loop head (the loop carries
    // in-flight loads), so every memory operation should be issued early in the iteration, where
    // the whole chunk's arithmetic covers its latency -- not at the end, where the drain would
    // expose the stores' round trip once per chunk.
    float o[kFrChunk];
    auto flush = [&](uint32_t fp, int Cp) {             // the stores of the chunk at frame fp
        const uint32_t tp = t00 + fp;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t q = (uint32_t)r * 64u + lane, oo = q >> 3, f2 = 2u * (q & 7u);
            const float4 vv = *(const float4 *)(stage + oo * kFrStride + 2u * f2);
            const uint32_t oi = inst0 + oo;
            const bool ok = oi < n && (int)f2 < Cp;     // else an offset past the buffer: dropped
            ch::st4(rR, ok ? oo * kRing + wrap48k((int64_t)tp + f2) * 8u : 0xFFFFFFF0u, vv);
        }
        if constexpr (COOP) {
            // the outputs, staged [ch][frame][instance] by the chunk (lane ch holds plane 1 - ch)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const uint32_t r = row_r(q), f = r >> 1;
                const float4 v = *(const float4 *)(ostage + (r & 1u) * kFrOutCh + f * 32u + (lane & 7u) * 4u);
                const bool ok = pinst < n && (int)f < Cp;
                ch::st4(rOut, ok ? (r & 1u) * (uint32_t)a.plane * 4u + (fp + f) * frame_b + pinst * 4u : 0xFFFFFFF0u, v);
            }
        } else {
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k)
                if (k < Cp) ch::st1(rOut, out_v, (fp + (uint32_t)k) * frame_b, o[k]);
        }
    };
    for (uint32_t f0 = 0; f0 < nf; f0 += kFrChunk) {
        C = (int)min((uint32_t)kFrChunk, nf - f0);
        const int Cn = f0 + kFrChunk < nf ? (int)min((uint32_t)kFrChunk, nf - f0 - kFrChunk) : 0;
        const uint32_t t = t00 + f0;                    // chunk's first position, unreduced
        const int rel = rel_of(t);
        // ---- 1. this chunk's window -> LDS from its two lines, patched with the last two chunks'
        //         writes: line L was loaded before chunk c-2's stores, L + 1 before chunk c-1's ----
        stage_lines();
        // (only delays below 2 chunks + a window reach those positions: skipped wave-uniformly
        // otherwise; rel = -D - 1 or -D - 2)
        if (f0 >= 2u * kFrChunk && __builtin_amdgcn_ballot_w64(-2 * kFrChunk - rel < kFrWin)) {
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k) {
                const int s = k - 2 * kFrChunk - rel;   // slot of position t - 32 + k
                if (s >= 0 && s < kFrWin) wcol[s * 64] = y2[k];
            }
        }
        if (f0 > 0 && __builtin_amdgcn_ballot_w64(-kFrChunk - rel < kFrWin)) {
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k) {
                const int s = k - kFrChunk - rel;       // slot of position t - 16 + k
                if (s >= 0 && s < kFrWin) wcol[s * 64] = y[k];
            }
        }
        if (f0 > 0) flush(f0 - kFrChunk, kFrChunk);     // the previous chunk was full
        // ---- 2. the next chunk's inputs and new line in flight (unconditional); L + 1 is carried ----
        if constexpr (COOP) {
#pragma unroll
            for (int q = 0; q < 4; ++q) xq[q] = ch::ld4(rIn, row_v(q, f0 + kFrChunk));
        } else {
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k) {
                const float vv = ch::ld1(rIn, io_v, min(f0 + kFrChunk + (uint32_t)k, nf - 1u) * frame_b);
                xn[k] = k < Cn ? vv : 0.f;
            }
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) lo[r] = nx[r];
        lcur = next_line(lcur);
        load_line(nx, next_line(lcur));
#pragma unroll
        for (int k = 0; k < kFrChunk; ++k) y2[k] = y[k];
        // ---- 3. the frames: C + 1 ticks; tick k runs frame k's delay line (both lanes, own
        //         channel) and one filter step per lane: D on frame k, F on frame k - 1 ----
        float b0p = 0.f;                                // F's input: D's b0 of the previous tick
        float a1p = 0.f;                                // components: F's value of the previous tick
        auto tick = [&](auto generic_tag, auto k_tag) {
            constexpr bool GENERIC = decltype(generic_tag)::value;
            constexpr int k = decltype(k_tag)::value;
            constexpr int kk = k < kFrChunk ? k : kFrChunk - 1;   // array index (tick kFrChunk has no frame)
            if (GENERIC && k > C) return;
            const bool frame_k = !GENERIC ? k < kFrChunk : k < C;   // this tick has a frame k
            float r = 0.f;
            if (frame_k) {
                // DelayLine::Read: a at delay D, b at D + 1 (slots k - D - rel, one below)
                const int sa = k - (int)D - rel;
                const float av = wcol[sa * 64], bv = wcol[(sa - 1) * 64];
                r = av + (bv - av) * frac;
                const float w = x[kk] + (feedback * r); // DelayLine::Write
                y[kk] = w;
                wcol[min(k - rel, kFrWin) * 64] = w;    // visible to later frames of this chunk
            }
            float lo = slow, ba = sband;
            const float so = svf_tick(ch ? b0p : r, sfreq, sdamp, sdrive, stype, lo, ba);
            // D steps on frames 0..C-1, F on frames -1+1..C: the idle end of each lane keeps its state
            const bool commit = ch ? (k >= 1 && filt_on) : frame_k;
            slow = commit ? lo : slow;
            sband = commit ? ba : sband;
            // F: channel 0 of frame k-1; D: channel 1 (0, or in topology 1 frame k-1's b0)
            if constexpr (!COMP) {
                if constexpr (k >= 1) o[k - 1] = (ch ? so : (fw ? b0p : 0.0f)) * master;
            } else {
                if constexpr (k >= 1) {
                    // every candidate in a register first: a select chain, not exec-mask branches
                    float f_out = so * master, d_in = fw ? b0p : 0.0f;
                    asm volatile("" : "+v"(f_out), "+v"(d_in));
                    d_in = comp ? a1p : d_in;
                    o[k - 1] = ch ? (pass0 ? b0p : f_out) : d_in * master;
                }
            }
            if (frame_k) {
                if constexpr (!COMP) {
                    // DelayFx: a = filtered * balance + in * (1 - balance) (D lane: channel 0)
                    const float a0 = (so * dbal) + (x[kk] * (1 - dbal));
                    // ReverbFx over the ReverbSc stub
                    const float vb = a0 * 0.8f;
                    const float b0 = (vb * rbal) + (a0 * (1 - rbal));
                    b0p = ch::pair_even(b0);
                } else {
                    // DelayFx's out = buf balance + in (1 - balance): D on its filtered read (channel 0),
                    // F on its raw read (channel 1 has no filter, FilterFx acts on channel 0 only)
                    const float da = ((ch ? r : so) * dbal) + (x[kk] * (1 - dbal));
                    // ReverbFx over the stub: on the delay's output, or on the input when alone
                    float dav = da, xin = x[kk];
                    const float src = topo == 3u ? xin : dav;
                    float rv = ((src * 0.8f) * rbal) + (src * (1 - rbal));
                    asm volatile("" : "+v"(rv), "+v"(dav), "+v"(xin));   // selects, not branches
                    // D: the value lane F filters / outputs next tick; F: its channel-1 output
                    float val = topo == 4u ? xin : rv;
                    val = topo == 2u ? dav : val;
                    b0p = ch::pair_even(val);
                    a1p = ch::pair_odd(val);
                }
            }
        };
        if (C == kFrChunk) static_for<kFrChunk + 1>([&](auto kt) { tick(std::false_type{}, kt); });
        else static_for<kFrChunk + 1>([&](auto kt) { tick(std::true_type{}, kt); });
        if constexpr (COOP) {
            // the next chunk's input rows through the staging (free since this chunk's flush) into
            // the lanes, and this chunk's outputs into their staging (read by the next flush)
            rows_to_lanes(xn, Cn);
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k) ostage[(1u - ch) * kFrOutCh + (uint32_t)k * 32u + j] = o[k];
        }
        // ---- 4. the chunk's writes -> LDS staging ([instance][frame][ch]); they leave as 128-B
        //         runs (8 lanes each) with the next chunk's flush ----
        {
            float *st = stage + j * kFrStride + ch;
#pragma unroll
            for (int k = 0; k < kFrChunk; ++k) st[2 * k] = y[k];
        }
#pragma unroll
        for (int k = 0; k < kFrChunk; ++k) x[k] = xn[k];
    }
    {
        const uint32_t fl = (nf - 1u) / kFrChunk * kFrChunk;   // the last chunk
        flush(fl, (int)(nf - fl));
    }
    if (!valid) return;
    a.state[(ch ? FRS_FLOW : FRS_DLOW) * n + i] = __float_as_uint(slow);
    a.state[(ch ? FRS_FBAND : FRS_DBAND) * n + i] = __float_as_uint(sband);
}

hipError_t launch_fxrack(const FxRackArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((a.n_frames & 3u) || (a.t0 & 1u) || a.t0 >= kFrMaxDelay) return hipErrorInvalidValue;
    if ((a.plane + (uint64_t)a.n_frames * a.n) * 4 >= (1ull << 32)) return hipErrorInvalidValue;
    const uint32_t waves = (a.n + 31) / 32;
    const uint32_t blocks = (waves + kFrThreads / 64 - 1) / (kFrThreads / 64);
    const size_t lds = (size_t)(kFrThreads / 64) * kFrRegion * sizeof(float);
    const bool coop = (a.n & 3u) == 0 && (a.plane & 3u) == 0 &&
                      (((uintptr_t)a.in | (uintptr_t)a.out) & 15u) == 0;
    if (a.components) {
        if (coop) hipLaunchKernelGGL((fxrack_block_v3<true, true>), dim3(blocks), dim3(kFrThreads), lds, s, a);
        else hipLaunchKernelGGL((fxrack_block_v3<true, false>), dim3(blocks), dim3(kFrThreads), lds, s, a);
    } else {
        if (coop) hipLaunchKernelGGL((fxrack_block_v3<false, true>), dim3(blocks), dim3(kFrThreads), lds, s, a);
        else hipLaunchKernelGGL((fxrack_block_v3<false, false>), dim3(blocks), dim3(kFrThreads), lds, s, a);
    }
    return hipGetLastError();
}

}  // namespace olfx
