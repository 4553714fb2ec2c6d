// ol_dsp_amd/csrc/olfx_internal.h -- kernel argument blocks, ring geometry and the
// host/device-shared scalar DSP helpers of libolfx.so.
//
// Everything here is written for gfx950 (CDNA4, wave64) and compiled with -ffp-contract=off so
// that the device arithmetic is the exact IEEE single-precision sequence the CPU oracle uses.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/olfx.h"

#define OLFX_HD __host__ __device__ __forceinline__

namespace olfx {

// ----------------------------------------------------------------------------------------------
// Dattorro plate: 13 power-of-two rings (reference libs/dattorro-verb/verb.cpp:65-98,173-212).
// ----------------------------------------------------------------------------------------------
enum DtLine {
    DT_PRE = 0, DT_IN0, DT_IN1, DT_IN2, DT_IN3,
    DT_AP1A, DT_DL1A, DT_AP2A, DT_DL2A,
    DT_AP1B, DT_DL1B, DT_AP2B, DT_DL2B,
    DT_NLINES
};
// nominal (TAP_MAIN) delay of each line
constexpr uint32_t kDtDelay[DT_NLINES] = {4800, 142, 107, 379, 277, 672, 4453, 1800, 3720,
                                          908, 4217, 2656, 3163};
// ring size = 2^(bit length of delay)
constexpr uint32_t dt_ring_size(uint32_t d) {
    uint32_t b = 0;
    while (d) { ++b; d >>= 1; }
    return 1u << b;
}
constexpr uint32_t kDtSize[DT_NLINES] = {
    dt_ring_size(4800), dt_ring_size(142), dt_ring_size(107), dt_ring_size(379),
    dt_ring_size(277), dt_ring_size(672), dt_ring_size(4453), dt_ring_size(1800),
    dt_ring_size(3720), dt_ring_size(908), dt_ring_size(4217), dt_ring_size(2656),
    dt_ring_size(3163)};
constexpr uint32_t dt_total_floats() {
    uint32_t s = 0;
    for (int l = 0; l < DT_NLINES; ++l) s += kDtSize[l];
    return s;
}
static_assert(dt_total_floats() == 42368, "dattorro ring geometry");

// Output tap delays (verb.cpp:187-212) and the stereo tap sums (verb.cpp:302-325).
// Left  = +DL1B.o1 +DL1B.o2 -AP2B.o2 +DL2B.o2 -DL1A.o3 -AP2A.o1 +DL2A.o1
// Right = +DL1A.o1 +DL1A.o2 -AP2A.o2 +DL2A.o2 -DL1B.o3 -AP2B.o1 +DL2B.o1
constexpr uint32_t kDl1A_o1 = 353, kDl1A_o2 = 3627, kDl1A_o3 = 1990;
constexpr uint32_t kAp2A_o1 = 187, kAp2A_o2 = 1228;
constexpr uint32_t kDl2A_o1 = 1066, kDl2A_o2 = 2673;
constexpr uint32_t kDl1B_o1 = 266, kDl1B_o2 = 2974, kDl1B_o3 = 2111;
constexpr uint32_t kAp2B_o1 = 335, kAp2B_o2 = 1913;
constexpr uint32_t kDl2B_o1 = 121, kDl2B_o2 = 1996;

// Derived per-instance coefficients (field-major [DTC_N][n] on the device).
// DTC_PREDELAY holds the per-instance pre-delay in samples (an integer 0..4800, exact in fp32).
enum { DTC_PREFILTER = 0, DTC_IN1, DTC_IN2, DTC_DD1, DTC_DAMPING, DTC_DECAY, DTC_DD2, DTC_PREDELAY, DTC_N };
// Per-instance recursive scalar state ([DTS_N][n]).
enum { DTS_LP_PRE = 0, DTS_LP_DAMP_A, DTS_LP_DAMP_B, DTS_N };

// Extra delay of both tank input all-passes at stream time t16 (verb.cpp:262-270): their read
// offset is decremented at every t16 = k*2048 < 32768 and incremented at every k*2048 >= 32768,
// *before* the sample at that t is processed.  For an instance created at t = 0 the count is
// closed-form, so every chunk can compute it without carrying the offset.
OLFX_HD uint32_t dt_ap1_extra(uint32_t t16) {
    uint32_t dec = ((t16 >> 11) < 15u ? (t16 >> 11) : 15u) + 1u;
    uint32_t inc = t16 >= 32768u ? ((t16 - 32768u) >> 11) + 1u : 0u;
    return dec - inc;
}

struct DattorroArgs {
    float *ring[DT_NLINES];     // ring l: [kDtSize[l]][n]   (position-major, instance fastest)
    float *state;               // [DTS_N][n]
    const float *coef;          // [DTC_N][n]
    const float *in;            // [2][..][n], channel planes `plane` floats apart
    float *out;                 // [2][..][n]
    uint64_t plane;             // floats between the channel planes of in / out (>= n_frames * n)
    uint32_t n;                 // instances
    uint32_t n_frames;
    uint32_t t0;                // stream time (frames since create) of the first frame, mod 2^16
    uint32_t in_ch;             // 1 or 2
    uint32_t cus;               // compute units of the device (olfx_create)
};
// Standalone reverb: the network for these pre-delays (dattorro.hip): v4 with the pre-delay ring
// position-major, v5 with it in rows ([8192/16][n][16])
enum { DT_NET_V4 = 0, DT_NET_V5 };
int dattorro_network(uint32_t n, uint32_t cus, bool uniform);
const char *dattorro_network_name(int net);
// the pre-delay ring's content into the other layout (tmp: a device buffer of the ring's size)
hipError_t launch_dattorro_pre_layout(const DattorroArgs &a, float *tmp, bool to_rows, hipStream_t s);

// ----------------------------------------------------------------------------------------------
// Deterministic cos(2*pi*x): used by the chorus LFO (RNBO cycle~).  Branch-free (selects only, no
// lane divergence): reduce to b in [0, 1/4] exactly, then one minimax polynomial of cos in
// theta^2 on [0, pi/2] (degree 8, Remez, coefficients rounded to float; round 2 used the Taylor
// series to theta^14: the same accuracy class at twice the operations).  Only +, -, *, rint and
// compares in a fixed order, so the host (oracle) and gfx950 produce identical bits under
// -ffp-contract=off.  |err| < 3e-7 (measured 1.8e-7; tests/test_oracle.py).
// ----------------------------------------------------------------------------------------------
// Horner in fused multiply-adds (spec v3, round 6: IEEE fusedMultiplyAdd, C fmaf on the host)
OLFX_HD float cos_poly(float t2) {                 // cos(theta), t2 = theta^2, theta in [0, pi/2]
    float r = __builtin_fmaf(2.31943868129747e-05f, t2, -0.001385592739097774f);
    r = __builtin_fmaf(r, t2, 0.041663989424705505f);
    r = __builtin_fmaf(r, t2, -0.4999993145465851f);
    return __builtin_fmaf(r, t2, 1.0f);
}
OLFX_HD float sin_poly(float th, float t2) {       // sin(theta), theta in [0, pi/2]
    float r = __builtin_fmaf(2.6000548132287804e-06f, t2, -0.00019806614727713168f);
    r = __builtin_fmaf(r, t2, 0.008333017118275166f);
    r = __builtin_fmaf(r, t2, -0.16666656732559204f);
    return th * __builtin_fmaf(r, t2, 1.0f);
}
OLFX_HD float cos2pi(float x) {
    const float u = x - rintf(x);                  // exact, u in [-0.5, 0.5]
    const float a = u < 0.0f ? -u : u;             // cos is even
    const bool hi = a > 0.25f;
    const float b = hi ? 0.5f - a : a;             // exact (Sterbenz); cos(2pi(1/2-b)) = -cos(2pi b)
    const float th = b * 6.28318530717958647692f;
    const float r = cos_poly(th * th);
    return hi ? -r : r;
}
// The pitch-shifter's crossfade windows at phasor phase p in [0, 1) (pitchshift.gendsp: tap 0's
// gain cos((p - 1/2) pi), tap 1's cos((p1 - 1/2) pi) with p1 = (p + 1/2) mod 1) are sin(pi p) and
// |cos(pi p)|, i.e. sin(pi q) and cos(pi q) for q = min(p, 1 - p) in [0, 1/2] (1 - p is exact: p is
// a 24-bit fraction): one argument, two short polynomials.
OLFX_HD void win_gains(float p, float &g0, float &g1) {
    const float q = fminf(p, 1.0f - p);
    const float th = q * 3.14159265358979323846f;
    const float t2 = th * th;
    g0 = sin_poly(th, t2);
    g1 = cos_poly(t2);
}

// ----------------------------------------------------------------------------------------------
// Chorus / pitch-shift (spec: DESIGN.md section 3, from modules/rnbo/patcher/mono-chorus.rnbopat
// and pitchshift.gendsp).  Per-instance rings are instance-major ([n][size]) because the taps are
// modulated per instance: each lane streams through its own ring.
// ----------------------------------------------------------------------------------------------
enum {
    // phasors are 64-bit fixed point (2^64 = one cycle), stored as a high and a low word
    CHC_LFO_INC = 0,    // high word of cycle~'s phase increment
    CHC_LFO_OFF,        // high word of cycle~'s phase offset
    CHC_PS_INC,         // high word of the pitch-shifter phasor's increment
    CHC_DEPTH,          // D = mstosamps(1 + 11 depth): high word of the double
    CHC_WINDOW,         // W = mstosamps(window) in 32.32 fixed point: integer part
    CHC_B0, CHC_B1, CHC_B2, CHC_A1, CHC_A2,   // lores~ (RBJ biquad LP, normalised by a0)
    CHC_MIX, CHC_DRY,   // mix, 1 - mix
    CHC_LFO_INC_LO, CHC_LFO_OFF_LO, CHC_PS_INC_LO,   // low words of the three above
    CHC_DEPTH_LO,       // low word of D
    CHC_WINDOW_LO,      // fraction of W (32.32)
    CHC_N
};
enum {
    CHS_LFO_ACC = 0,    // high word of cycle~'s 64-bit phase
    CHS_PS_ACC,         // high word of the pitch-shifter's 64-bit phase
    CHS_Z1L, CHS_Z2L, CHS_Z1R, CHS_Z2R,   // biquad TDF-II state per channel
    CHS_LFO_LO, CHS_PS_LO,                // low words of the two phases
    CHS_N
};

// Tap delays (spec v2, round 4).  Round 3 formed both delays in fp32 from the
// phasors' top 24 bits: the pitch delay p W (W up to 480 samples) to 2^-15 sample, the chorus delay
// D cos + D (D up to 576) from a cosine good to 2e-7, i.e. to ~1e-4 sample -- that, not the fp32
// signal arithmetic, was the spec's deviation from double precision (1.3e-4 / 1.6e-4 of the signal,
// tests/test_oracle.py test_chorus_deviation_by_stage).  Now:
//   pitch-shifter: d = p W in 32.32 fixed point, p = the phasor's high word / 2^32 and W in 32.32
//     (exact integer arithmetic), clamped to [1, pmax]; the fraction rounded once to fp32;
//   chorus: the LFO phase to 53 bits, cos(2 pi x) by a double Taylor polynomial (|err| < 4e-15),
//     d = cos D + D in double (D double), clamped to [0, cmax]; the fraction rounded once to fp32.
//     Spec v2.1 (round 4): the polynomial's Horner steps and cos D + D are fused multiply-adds.
// Gains, interpolation, lores~ and the mix stay fp32.  Host and gfx950 evaluate these identically
// (integer ops, IEEE double +, * and fma in a fixed order, no other contraction).
OLFX_HD void pitch_split(uint32_t ph, uint32_t wi, uint32_t wf, uint32_t pmax, uint32_t &di, float &fr) {
    const uint64_t d = (uint64_t)ph * wi + (((uint64_t)ph * wf) >> 32);     // p W, 32.32
    // clamp to [1, pmax] in 32.32 on the two words (the oracle clamps the 64-bit value; the same
    // result): below 1 or at / above pmax the fraction is 0, the integer part the bound
    const uint32_t dh = (uint32_t)(d >> 32);
    const bool inside = dh >= 1u && dh < pmax;
    di = dh < 1u ? 1u : (dh > pmax ? pmax : dh);
    fr = inside ? (float)(uint32_t)d * 2.3283064365386963e-10f : 0.0f;      // 2^-32: exact scaling
}
// r t2 + c as one v_fma_f64 with the constant in an SGPR pair: left to itself the compiler keeps the
// constants in VGPR pairs and emits v_fmac_f64 (destination = addend), i.e. a v_mov_b64 of the
// constant before each step -- 7 extra VALU per cosine, 8 cosines per lane and chunk in the chorus
OLFX_HD double fma_dc(double r, double t2, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double d;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(d) : "v"(r), "v"(t2), "s"(c));
    return d;
#else
    return __builtin_fma(r, t2, c);
#endif
}
OLFX_HD double cos2pi_d(double x) {
    const double u = x - rint(x);                  // exact, u in [-0.5, 0.5]
    const double a = u < 0.0 ? -u : u;
    const bool hi = a > 0.25;
    const double b = hi ? 0.5 - a : a;             // exact
    const double th = b * 6.283185307179586;
    const double t2 = th * th;
    // cos(th) = sum (-1)^k th^2k / (2k)!, k <= 9 (th <= pi/2: truncation < 4e-15), Horner in th^2
    // with fused multiply-adds (IEEE fusedMultiplyAdd: C fma on the host, v_fma_f64 here -- the
    // same bits; spec v2.1, round 4: half the double operations of the unfused Horner)
    double r = -1.5619206968586225e-16;                        // -1 / 18!
    r = fma_dc(r, t2, 4.779477332387385e-14);                  //  1 / 16!
    r = fma_dc(r, t2, -1.1470745597729725e-11);                // -1 / 14!
    r = fma_dc(r, t2, 2.08767569878681e-09);                   //  1 / 12!
    r = fma_dc(r, t2, -2.755731922398589e-07);                 // -1 / 10!
    r = fma_dc(r, t2, 2.48015873015873e-05);                   //  1 / 8!
    r = fma_dc(r, t2, -0.001388888888888889);                  // -1 / 6!
    r = fma_dc(r, t2, 0.041666666666666664);                   //  1 / 4!
    r = __builtin_fma(r, t2, -0.5);
    r = __builtin_fma(r, t2, 1.0);
    return hi ? -r : r;
}
// cos(2 pi x) for the 53-bit phase x = (phase >> 11) 2^-53, exactly cos2pi_d(x) with its reduction
// done in integers: u = x - rint(x) is the phase's high word read as SIGNED (u in [-1/2, 1/2); at
// x = 1/2, u = -1/2 where rint gives +1/2: the same |u|), and u = hi 2^-32 + (lo >> 11) 2^-53 is one
// exact fma (53 significant bits).  Round 5: 5 VALU instead of 8 for the conversion and reduction.
OLFX_HD double cos2pi_phase(uint64_t phase) {
    const int32_t sh = (int32_t)(uint32_t)(phase >> 32);
    const uint32_t lo = (uint32_t)phase >> 11;
    const double u = __builtin_fma((double)sh, 2.3283064365386963e-10, (double)lo * 1.1102230246251565e-16);
    const double a = __builtin_fabs(u);
    const bool hi = a > 0.25;
    const double b = hi ? 0.5 - a : a;             // exact
    const double th = b * 6.283185307179586;
    const double t2 = th * th;
    double r = -1.5619206968586225e-16;                        // the Horner steps of cos2pi_d
    r = fma_dc(r, t2, 4.779477332387385e-14);
    r = fma_dc(r, t2, -1.1470745597729725e-11);
    r = fma_dc(r, t2, 2.08767569878681e-09);
    r = fma_dc(r, t2, -2.755731922398589e-07);
    r = fma_dc(r, t2, 2.48015873015873e-05);
    r = fma_dc(r, t2, -0.001388888888888889);
    r = fma_dc(r, t2, 0.041666666666666664);
    r = __builtin_fma(r, t2, -0.5);
    r = __builtin_fma(r, t2, 1.0);
    return hi ? -r : r;
}
OLFX_HD double chorus_delay(uint64_t phase, double D, double cmax) {
    const double d = __builtin_fma(cos2pi_phase(phase), D, D);
    // clamp to [0, cmax] as min / max (one v_max_f64 + one v_min_f64; the compare-select form cost
    // two compares, four selects and their hazard waits): equal for every non-NaN d, and d is never
    // -0 (cos = -1 gives D - D = +0)
    return __builtin_fmin(__builtin_fmax(d, 0.0), cmax);
}
OLFX_HD void chorus_split(uint64_t phase, double D, double cmax, uint32_t &di, float &fr) {
    const double d = chorus_delay(phase, D, cmax);
    di = (uint32_t)d;
    fr = (float)(d - (double)di);                  // the subtraction is exact
}
// two chorus_splits with their Horner chains interleaved (each step's operand is two instructions
// back: no dependent double-precision pair back to back), the same operations per phase
OLFX_HD void chorus_split2(uint64_t ph0, uint64_t ph1, double D, double cmax, uint32_t &di0, float &fr0,
                           uint32_t &di1, float &fr1) {
    const int32_t s0 = (int32_t)(uint32_t)(ph0 >> 32), s1 = (int32_t)(uint32_t)(ph1 >> 32);
    const uint32_t l0 = (uint32_t)ph0 >> 11, l1 = (uint32_t)ph1 >> 11;
    const double u0 = __builtin_fma((double)s0, 2.3283064365386963e-10, (double)l0 * 1.1102230246251565e-16);
    const double u1 = __builtin_fma((double)s1, 2.3283064365386963e-10, (double)l1 * 1.1102230246251565e-16);
    const double a0 = __builtin_fabs(u0), a1 = __builtin_fabs(u1);
    const bool h0 = a0 > 0.25, h1 = a1 > 0.25;
    const double b0 = h0 ? 0.5 - a0 : a0, b1 = h1 ? 0.5 - a1 : a1;
    const double th0 = b0 * 6.283185307179586, th1 = b1 * 6.283185307179586;
    const double t0 = th0 * th0, t1 = th1 * th1;
    double r0 = -1.5619206968586225e-16, r1 = -1.5619206968586225e-16;
    r0 = fma_dc(r0, t0, 4.779477332387385e-14);    r1 = fma_dc(r1, t1, 4.779477332387385e-14);
    r0 = fma_dc(r0, t0, -1.1470745597729725e-11);  r1 = fma_dc(r1, t1, -1.1470745597729725e-11);
    r0 = fma_dc(r0, t0, 2.08767569878681e-09);     r1 = fma_dc(r1, t1, 2.08767569878681e-09);
    r0 = fma_dc(r0, t0, -2.755731922398589e-07);   r1 = fma_dc(r1, t1, -2.755731922398589e-07);
    r0 = fma_dc(r0, t0, 2.48015873015873e-05);     r1 = fma_dc(r1, t1, 2.48015873015873e-05);
    r0 = fma_dc(r0, t0, -0.001388888888888889);    r1 = fma_dc(r1, t1, -0.001388888888888889);
    r0 = fma_dc(r0, t0, 0.041666666666666664);     r1 = fma_dc(r1, t1, 0.041666666666666664);
    r0 = __builtin_fma(r0, t0, -0.5);              r1 = __builtin_fma(r1, t1, -0.5);
    r0 = __builtin_fma(r0, t0, 1.0);               r1 = __builtin_fma(r1, t1, 1.0);
    const double c0 = h0 ? -r0 : r0, c1 = h1 ? -r1 : r1;
    const double d0 = __builtin_fmin(__builtin_fmax(__builtin_fma(c0, D, D), 0.0), cmax);
    const double d1 = __builtin_fmin(__builtin_fmax(__builtin_fma(c1, D, D), 0.0), cmax);
    di0 = (uint32_t)d0;
    di1 = (uint32_t)d1;
    fr0 = (float)(d0 - (double)di0);
    fr1 = (float)(d1 - (double)di1);
}

struct ChorusArgs {
    float *pitch_ring;          // [n][psize][2]  (stereo-interleaved: L and R share every tap)
    float *chorus_ring;         // [n][csize][2]
    uint32_t *state;            // [CHS_N][n] (floats stored bitwise)
    const uint32_t *coef;       // [CHC_N][n]
    const float *in;            // [2][..][n], channel planes `plane` floats apart
    float *out;                 // [2][..][n]
    uint64_t plane;             // floats between the channel planes of in / out (>= n_frames * n)
    uint32_t n, n_frames;
    uint32_t t0;                // write position of the first frame (mod ring sizes)
    uint32_t psize, csize;      // ring sizes (powers of two)
    uint32_t mode;              // 0 = full chorus, 1 = pitch-shift stage only
};

// ----------------------------------------------------------------------------------------------
// Voice (SynthVoice): registers only.
// ----------------------------------------------------------------------------------------------
enum {
    VCC_ATK_D0A = 0, VCC_ATK_TGT_A, VCC_DEC_D0A, VCC_REL_D0A, VCC_SUS_A,   // amp env
    VCC_ATK_D0F, VCC_ATK_TGT_F, VCC_DEC_D0F, VCC_REL_D0F, VCC_SUS_F,       // filter env
    VCC_AMP_AMT, VCC_CUTOFF, VCC_FENV_AMT,
    VCC_DAMP_RES,       // 2 * (1 - powf(res, 0.25))   (Svf::SetRes, computed on host)
    VCC_DRIVE,          // pre_drive * res
    VCC_PORT_COEF,      // expf(-1/(htime*sr))
    VCC_FC_MAX,         // sr / 3
    VCC_SR,             // sample rate
    VCC_INV_SR,         // Oscillator sr_recip_ = 1/sr
    VCC_N,
    // MoogFilter voices reuse the Svf-only slots for the daisysp::LadderFilter coefficients
    VCC_LADDER_K = VCC_DAMP_RES,      // 4 * clamp(res, 0, 1.8)        (LadderFilter::SetRes)
    VCC_LADDER_DRIVE = VCC_DRIVE,     // input drive_scaled_ (0.5: Init; MoogFilter::SetDrive is a no-op)
    VCC_LADDER_WREC = VCC_FC_MAX      // sr_int_recip_ = 1 / (4 sr)     (4x oversampling)
};
enum {
    VCS_PHASE = 0, VCS_PORT_Z, VCS_ENVA_X, VCS_ENVF_X, VCS_LOW, VCS_BAND, VCS_FREQ,
    VCS_FLAGS,          // bits 0-2 amp mode, 3-5 filt mode, 6 gate(amp prev), 7 gate(filt prev), 8 gate
    VCS_N,
    // MoogFilter voices append the LadderFilter state: z0_[4], z1_[4], oldinput_ (VCS_LOW/BAND unused)
    VCS_LZ0 = VCS_N, VCS_LZ1 = VCS_LZ0 + 4, VCS_LOLD = VCS_LZ1 + 4,
    VCS_N_MOOG
};
inline bool is_voice_kind(int k) { return k == OLFX_KIND_VOICE || k == OLFX_KIND_VOICE_MOOG; }
inline uint32_t voice_state_slots(int k) { return k == OLFX_KIND_VOICE_MOOG ? (uint32_t)VCS_N_MOOG : (uint32_t)VCS_N; }

// Note events of one block, folded per voice on the host (olfx_engine.cpp fold_events) and applied
// by the voice kernel itself as its first act on the voice's state (SynthVoice.h:231-268: the
// events of a block compose field by field -- the last gate call wins, any NoteOn retriggers, the
// last NoteOn / SetFrequency sets the pitch).
enum : uint32_t {
    VEV_GATE_SET = 1u,          // gate := VEV_GATE_ON bit (NoteOn / GateOn / NoteOff / GateOff)
    VEV_GATE_ON = 2u,
    VEV_RETRIGGER = 4u,         // Adsr::Retrigger(true) on both envelopes: mode ATTACK, x = 0
    VEV_FREQ = 8u,              // freq_ := the record's frequency (mtof(note) for NoteOn, SetFrequency's Hz)
    VEV_MORE = 0x80u,           // (slot 0 of a crowded workgroup) its records are in the overflow list
};
// Event records, 8 B: x = (voice & 63) | VEV_* ops << 8, y = frequency bits; x = 0 is an empty slot.
// Workgroup g (64 voices) owns the kVevCap fixed slots ev[g kVevCap ..]: the kernel reads them in
// one host-link round trip without first reading where they are.  A workgroup with more than
// kVevCap records puts them all in the overflow list and marks slot 0:
// x = VEV_MORE << 8 | count << 16, y = first record in ev_more (a second round trip, for it only).
constexpr uint32_t kVevCap = 4;

struct VoiceArgs {
    float *state;               // [VCS_N][n], MoogFilter voices [VCS_N_MOOG][n]
    const float *coef;          // [VCC_N][n]
    float *out;                 // [1][n_frames][n]
    uint32_t n, n_frames;
    uint32_t moog;              // 1: daisysp::LadderFilter (MoogFilter) in place of the Svf
    // this block's events (nullptr: none), at most one record per voice (kVevCap above)
    const uint2 *ev;            // [n_groups][kVevCap] fixed slots, n_groups = ceil(n / 64)
    const uint2 *ev_more;       // overflow list
};

// Coefficient records of the instances whose parameters changed (olfx_engine.cpp upload_params):
// word w of record r goes to dst[s][(w - first word of segment s) * stride[s] + inst[r]].  Field-
// major records ([w][m]) so consecutive threads write consecutive instances.
struct CoefScatterArgs {
    const uint32_t *inst;       // [m] instance of each record; nullptr = the identity (m == every instance)
    const uint32_t *val;        // [W][m]
    uint32_t m, W;
    uint32_t nseg;
    uint32_t *dst[3];
    uint32_t words[3];          // words of each segment (sum = W)
    uint32_t stride[3];         // instance stride of each segment's field-major array
};
hipError_t launch_coef_scatter(const CoefScatterArgs &a, hipStream_t s);

// ----------------------------------------------------------------------------------------------
// Effect rack ol::fx::FxRack<2> (fxrack.hip): delay lines + two Svf (channel 0) + ReverbSc stub.
// ----------------------------------------------------------------------------------------------
constexpr uint32_t kFrMaxDelay = 48000;     // MAX_DELAY (modules/fxlib/Fx.h:23): ring positions
enum {
    FRC_DELAY = 0,      // uint: DelayLine delay_ (integer part, clamped to 47999)
    FRC_FRAC,           // DelayLine frac_
    FRC_FEEDBACK, FRC_DBAL,
    FRC_DFREQ, FRC_DDAMP, FRC_DDRIVE,       // DelayFx filter_ Svf (LowPass)
    FRC_RBAL,                               // ReverbFx balance
    FRC_FFREQ, FRC_FDAMP, FRC_FDRIVE,       // FxRack filter1 Svf
    FRC_FTYPE,          // uint: 0 low, 1 band, 2 high, 3 notch, 4 peak
    FRC_MASTER,
    FRC_TOPO,           // uint: OLFX_FR_TOPOLOGY (0..4)
    FRC_N
};
enum { FRS_DLOW = 0, FRS_DBAND, FRS_FLOW, FRS_FBAND, FRS_N };
struct FxRackArgs {
    float *ring;                // [n][kFrMaxDelay][2] stereo-interleaved delay lines
    uint32_t *state;            // [FRS_N][n] (floats stored bitwise)
    const uint32_t *coef;       // [FRC_N][n]
    const float *in;            // [2][..][n]
    float *out;                 // [2][..][n]
    uint64_t plane;
    uint32_t n, n_frames;
    uint32_t t0;                // ring position of the first frame: frames since create mod 48000
    uint32_t components;        // some instance is a standalone component (topology 2..4)
};

// Launchers (defined in the .hip files).
hipError_t launch_fxrack(const FxRackArgs &a, hipStream_t s);
// The fused chain (chain.hip): chorus -> pitch-shift -> dattorro in one launch.  c1 / c2 / d
// carry each stage's rings, state and coefficients (their in / out fields are unused); the
// reverb stage's instance count d.n is n rounded up to 64 (padding instances compute harmlessly).
struct ChainArgs {
    ChorusArgs c1, c2;
    DattorroArgs d;
    const float *in;            // [2][..][n]
    float *out;                 // [2][..][n]
    uint64_t plane;             // floats between channel planes of in / out
    uint32_t n, n_frames;       // real instances; frames (multiple of 4)
    uint32_t cus;               // compute units of the device (the persistent grid), from olfx_create
};

hipError_t launch_dattorro(const DattorroArgs &a, int net, hipStream_t s);
hipError_t launch_chain(const ChainArgs &a, hipStream_t s);
hipError_t launch_chorus(const ChorusArgs &a, hipStream_t s);
// the chorus kernel launch_chorus picks for n instances, ring sizes and cooperative I/O

hipError_t launch_voice(const VoiceArgs &a, hipStream_t s);

// ----------------------------------------------------------------------------------------------
// Voice buses (mix.hip): the Polyvoice / VoiceMap sums.  Bus b of frame f = out[f][b] plus the
// voices order[off[b] .. off[b+1]) of in[f][*], added one at a time in that order
// (modules/synthlib/Polyvoice.h:28-33, VoiceMap.h:64-73).
// ----------------------------------------------------------------------------------------------
struct MixArgs {
    const float *in;            // [n_frames][n] voice outputs
    float *out;                 // [n_frames][n_buses], accumulated into
    const uint32_t *off;        // [n_buses + 1]
    const uint32_t *order;      // [off[n_buses]] voice indices
    uint32_t n, n_buses, n_frames;
    // buses are contiguous voice runs in voice order (order[k] == k) on multiples of 4 voices
    // (voice_mix_v4's float4 runs), else 0 (voice_mix_v2)
    uint32_t quad;
};
hipError_t launch_mix(const MixArgs &a, hipStream_t s);

// host side: record a global error message (olfx_last_error(NULL))
void internal_set_error(const char *msg);

}  // namespace olfx
