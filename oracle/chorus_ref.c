/*
 * oracle/chorus_ref.c -- CPU spec oracle for the RNBO stereo chorus and the gen~ pitch-shifter.
 *
 * TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).  Never part of the product.
 *
 * Parity status: UNPINNED.  The reference defines the chorus and pitch-shift only as Max/RNBO and
 * gen~ patches (modules/rnbo/patcher/mono-chorus.rnbopat, stereo-chorus.rnbopat,
 * pitchshift.gendsp); Max/RNBO/genlib are proprietary and absent, and the RNBO C++ export is
 * git-ignored (modules/rnbo/patcher/.gitignore:1).  No reference test, fixture or golden vector
 * covers them.  This file restates the patch dataflow exactly as written (per-object citations
 * below) with the build's declared spec choices:
 *   - fp32 signal arithmetic (gen~/RNBO compute in double);
 *   - phasors as 64-bit fixed-point accumulators (2^64 = one cycle; the increment rounding drifts a
 *     phase by < 2^-64 cycle per sample), their top 24 bits -> the float phase of the crossfade
 *     gains (exact);
 *   - tap delays precise (spec v2, round 4): the pitch-shifter's p W in 32.32 fixed point from the
 *     phasor's high word (pitch_split), the chorus's D cos(2 pi x) + D in double from a 53-bit phase
 *     and a double Taylor cosine (chorus_split); each split into an integer delay and an fp32
 *     fraction.  Round 3 formed both delays in fp32 (2^-15 .. 1e-4 sample of error), which was the
 *     whole of the spec's 1.3e-4 / 1.6e-4 deviation from double arithmetic;
 *   - cos(2 pi x) by a fixed minimax polynomial (oracle_cos2pi below), standing in for cycle~'s
 *     wavetable, and the crossfade windows cos((p - .5) pi) by sin / cos polynomials of one
 *     argument (oracle_win_gains), standing in for gen~'s cos;
 *   - gen Delay.read: linear interpolation, delay clamped to [1, size-2] (read before write);
 *     RNBO delay~: linear interpolation, delay clamped to [0, size-2] (write before read);
 *   - lores~: RBJ biquad low-pass (transposed direct form II), Q = 1/sqrt(2) + 20 q^3;
 *   - spec v3 (round 6): the fp32 signal path in fused multiply-adds -- the gain polynomials'
 *     Horner steps, interpolation x0 + fr (x1 - x0), the crossfade t1 g1 + t0 g0, lores~ and the
 *     dry / wet mix, each as written here (C99 fmaf, as the GPU's v_fma_f32).
 *
 * Dataflow (mono-chorus.rnbopat patchlines):
 *   in~1 -> gen~ pitchshift (:1119) -> delay~ (:1793) -> lores~ (:1808) -> *~ mix (:1302) -> +~ -> out~1
 *   in~1 -> *~ (1 - mix) (:1157, !- 1 :1176) -> +~ (:1191)
 *   param rate (:4353) -> scale 0 1 0.01 0.5 (:3935) -> cycle~ freq (:3002); param phase (:3420) -> cycle~ phase
 *   param depth (:3854) -> scale 0 1 1 12 1 (:3436) -> mstosamps (:3897) = D;
 *   cycle~ * D (:2935) + D (:2920) -> delay~ time;  param cutoff (:2660) -> scale 0 1 300 15000 1
 *   (:2242) -> lores~ cutoff; param q (:2226) -> lores~ resonance
 * pitchshift gencode (mono-chorus.rnbopat:962, pitchshift.gendsp:19-305):
 *   W = mstosamps(window); ph = phasor(in2); p0 = ph % 1; p1 = (ph + .5) % 1;
 *   out1 = read(p1 W) cos((p1-.5) pi) + read(p0 W) cos((p0-.5) pi); write(in1)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static float clampf_(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

static uint32_t pow2ge(uint32_t x) { uint32_t p = 1; while (p < x) p <<= 1; return p; }

#define TWO64 18446744073709551616.0

/* a fraction of a cycle [0, 1] as 64-bit fixed point; 1.0 (and anything rounding to it) wraps to 0 */
static uint64_t fix64(double cycles)
{
    const double v = floor(cycles * TWO64 + 0.5);
    return v <= 0 ? 0u : (v >= TWO64 ? (uint64_t)(v - TWO64) : (uint64_t)v);
}

/* the float phase of a 64-bit accumulator: its top 24 bits, exact in fp32 */
static float unit24(uint64_t acc) { return (float)((uint32_t)(acc >> 32) >> 8) * 5.9604644775390625e-8f; }

/* minimax polynomials on [0, pi/2] in theta^2 (degree 8 cos, degree 9 sin; Remez, coefficients
   rounded to float): the same operations in the same order as the GPU (spec choice, DESIGN.md
   section 3); Horner in fused multiply-adds (spec v3, round 6: C99 fmaf, correctly rounded, as
   v_fma_f32) */
static float cos_poly(float t2)
{
    float r = fmaf(2.31943868129747e-05f, t2, -0.001385592739097774f);
    r = fmaf(r, t2, 0.041663989424705505f);
    r = fmaf(r, t2, -0.4999993145465851f);
    return fmaf(r, t2, 1.0f);
}

static float sin_poly(float th, float t2)
{
    float r = fmaf(2.6000548132287804e-06f, t2, -0.00019806614727713168f);
    r = fmaf(r, t2, 0.008333017118275166f);
    r = fmaf(r, t2, -0.16666656732559204f);
    return th * fmaf(r, t2, 1.0f);
}

/* cos(2 pi x): reduce to b in [0, 1/4] (exact), then cos_poly */
float oracle_cos2pi(float x)
{
    const float u = x - rintf(x);
    const float a = u < 0.0f ? -u : u;
    const int hi = a > 0.25f;
    const float b = hi ? 0.5f - a : a;
    const float th = b * 6.28318530717958647692f;
    const float r = cos_poly(th * th);
    return hi ? -r : r;
}

/* the crossfade windows of the pitch-shifter at phase p (pitchshift.gendsp: cos((p0 - .5) pi) and
   cos((p1 - .5) pi), p1 = (p0 + .5) % 1) = sin(pi q), cos(pi q), q = min(p, 1 - p) */
void oracle_win_gains(float p, float *g0, float *g1)
{
    const float q = fminf(p, 1.0f - p);
    const float th = q * 3.14159265358979323846f;
    const float t2 = th * th;
    *g0 = sin_poly(th, t2);
    *g1 = cos_poly(t2);
}

typedef struct {
    uint64_t lfo_inc, lfo_off, ps_inc, Wfix;   /* Wfix: W in 32.32 fixed point */
    double D;
    float b0, b1, b2, a1, a2, mix, dry;
} chcoef_t;

typedef struct {
    uint64_t lfo_acc, ps_acc;
    float z1[2], z2[2];
    float *pring[2], *cring[2];
} chstate_t;

struct oracle_chorus {
    int n, mode;
    double sr;
    uint32_t psize, csize;
    uint64_t w;                /* stream write position */
    float *pool;
    chcoef_t *k;
    chstate_t *s;
    float *params;             /* [n][OCH_NPARAMS] */
};

static void derive(const float *p, double sr, chcoef_t *c)
{
    const double pitch = clampf_(p[OCH_PITCH], 0.0f, 3.0f);
    const double mix = clampf_(p[OCH_MIX], 0.0f, 1.0f);
    const double q = clampf_(p[OCH_Q], 0.0f, 1.0f);
    const double cutoff = clampf_(p[OCH_CUTOFF], 0.0f, 1.0f);
    const double phase = clampf_(p[OCH_PHASE], 0.0f, 1.0f);
    const double depth = clampf_(p[OCH_DEPTH], 0.08f, 1.0f);
    const double rate = clampf_(p[OCH_RATE], 0.01f, 1.0f);
    const double window = clampf_(p[OCH_WINDOW], 4.0f, 10.0f);
    const double rate_hz = 0.01 + rate * (0.5 - 0.01);
    const double depth_ms = 1.0 + depth * (12.0 - 1.0);
    const double fc = 300.0 + cutoff * (15000.0 - 300.0);
    c->lfo_inc = fix64(rate_hz / sr);
    c->lfo_off = fix64(phase);                 /* phase 1.0 wraps to 0: L and R share the LFO */
    c->ps_inc = fix64(pitch / sr);
    c->D = depth_ms * sr / 1000.0;
    c->Wfix = (uint64_t)floor(window * sr / 1000.0 * 4294967296.0 + 0.5);
    const double Q = 0.70710678118654752 + 20.0 * q * q * q;
    const double w0 = 2.0 * 3.14159265358979323846 * fc / sr;
    const double cw = cos(w0), sw = sin(w0);
    const double alpha = sw / (2.0 * Q);
    const double a0 = 1.0 + alpha;
    c->b0 = (float)((1.0 - cw) * 0.5 / a0);
    c->b1 = (float)((1.0 - cw) / a0);
    c->b2 = (float)((1.0 - cw) * 0.5 / a0);
    c->a1 = (float)(-2.0 * cw / a0);
    c->a2 = (float)((1.0 - alpha) / a0);
    c->mix = (float)mix;
    c->dry = 1.0f - c->mix;
}

static void default_params(float *p)
{
    p[OCH_PITCH] = 0.0f; p[OCH_MIX] = 0.5f; p[OCH_Q] = 0.5f; p[OCH_CUTOFF] = 0.3f;
    p[OCH_PHASE] = 1.0f; p[OCH_DEPTH] = 0.5f; p[OCH_RATE] = 0.2f; p[OCH_WINDOW] = 10.0f;
}

oracle_chorus *oracle_chorus_create(int n_inst, float sample_rate, int mode)
{
    if (n_inst <= 0 || (mode != 0 && mode != 1)) return NULL;
    oracle_chorus *o = (oracle_chorus *)calloc(1, sizeof(*o));
    if (!o) return NULL;
    o->n = n_inst;
    o->mode = mode;
    o->sr = sample_rate;
    o->psize = pow2ge((uint32_t)ceil(10.0 * sample_rate / 1000.0) + 2);
    o->csize = pow2ge(2u * (uint32_t)ceil(12.0 * sample_rate / 1000.0) + 2);
    const size_t per = 2u * (o->psize + o->csize);
    o->pool = (float *)calloc(per * (size_t)n_inst, sizeof(float));
    o->k = (chcoef_t *)calloc((size_t)n_inst, sizeof(chcoef_t));
    o->s = (chstate_t *)calloc((size_t)n_inst, sizeof(chstate_t));
    o->params = (float *)calloc((size_t)n_inst * OCH_NPARAMS, sizeof(float));
    if (!o->pool || !o->k || !o->s || !o->params) { oracle_chorus_destroy(o); return NULL; }
    for (int i = 0; i < n_inst; i++) {
        float *base = o->pool + per * (size_t)i;
        o->s[i].pring[0] = base;
        o->s[i].pring[1] = base + o->psize;
        o->s[i].cring[0] = base + 2 * o->psize;
        o->s[i].cring[1] = base + 2 * o->psize + o->csize;
        default_params(o->params + (size_t)i * OCH_NPARAMS);
        derive(o->params + (size_t)i * OCH_NPARAMS, o->sr, &o->k[i]);
    }
    return o;
}

void oracle_chorus_destroy(oracle_chorus *o)
{
    if (!o) return;
    free(o->pool); free(o->k); free(o->s); free(o->params); free(o);
}

int oracle_chorus_set(oracle_chorus *o, int inst, int field, float value)
{
    if (!o || inst < 0 || inst >= o->n || field < 0 || field >= OCH_NPARAMS) return -1;
    o->params[(size_t)inst * OCH_NPARAMS + field] = value;
    derive(o->params + (size_t)inst * OCH_NPARAMS, o->sr, &o->k[inst]);
    return 0;
}

/* linear interpolation at delay di + fr (gen Delay.read / delay~): x0 + fr (x1 - x0), one fused
   multiply-add (spec v3) */
static float read_split(const float *ring, uint32_t mask, uint32_t w, uint32_t di, float fr)
{
    const float x0 = ring[(w - di) & mask];
    const float x1 = ring[(w - di - 1u) & mask];
    return fmaf(fr, x1 - x0, x0);
}

/* the pitch-shifter's tap delay p W, p = ph / 2^32 (the phasor's high word), W = Wfix / 2^32:
   32.32 fixed point by exact integer arithmetic, clamped to [1, pmax], fraction rounded to fp32 */
static void pitch_split(uint32_t ph, uint64_t Wfix, uint32_t pmax, uint32_t *di, float *fr)
{
    const uint64_t d = (uint64_t)ph * (uint32_t)(Wfix >> 32) + (((uint64_t)ph * (uint32_t)Wfix) >> 32);
    const uint64_t lo = 1ull << 32, hi = (uint64_t)pmax << 32;
    const uint64_t c = d < lo ? lo : (d > hi ? hi : d);
    *di = (uint32_t)(c >> 32);
    *fr = (float)(uint32_t)c * 2.3283064365386963e-10f;
}

/* cos(2 pi x) in double: exact reduction to b in [0, 1/4], Taylor series of cos to th^18 in th^2
   (|err| < 4e-15), Horner in fused multiply-adds (C99 fma: correctly rounded, as v_fma_f64; spec
   v2.1), no other contraction -- the same operations as the GPU */
double oracle_cos2pi_d(double x)
{
    const double u = x - rint(x);
    const double a = u < 0.0 ? -u : u;
    const int hi = a > 0.25;
    const double b = hi ? 0.5 - a : a;
    const double th = b * 6.283185307179586;
    const double t2 = th * th;
    double r = -1.5619206968586225e-16;
    r = fma(r, t2, 4.779477332387385e-14);
    r = fma(r, t2, -1.1470745597729725e-11);
    r = fma(r, t2, 2.08767569878681e-09);
    r = fma(r, t2, -2.755731922398589e-07);
    r = fma(r, t2, 2.48015873015873e-05);
    r = fma(r, t2, -0.001388888888888889);
    r = fma(r, t2, 0.041666666666666664);
    r = fma(r, t2, -0.5);
    r = fma(r, t2, 1.0);
    return hi ? -r : r;
}

/* the chorus tap delay D cos(2 pi x) + D from the LFO's 64-bit phase (53 bits used), in double,
   clamped to [0, cmax]; integer part and fp32 fraction */
static void chorus_split(uint64_t phase, double D, double cmax, uint32_t *di, float *fr)
{
    const double x = (double)(phase >> 11) * 1.1102230246251565e-16;
    double d = fma(oracle_cos2pi_d(x), D, D);
    d = d < 0.0 ? 0.0 : (d > cmax ? cmax : d);
    *di = (uint32_t)d;
    *fr = (float)(d - (double)*di);
}

/* One frame of one instance (both channels): the per-sample operator body shared by the bank
   (oracle_chorus_process) and the config-1 loop (oracle_chorus_c1). */
static void chorus_frame(const oracle_chorus *o, const chcoef_t *k, chstate_t *s, uint32_t w,
                         const float x[2], float y[2])
{
    const uint32_t pmask = o->psize - 1, cmask = o->csize - 1;
    uint32_t cdi, di0, di1;
    float cfr, fr0, fr1;
    chorus_split(s->lfo_acc + k->lfo_off, k->D, (double)(o->csize - 2), &cdi, &cfr);
    s->lfo_acc += k->lfo_inc;
    const uint32_t ph = (uint32_t)(s->ps_acc >> 32);
    const float p0 = unit24(s->ps_acc);
    s->ps_acc += k->ps_inc;
    float g0, g1;
    oracle_win_gains(p0, &g0, &g1);
    pitch_split(ph, k->Wfix, o->psize - 2, &di0, &fr0);
    pitch_split(ph + 0x80000000u, k->Wfix, o->psize - 2, &di1, &fr1);   /* p1 = (p0 + 1/2) % 1 */
    for (int c = 0; c < 2; c++) {
        const float t0 = read_split(s->pring[c], pmask, w, di0, fr0);
        const float t1 = read_split(s->pring[c], pmask, w, di1, fr1);
        const float ps = fmaf(t1, g1, t0 * g0);                        /* spec v3 */
        s->pring[c][w & pmask] = x[c];
        if (o->mode == 0) {
            s->cring[c][w & cmask] = ps;
            const float wet = read_split(s->cring[c], cmask, w, cdi, cfr);
            const float lp = fmaf(k->b0, wet, s->z1[c]);                /* lores~, spec v3 */
            s->z1[c] = fmaf(-k->a1, lp, k->b1 * wet) + s->z2[c];
            s->z2[c] = fmaf(-k->a2, lp, k->b2 * wet);
            y[c] = fmaf(lp, k->mix, x[c] * k->dry);
        } else {
            y[c] = ps;
        }
    }
}

/* in/out [2][n_frames][n] */
int oracle_chorus_process(oracle_chorus *o, const float *in, float *out, int n_frames, int n_threads)
{
    if (!o || n_frames < 0) return -1;
    const long n = o->n;
    const long plane = n * (long)n_frames;
    const uint32_t w0 = (uint32_t)o->w;
    (void)n_threads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
#endif
    for (long i = 0; i < n; i++) {
        for (int f = 0; f < n_frames; f++) {
            const float x[2] = {in[(long)f * n + i], in[plane + (long)f * n + i]};
            float y[2];
            chorus_frame(o, &o->k[i], &o->s[i], w0 + (uint32_t)f, x, y);
            out[(long)f * n + i] = y[0];
            out[plane + (long)f * n + i] = y[1];
        }
    }
    o->w += (uint64_t)n_frames;
    return 0;
}

/* BASELINE configs[0] / SURVEY 8d C1: ONE chorus instance on one core, in the shape of the
   reference's fx_test.cpp:45-54 loop -- per block of `block` frames, per frame: next input
   sample (xorshift32 noise of instance 0, SURVEY 8d seeds), process(), isnan check -- over
   n_frames frames.  Returns the number of NaN outputs; *sum_abs = sum |y| (keeps the work live). */
long oracle_chorus_c1(float sample_rate, const float *params, long n_frames, int block, double *sum_abs)
{
    oracle_chorus *o = oracle_chorus_create(1, sample_rate, 0);
    if (!o || block <= 0) { oracle_chorus_destroy(o); return -1; }
    for (int f = 0; f < OCH_NPARAMS; f++) oracle_chorus_set(o, 0, f, params[f]);
    uint32_t s[2] = {(0x9E3779B9u ^ (1u * 0x85EBCA6Bu)) | 1u, (0x9E3779B9u ^ (2u * 0x85EBCA6Bu)) | 1u};
    long nans = 0;
    double acc = 0.0;
    for (long f0 = 0; f0 < n_frames; f0 += block) {
        const long C = n_frames - f0 < block ? n_frames - f0 : block;
        for (long f = 0; f < C; f++) {
            float x[2], y[2];
            for (int c = 0; c < 2; c++) {
                s[c] ^= s[c] << 13; s[c] ^= s[c] >> 17; s[c] ^= s[c] << 5;
                x[c] = (float)(int32_t)s[c] / 2147483648.0f * 0.5f;
            }
            chorus_frame(o, &o->k[0], &o->s[0], (uint32_t)o->w, x, y);
            o->w++;
            nans += isnan(y[0]) + isnan(y[1]);
            acc += fabs((double)y[0]) + fabs((double)y[1]);
        }
    }
    oracle_chorus_destroy(o);
    if (sum_abs) *sum_abs = acc;
    return nans;
}
