/*
 * oracle/chorus_ref_f64.c -- the RNBO stereo chorus / gen~ pitch-shifter restated in DOUBLE
 * precision, as gen~ and RNBO compute (TEST INFRASTRUCTURE ONLY: tests/ and nothing else).
 *
 * Purpose: the build's spec (oracle/chorus_ref.c) declares fp32 arithmetic
 * and fixed-point phasors where gen~/RNBO use double.  This restatement removes exactly those two
 * choices and keeps every other one, so tests/test_oracle.py can MEASURE the fp32 spec's
 * deviation from double-precision arithmetic on the same inputs instead of asserting it.
 * Parity stays UNPINNED: RNBO/genlib are absent, and the other spec choices (cycle~ as an exact
 * cosine instead of RNBODefaultSinus, lores~ as an RBJ biquad) are shared by both restatements.
 *
 * Graph (same citations as chorus_ref.c): mono-chorus.rnbopat
 *   y = (1-mix) x + mix * lores~( delay~( pitchshift(x, pitch), D cycle~(rate_hz, phase) + D ) )
 * pitchshift gencode (mono-chorus.rnbopat:962, pitchshift.gendsp:19-305), in double:
 *   ph = phasor(shift): output, then ph += shift / sr, wrapped to [0, 1);  p0 = ph, p1 = (ph + .5) % 1
 *   out = read(p1 W) cos((p1 - .5) pi) + read(p0 W) cos((p0 - .5) pi);  write(x) after the reads
 *   (gen Delay.read: linear, delay clamped to >= 1; delay~: write before read, linear, >= 0)
 * cycle~(rate_hz, phase): cos(2 pi (ph_lfo + phase)), ph_lfo a double phasor.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include "oracle.h"

static uint32_t pow2ge64(uint32_t x) { uint32_t p = 1; while (p < x) p <<= 1; return p; }
static double clampd(double x, double lo, double hi) { return x < lo ? lo : (x > hi ? hi : x); }

typedef struct {
    double lfo_ph, ps_ph, z1[2], z2[2];
    double lfo_inc, lfo_off, ps_inc, D, W, b0, b1, b2, a1, a2, mix;
    double *pring[2], *cring[2];
} ch64_t;

struct oracle_chorus64 {
    int n, mode, quantize, f32;
    double sr;
    uint32_t psize, csize;
    uint64_t w;
    double *pool;
    ch64_t *v;
    double *params;            /* [n][OCH_NPARAMS] */
};

/* quantize = 1: phasor increments rounded to the fp32 spec's 64-bit fixed point (chorus_ref.c
   fix64), so the remaining deviation is the fp32 arithmetic alone */
static double q64(double inc) { return floor(inc * 18446744073709551616.0 + 0.5) / 18446744073709551616.0; }

static void derive64(const double *p, double sr, int quantize, ch64_t *c)
{
    const double pitch = clampd(p[OCH_PITCH], 0.0, 3.0);
    const double q = clampd(p[OCH_Q], 0.0, 1.0);
    const double cutoff = clampd(p[OCH_CUTOFF], 0.0, 1.0);
    const double depth = clampd(p[OCH_DEPTH], 0.08, 1.0);
    const double rate = clampd(p[OCH_RATE], 0.01, 1.0);
    const double window = clampd(p[OCH_WINDOW], 4.0, 10.0);
    c->mix = clampd(p[OCH_MIX], 0.0, 1.0);
    c->lfo_off = clampd(p[OCH_PHASE], 0.0, 1.0);
    c->lfo_inc = (0.01 + rate * (0.5 - 0.01)) / sr;          /* scale 0 1 0.01 0.5, :3935 */
    c->ps_inc = pitch / sr;
    if (quantize) { c->lfo_inc = q64(c->lfo_inc); c->ps_inc = q64(c->ps_inc); }
    c->D = (1.0 + depth * (12.0 - 1.0)) * sr / 1000.0;       /* mstosamps(scale 0 1 1 12), :3436 */
    c->W = window * sr / 1000.0;
    const double fc = 300.0 + cutoff * (15000.0 - 300.0);    /* :2242 */
    const double Q = 0.70710678118654752 + 20.0 * q * q * q;
    const double w0 = 2.0 * 3.14159265358979323846 * fc / sr;
    const double cw = cos(w0), sw = sin(w0);
    const double alpha = sw / (2.0 * Q), a0 = 1.0 + alpha;
    c->b0 = (1.0 - cw) * 0.5 / a0;
    c->b1 = (1.0 - cw) / a0;
    c->b2 = (1.0 - cw) * 0.5 / a0;
    c->a1 = -2.0 * cw / a0;
    c->a2 = (1.0 - alpha) / a0;
}

oracle_chorus64 *oracle_chorus64_create(int n_inst, double sample_rate, int mode)
{
    if (n_inst <= 0 || (mode & ~0x7FF)) return NULL;
    oracle_chorus64 *o = (oracle_chorus64 *)calloc(1, sizeof(*o));
    if (!o) return NULL;
    o->n = n_inst; o->mode = mode & 1; o->quantize = (mode >> 1) & 1; o->f32 = mode >> 2; o->sr = sample_rate;
    o->psize = pow2ge64((uint32_t)ceil(10.0 * sample_rate / 1000.0) + 2);
    o->csize = pow2ge64(2u * (uint32_t)ceil(12.0 * sample_rate / 1000.0) + 2);
    const size_t per = 2u * (o->psize + o->csize);
    o->pool = (double *)calloc(per * (size_t)n_inst, sizeof(double));
    o->v = (ch64_t *)calloc((size_t)n_inst, sizeof(ch64_t));
    o->params = (double *)calloc((size_t)n_inst * OCH_NPARAMS, sizeof(double));
    if (!o->pool || !o->v || !o->params) { oracle_chorus64_destroy(o); return NULL; }
    for (int i = 0; i < n_inst; i++) {
        double *base = o->pool + per * (size_t)i, *p = o->params + (size_t)i * OCH_NPARAMS;
        o->v[i].pring[0] = base;
        o->v[i].pring[1] = base + o->psize;
        o->v[i].cring[0] = base + 2 * o->psize;
        o->v[i].cring[1] = base + 2 * o->psize + o->csize;
        p[OCH_PITCH] = 0.0; p[OCH_MIX] = 0.5; p[OCH_Q] = 0.5; p[OCH_CUTOFF] = 0.3;   /* RNBO defaults */
        p[OCH_PHASE] = 1.0; p[OCH_DEPTH] = 0.5; p[OCH_RATE] = 0.2; p[OCH_WINDOW] = 10.0;
        derive64(p, o->sr, o->quantize, &o->v[i]);
    }
    return o;
}

void oracle_chorus64_destroy(oracle_chorus64 *o)
{
    if (!o) return;
    free(o->pool); free(o->v); free(o->params); free(o);
}

int oracle_chorus64_set(oracle_chorus64 *o, int inst, int field, double value)
{
    if (!o || inst < 0 || inst >= o->n || field < 0 || field >= OCH_NPARAMS) return -1;
    o->params[(size_t)inst * OCH_NPARAMS + field] = value;
    derive64(o->params + (size_t)inst * OCH_NPARAMS, o->sr, o->quantize, &o->v[inst]);
    return 0;
}

static double wrap1(double x) { return x - floor(x); }

/* Stage-by-stage decomposition of the fp32 spec's deviation (tests/test_oracle.py
   test_chorus_deviation_by_stage): mode bits 2.. select stages computed as the fp32 spec computes
   them (chorus_ref.c chorus_frame), everything else in double:
     F32_PDELAY   pitch tap delays: 24-bit phase (unit24), d = p W in fp32, fp32 split
     F32_PGAIN    crossfade gains: the fp32 sin / cos polynomials (oracle_win_gains)
     F32_PINTERP  pitch taps' interpolation and the crossfade sum in fp32
     F32_CDELAY   chorus delay: cos2pi polynomial of the 24-bit phase, lfo D + D in fp32
     F32_CINTERP  chorus tap interpolation in fp32
     F32_LORES    lores~ coefficients and state in fp32
     F32_MIX      x dry + lp mix in fp32 */
enum { F32_PDELAY = 1, F32_PGAIN = 2, F32_PINTERP = 4, F32_CDELAY = 8, F32_CINTERP = 16, F32_LORES = 32, F32_MIX = 64,
       /* candidate precise delays: the pitch delay in 32.32 fixed point (the phasor's top 32 bits x W
          in 32.32), the chorus delay from a 53-bit phase in double; both split into an integer and
          an fp32 fraction */
       FIX_PDELAY = 128, DBL_CDELAY = 256 };

/* split of a non-negative delay given as an integer and a fraction in [0, 1) */
static double readsplit(const double *ring, uint32_t mask, uint64_t w, uint32_t di, float fr, int f32i)
{
    const double x0 = ring[(w - di) & mask], x1 = ring[(w - di - 1u) & mask];
    if (!f32i) return x0 + (double)fr * (x1 - x0);
    const float x0f = (float)x0, x1f = (float)x1;
    return (double)(x0f + fr * (x1f - x0f));
}
/* 32.32 fixed-point pitch delay of phase p (cycles) and window W (samples), clamped to [1, pmax] */
static void pdelay_fix(double p, double W, double pmax, uint32_t *di, float *fr)
{
    const uint64_t ph = (uint64_t)floor(p * 4294967296.0);
    const unsigned __int128 wf = (unsigned __int128)(uint64_t)floor(W * 4294967296.0 + 0.5);
    uint64_t d = (uint64_t)(((unsigned __int128)ph * wf) >> 32);
    const uint64_t lo = 1ull << 32, hi = (uint64_t)pmax << 32;
    d = d < lo ? lo : (d > hi ? hi : d);
    *di = (uint32_t)(d >> 32);
    *fr = (float)(uint32_t)d * 2.3283064365386963e-10f;
}


static double unit24d(double ph) { return floor(ph * 16777216.0) / 16777216.0; }

static double readf(const double *ring, uint32_t mask, uint64_t w, double d, double dmin, int f32d, int f32i)
{
    if (!f32d) {
        d = d < dmin ? dmin : d;
        const uint64_t di = (uint64_t)d;
        const double fr = d - (double)di;
        const double x0 = ring[(w - di) & mask], x1 = ring[(w - di - 1u) & mask];
        if (!f32i) return x0 + fr * (x1 - x0);
        const float x0f = (float)x0, x1f = (float)x1, frf = (float)fr;
        return (double)(x0f + frf * (x1f - x0f));
    }
    float df = (float)d;
    df = df < (float)dmin ? (float)dmin : df;
    const uint32_t di = (uint32_t)df;
    const float fr = df - (float)di;
    const double x0 = ring[(w - di) & mask], x1 = ring[(w - di - 1u) & mask];
    if (!f32i) return x0 + (double)fr * (x1 - x0);
    const float x0f = (float)x0, x1f = (float)x1;
    return (double)(x0f + fr * (x1f - x0f));
}

/* in: float [2][n_frames][n] (the same inputs as the fp32 oracle); out: double [2][n_frames][n] */
int oracle_chorus64_process(oracle_chorus64 *o, const float *in, double *out, int n_frames)
{
    if (!o || n_frames < 0) return -1;
    const long n = o->n, plane = n * (long)n_frames;
    const uint32_t pmask = o->psize - 1, cmask = o->csize - 1;
    const double pi = 3.14159265358979323846;
    for (long i = 0; i < n; i++) {
        ch64_t *s = &o->v[i];
        for (int f = 0; f < n_frames; f++) {
            const uint64_t w = o->w + (uint64_t)f;
            const int F = o->f32;
            const double lph = wrap1(s->lfo_ph + s->lfo_off);
            double dch;
            uint32_t cdi = 0;
            float cfr = 0.f;
            if (F & DBL_CDELAY) {
                const double ph53 = floor(lph * 9007199254740992.0) / 9007199254740992.0;
                double dd = cos(2.0 * pi * ph53) * s->D + s->D;
                const double cmaxd = (double)(o->csize - 2);
                dd = dd < 0.0 ? 0.0 : (dd > cmaxd ? cmaxd : dd);
                cdi = (uint32_t)dd;
                cfr = (float)(dd - (double)cdi);
                dch = dd;
            } else if (F & F32_CDELAY) {
                const float lfo = oracle_cos2pi((float)unit24d(lph));
                dch = (double)(lfo * (float)s->D + (float)s->D);
            } else {
                dch = cos(2.0 * pi * lph) * s->D + s->D;
            }
            s->lfo_ph = wrap1(s->lfo_ph + s->lfo_inc);
            const double p0 = s->ps_ph, p1 = wrap1(s->ps_ph + 0.5);
            s->ps_ph = wrap1(s->ps_ph + s->ps_inc);
            double g0 = cos((p0 - 0.5) * pi), g1 = cos((p1 - 0.5) * pi);
            if (F & F32_PGAIN) {
                float a, b;
                oracle_win_gains((float)unit24d(p0), &a, &b);
                g0 = a; g1 = b;
            }
            double d0 = p0 * s->W, d1 = p1 * s->W;
            if (F & F32_PDELAY) {
                d0 = (double)((float)unit24d(p0) * (float)s->W);
                d1 = (double)((float)unit24d(p1) * (float)s->W);
            }
            for (int c = 0; c < 2; c++) {
                const double x = in[c * plane + (long)f * n + i];
                double t1, t0;
                if (F & FIX_PDELAY) {
                    uint32_t di; float fr;
                    const double pmaxd = (double)(o->psize - 2);
                    pdelay_fix(p1, s->W, pmaxd, &di, &fr);
                    t1 = readsplit(s->pring[c], pmask, w, di, fr, F & F32_PINTERP);
                    pdelay_fix(p0, s->W, pmaxd, &di, &fr);
                    t0 = readsplit(s->pring[c], pmask, w, di, fr, F & F32_PINTERP);
                } else {
                    t1 = readf(s->pring[c], pmask, w, d1, 1.0, F & F32_PDELAY, F & F32_PINTERP);
                    t0 = readf(s->pring[c], pmask, w, d0, 1.0, F & F32_PDELAY, F & F32_PINTERP);
                }
                const double ps = (F & F32_PINTERP) ? (double)((float)t1 * (float)g1 + (float)t0 * (float)g0)
                                                    : t1 * g1 + t0 * g0;
                s->pring[c][w & pmask] = x;
                double y = ps;
                if (o->mode == 0) {
                    s->cring[c][w & cmask] = ps;
                    const double wet = (F & DBL_CDELAY) ? readsplit(s->cring[c], cmask, w, cdi, cfr, F & F32_CINTERP)
                                                        : readf(s->cring[c], cmask, w, dch, 0.0, F & F32_CDELAY, F & F32_CINTERP);
                    double lp;
                    if (F & F32_LORES) {
                        const float wf = (float)wet, lpf = (float)s->b0 * wf + (float)s->z1[c];
                        s->z1[c] = (double)(((float)s->b1 * wf - (float)s->a1 * lpf) + (float)s->z2[c]);
                        s->z2[c] = (double)((float)s->b2 * wf - (float)s->a2 * lpf);
                        lp = lpf;
                    } else {
                        lp = s->b0 * wet + s->z1[c];
                        s->z1[c] = (s->b1 * wet - s->a1 * lp) + s->z2[c];
                        s->z2[c] = s->b2 * wet - s->a2 * lp;
                    }
                    y = (F & F32_MIX) ? (double)((float)x * (1.0f - (float)s->mix) + (float)lp * (float)s->mix)
                                      : x * (1.0 - s->mix) + lp * s->mix;
                }
                out[c * plane + (long)f * n + i] = y;
            }
        }
    }
    o->w += (uint64_t)n_frames;
    return 0;
}
