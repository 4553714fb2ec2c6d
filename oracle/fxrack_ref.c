/*
 * oracle/fxrack_ref.c -- CPU oracle for the fxlib effect rack, ol::fx::FxRack<2>
 * (modules/fxlib/Fx.h:398-492): DelayFx<2> -> ReverbFx<2> -> FilterFx<2> -> x master volume.
 *
 * TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).  Never part of the product.
 *
 * The rack composition is in-tree and restated literally:
 *   FxRack::Process        Fx.h:432-440  delay -> reverb -> filter1 -> buf_c[i] * master_volume
 *   DelayFx::Process       Fx.h:193-206  per channel: buf = Read(); Write(in + feedback * buf);
 *                                        filter_ (a FilterFx, channel 0 only) in place;
 *                                        out = buf * balance + in * (1 - balance)
 *   DelayFx::Init/Update   Fx.h:183-217  filter_ cutoff = scale(64, 0,127, 0,20000, 1),
 *                                        resonance = scale(24, 0,127, 0,1, 1);
 *                                        SetDelay(scale(time, 0,1, 0,MAX_DELAY=48000, 1))
 *   ReverbFx::Process      Fx.h:293-299  out = verb * balance + in * (1 - balance)
 *   DaisyVerb -> the in-tree daisysp::ReverbSc stub (Reverb.h:12-40): out = in * 0.8f
 *   FilterFx::Process      Fx.h:88-108   SvfFilter processes frame[0] only (Filter.h:85-91)
 *   ol::core::scale        corelib/ol_corelib.h:31-44
 * Reference behaviour kept as is: FilterFx writes only channel 0 of its output, and FxRack's
 * buf_c is zero-initialised (Fx.h:408), so the rack's channel 1 output is always 0.
 *
 * Parity status: UNPINNED for the DaisySP primitives (DelayLine, Svf).  They are third-party
 * (DaisySP, pinned only as "commit": "master", submodules.json:74-80) and absent here; their
 * published algorithm is restated (DelayLine: write pointer decrements, Read = linear
 * interpolation between delay and delay + 1; Svf: double-sampled Chamberlin, as in voice_ref.c).
 * The reference's own test at this boundary (test/fx_test.cpp:25-55: DelayFx fed a 20 kHz sine
 * for one second never outputs NaN) is reproduced by tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define MAX_DELAY 48000
#define MINF(a, b) ((a) < (b) ? (a) : (b))

static float fclampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

/* ol::core::scale (ol_corelib.h:27-44), t_sample = float */
static float core_scale(float in, float inlow, float inhigh, float outlow, float outhigh, float power)
{
    const float denom = inhigh - inlow;
    const float inscale = denom == 0.f ? 0.f : (float)(1.f / denom);
    const float outdiff = outhigh - outlow;
    float value = (in - inlow) * inscale;
    if (value > 0.0f) value = powf(value, power);
    else if (value < 0.0f) value = -powf(-value, power);
    return (value * outdiff) + outlow;
}

/* daisysp::Svf */
typedef struct {
    float sr, fc_max, freq, damp, res, pre_drive, drive;
    float low, band;
} svf_t;

static void svf_init(svf_t *s, float sr)
{
    memset(s, 0, sizeof(*s));
    s->sr = sr; s->fc_max = sr / 3.f;
    s->res = 0.5f; s->drive = 0.5f; s->pre_drive = 0.5f; s->freq = 0.25f; s->damp = 0.f;
}
static float svf_damp(const svf_t *s)
{
    return MINF(2.0f * (1.0f - powf(s->res, 0.25f)), MINF(2.0f, 2.0f / s->freq - s->freq * 0.5f));
}
static void svf_set_freq(svf_t *s, float f)
{
    const float fc = fclampf(f, 1.0e-6f, s->fc_max);
    s->freq = 2.0f * sinf(3.1415927410125732f * MINF(0.25f, fc / (s->sr * 2.0f)));
    s->damp = svf_damp(s);
}
static void svf_set_res(svf_t *s, float r)
{
    s->res = fclampf(r, 0.f, 1.f);
    s->damp = svf_damp(s);
    s->drive = s->pre_drive * s->res;
}
static void svf_set_drive(svf_t *s, float d)
{
    s->pre_drive = fclampf(d * 0.1f, 0.f, 1.f);
    s->drive = s->pre_drive * s->res;
}
/* Svf::Process, then the output selected by FilterFx's type (Fx.h:90-106):
   0 low, 1 band, 2 high, 3 notch, 4 peak */
static float svf_process(svf_t *s, float in, int type)
{
    float notch = in - s->damp * s->band;
    s->low = s->low + s->freq * s->band;
    float high = notch - s->low;
    s->band = s->freq * high + s->band - s->drive * s->band * s->band * s->band;
    float o_low = 0.5f * s->low, o_high = 0.5f * high, o_band = 0.5f * s->band;
    float o_peak = 0.5f * (s->low - high), o_notch = 0.5f * notch;
    notch = in - s->damp * s->band;
    s->low = s->low + s->freq * s->band;
    high = notch - s->low;
    s->band = s->freq * high + s->band - s->drive * s->band * s->band * s->band;
    o_low += 0.5f * s->low;
    o_high += 0.5f * high;
    o_band += 0.5f * s->band;
    o_peak += 0.5f * (s->low - high);
    o_notch += 0.5f * notch;
    switch (type) {
    case 1: return o_band;
    case 2: return o_high;
    case 3: return o_notch;
    case 4: return o_peak;
    default: return o_low;
    }
}

/* daisysp::DelayLine<float, 48000> */
typedef struct {
    float line[MAX_DELAY];
    uint32_t write_ptr, delay;
    float frac;
} delay_t;

static void delay_reset(delay_t *d) { memset(d->line, 0, sizeof(d->line)); d->write_ptr = 0; d->delay = 1; d->frac = 0.f; }
static void delay_set(delay_t *d, float delay)
{
    const int32_t id = (int32_t)delay;
    d->frac = delay - (float)id;
    d->delay = (uint32_t)id < MAX_DELAY ? (uint32_t)id : MAX_DELAY - 1;
}
static float delay_read(const delay_t *d)
{
    const float a = d->line[(d->write_ptr + d->delay) % MAX_DELAY];
    const float b = d->line[(d->write_ptr + d->delay + 1) % MAX_DELAY];
    return a + (b - a) * d->frac;
}
static void delay_write(delay_t *d, float x)
{
    d->line[d->write_ptr] = x;
    d->write_ptr = (d->write_ptr - 1 + MAX_DELAY) % MAX_DELAY;
}

typedef struct {
    delay_t dl[2];
    svf_t dfilt, filt;          /* DelayFx::filter_ and FxRack::filter1 (channel 0 only) */
    float p[OFR_NPARAMS];
} rack_t;

struct oracle_fxrack {
    int n;
    float sr;
    rack_t *r;
};

/* FilterFx::Update (Fx.h:110-114): SetFreq, SetRes, SetDrive in that order */
static void filterfx_update(svf_t *s, float cutoff, float res, float drive)
{
    svf_set_freq(s, cutoff);
    svf_set_res(s, res);
    svf_set_drive(s, drive);
}

static void rack_update(rack_t *r)
{
    /* DelayFx::Update: SetDelay(scale(time, 0, 1, 0, MAX_DELAY, 1)) on both lines, filter_.Update() */
    const float dly = core_scale(r->p[OFR_DELAY_TIME], 0.f, 1.f, 0.f, (float)MAX_DELAY, 1.f);
    delay_set(&r->dl[0], dly);
    delay_set(&r->dl[1], dly);
    filterfx_update(&r->dfilt, r->p[OFR_DELAY_CUTOFF], r->p[OFR_DELAY_RESONANCE], 0.f);
    /* ReverbFx::Update: SetTime/SetCutoff reach only the ReverbSc stub's unused members */
    filterfx_update(&r->filt, r->p[OFR_FILTER_CUTOFF], r->p[OFR_FILTER_RESONANCE], r->p[OFR_FILTER_DRIVE]);
}

void oracle_fxrack_defaults(float *p)
{
    p[OFR_DELAY_TIME] = 0.5f;                                           /* Fx.h:172 */
    p[OFR_DELAY_FEEDBACK] = 0.5f;                                       /* Fx.h:173 */
    p[OFR_DELAY_BALANCE] = 0.33f;                                       /* Fx.h:174 */
    p[OFR_DELAY_CUTOFF] = core_scale(64.f, 0.f, 127.f, 0.f, 20000.f, 1.f);   /* Fx.h:188, :120 */
    p[OFR_DELAY_RESONANCE] = core_scale(24.f, 0.f, 127.f, 0.f, 1.f, 1.f);     /* Fx.h:189, :117 */
    p[OFR_REVERB_BALANCE] = 0.1f;                                       /* Fx.h:282 */
    p[OFR_FILTER_CUTOFF] = 20000.f;                                     /* Fx.h:75 */
    p[OFR_FILTER_RESONANCE] = 0.f;
    p[OFR_FILTER_DRIVE] = 0.f;
    p[OFR_FILTER_TYPE] = 0.f;                                           /* LowPass */
    p[OFR_MASTER_VOLUME] = 0.8f;                                        /* Fx.h:405 */
    p[OFR_TOPOLOGY] = 0.f;                                              /* FxRack<2>::Process */
}

static void rack_init(rack_t *r, float sr)
{
    memset(r, 0, sizeof(*r));
    delay_reset(&r->dl[0]);
    delay_reset(&r->dl[1]);
    svf_init(&r->dfilt, sr);
    svf_init(&r->filt, sr);
    oracle_fxrack_defaults(r->p);
    rack_update(r);
}

static void rack_tick(rack_t *r, const float in[2], float out[2])
{
    const float *p = r->p;
    float buf[2];
    /* DelayFx::Process */
    for (int i = 0; i < 2; ++i) {
        buf[i] = delay_read(&r->dl[i]);
        delay_write(&r->dl[i], in[i] + (p[OFR_DELAY_FEEDBACK] * buf[i]));
    }
    buf[0] = svf_process(&r->dfilt, buf[0], 0);        /* FilterFx (LowPass), channel 0 in place */
    float a[2], b[2];
    for (int i = 0; i < 2; ++i) a[i] = (buf[i] * p[OFR_DELAY_BALANCE]) + (in[i] * (1 - p[OFR_DELAY_BALANCE]));
    /* the components alone, each as the firmware's objects run it (main.cpp:82-85):
       2 DelayFx<2>::Process (Fx.h:193-206): the rack's delay stage, both channels out */
    if (p[OFR_TOPOLOGY] == 2.f) {
        out[0] = a[0];
        out[1] = a[1];
        return;
    }
    /* 3 ReverbFx<2>::Process over DaisyVerb<2> and the ReverbSc stub (Fx.h:293-299, Reverb.h:26-31,
       :82-91): per channel 0.8 in balance + in (1 - balance); the delay line runs unobserved */
    if (p[OFR_TOPOLOGY] == 3.f) {
        for (int i = 0; i < 2; ++i) {
            const float v = in[i] * 0.8f;
            out[i] = (v * p[OFR_REVERB_BALANCE]) + (in[i] * (1 - p[OFR_REVERB_BALANCE]));
        }
        return;
    }
    /* 4 FilterFx<2>::Process (Fx.h:88-108): the Svf on channel 0 with the selected output; channel 1
       of frame_out is not written (Filter.h:85-91): in place -- the firmware's use -- it keeps
       channel 1 of the input */
    if (p[OFR_TOPOLOGY] == 4.f) {
        out[0] = svf_process(&r->filt, in[0], (int)p[OFR_FILTER_TYPE]);
        out[1] = in[1];
        return;
    }
    if (p[OFR_TOPOLOGY] == 1.f) {
        /* ol_daisy/app/synth/main.cpp:78-86: delay_fx (DelayFx<1>: line 0 and its filter, the same
           arithmetic as the rack's channel 0) on mono; stereo[0] = stereo[1] = mono;
           reverb_fx.Process(stereo, stereo); filter_fx.Process(stereo, stereo) writes channel 0
           only, so channel 1 keeps the reverb's output; no master volume */
        const float m = a[0];
        const float v = m * 0.8f;
        const float rv = (v * p[OFR_REVERB_BALANCE]) + (m * (1 - p[OFR_REVERB_BALANCE]));
        out[0] = svf_process(&r->filt, rv, (int)p[OFR_FILTER_TYPE]);
        out[1] = rv;
        return;
    }
    /* ReverbFx::Process over the ReverbSc stub */
    for (int i = 0; i < 2; ++i) {
        const float v = a[i] * 0.8f;
        b[i] = (v * p[OFR_REVERB_BALANCE]) + (a[i] * (1 - p[OFR_REVERB_BALANCE]));
    }
    /* FilterFx::Process: channel 0 only; buf_c[1] stays 0 */
    const float c0 = svf_process(&r->filt, b[0], (int)p[OFR_FILTER_TYPE]);
    out[0] = c0 * p[OFR_MASTER_VOLUME];
    out[1] = 0.0f * p[OFR_MASTER_VOLUME];
}

oracle_fxrack *oracle_fxrack_create(int n_inst, float sample_rate)
{
    if (n_inst <= 0) return NULL;
    oracle_fxrack *o = (oracle_fxrack *)calloc(1, sizeof(*o));
    if (!o) return NULL;
    o->n = n_inst;
    o->sr = sample_rate;
    o->r = (rack_t *)malloc((size_t)n_inst * sizeof(rack_t));
    if (!o->r) { free(o); return NULL; }
    for (int i = 0; i < n_inst; ++i) rack_init(&o->r[i], sample_rate);
    return o;
}

void oracle_fxrack_destroy(oracle_fxrack *o)
{
    if (!o) return;
    free(o->r);
    free(o);
}

int oracle_fxrack_set(oracle_fxrack *o, int inst, int field, float value)
{
    if (!o || inst < 0 || inst >= o->n || field < 0 || field >= OFR_NPARAMS) return -1;
    o->r[inst].p[field] = value;
    rack_update(&o->r[inst]);
    return 0;
}

int oracle_fxrack_process(oracle_fxrack *o, const float *in, float *out, int n_frames, int n_threads)
{
    if (!o || !in || !out || n_frames < 0) return -1;
    const long n = o->n;
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
    for (long i = 0; i < n; ++i) {
        for (int f = 0; f < n_frames; ++f) {
            const float x[2] = {in[(long)f * n + i], in[((long)n_frames + f) * n + i]};
            float y[2];
            rack_tick(&o->r[i], x, y);
            out[(long)f * n + i] = y[0];
            out[((long)n_frames + f) * n + i] = y[1];
        }
    }
    return 0;
}
