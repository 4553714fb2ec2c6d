/*
 * oracle/dattorro_ref.c -- CPU restatement of the reference Dattorro plate reverb.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (ol_dsp_amd/, libolfx.so) links,
 * loads or calls this file.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, and only as the checker / CPU baseline.
 *
 * Parity status: PINNED.  This restatement is checked bit-for-bit against
 *   (1) the reference itself, compiled from /root/reference/libs/dattorro-verb/verb.cpp
 *       by oracle/Makefile into oracle/_ref/ (in the dev container only), and
 *   (2) the committed golden vectors in tests/golden/ (impulse KATs + the 10 s
 *       xorshift-noise FNV-1a-64 hash 725e69018b5e52f2 recorded in SURVEY.md section 8c).
 *
 * Algorithm followed (file:line into the reference, /root/reference/libs/dattorro-verb/):
 *   ring geometry      verb.cpp:65-98   (size = 2^bits(delay), mask, read offset = size - delay)
 *   tap offsets        verb.cpp:173-212 (13 lines, 11 extra output taps)
 *   default params     verb.cpp:214-221
 *   setters            verb.cpp:137-170 (preDelay float->uint16 truncation; decay -> dd2 clamp)
 *   per-sample process verb.cpp:258-299 (t&0x7ff modulation of the tank APF taps, predelay,
 *                                        1-pole LPF, 4 input APFs, 2 cross-coupled tank halves)
 *   stereo taps        verb.cpp:302-325 (7 signed taps each, read at the post-increment t)
 *   fxlib glue         modules/fxlib/ReverbFx.cpp:11-27 (stereo in -> (l+r)/2 -> L/R out)
 *
 * Build: -O2 -ffp-contract=off (no FMA contraction, denormals kept), see oracle/Makefile.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

/* Line identifiers, in the order the reference allocates them (verb.cpp:177-212). */
enum {
    L_PRE = 0,
    L_IN0, L_IN1, L_IN2, L_IN3,
    L_AP1A, L_DL1A, L_AP2A, L_DL2A,   /* tank half 0 */
    L_AP1B, L_DL1B, L_AP2B, L_DL2B,   /* tank half 1 */
    L_COUNT
};

/* nominal delay of each line (its TAP_MAIN), verb.cpp:177-210 */
static const uint16_t k_nominal[L_COUNT] = {
    4800, 142, 107, 379, 277, 672, 4453, 1800, 3720, 908, 4217, 2656, 3163
};

/* extra output taps: {line, tap index 1..3, delay}, verb.cpp:187-212 */
static const struct { int line, tap; uint16_t delay; } k_extra[] = {
    {L_DL1A, 1, 353}, {L_DL1A, 2, 3627}, {L_DL1A, 3, 1990},
    {L_AP2A, 1, 187}, {L_AP2A, 2, 1228},
    {L_DL2A, 1, 1066}, {L_DL2A, 2, 2673},
    {L_DL1B, 1, 266}, {L_DL1B, 2, 2974}, {L_DL1B, 3, 2111},
    {L_AP2B, 1, 335}, {L_AP2B, 2, 1913},
    {L_DL2B, 1, 121}, {L_DL2B, 2, 1996},
};

typedef struct {
    float   *mem;
    uint16_t mask;
    uint16_t off[4];     /* read offsets, uint16 exactly like the reference */
} ring_t;

typedef struct {
    ring_t   ring[L_COUNT];
    float    lp_pre, lp_damp[2];
    float    a_prefilter, a_in1, a_in2, a_dd1, a_damping, a_decay, a_dd2;
    uint16_t t;
} verb_t;

struct oracle_dattorro {
    int      n;
    float   *pool;       /* all ring memory of all instances */
    verb_t  *v;
};

static uint16_t pow2_above(uint16_t d)
{
    uint16_t bits = 0;
    while (d) { bits++; d >>= 1; }
    return (uint16_t)(1u << bits);
}

size_t oracle_dattorro_state_floats(void)
{
    size_t s = 0;
    for (int l = 0; l < L_COUNT; l++) s += pow2_above(k_nominal[l]);
    return s;
}

static void set_tap(ring_t *r, int tap, uint16_t delay)
{
    r->off[tap] = (uint16_t)(r->mask + 1 - delay);
}

static void verb_set(verb_t *v, int field, float value)
{
    switch (field) {
    case ODT_PREDELAY: {
        /* verb.cpp:137-139: the product value*4800.f is converted to uint16 (truncation) */
        float d = value * 4800.0f;
        set_tap(&v->ring[L_PRE], 0, d <= 0.0f ? 0 : (uint16_t)d);
        break;
    }
    case ODT_PREFILTER:          v->a_prefilter = value; break;
    case ODT_INPUT_DIFFUSION1:   v->a_in1 = value; break;
    case ODT_INPUT_DIFFUSION2:   v->a_in2 = value; break;
    case ODT_DECAY_DIFFUSION:    v->a_dd1 = value; break;
    case ODT_DECAY: {
        /* verb.cpp:49,162-165: value+0.15 is double, narrowed to float by clamp()'s
           t_sample parameter, then clamped to [0.25, 0.5] */
        float x = (float)((double)value + 0.15);
        v->a_decay = value;
        v->a_dd2 = x < 0.25f ? 0.25f : (x > 0.5f ? 0.5f : x);
        break;
    }
    case ODT_DAMPING:            v->a_damping = value; break;
    default: break;
    }
}

static void verb_init(verb_t *v, float *mem)
{
    memset(v, 0, sizeof(*v));
    for (int l = 0; l < L_COUNT; l++) {
        uint16_t size = pow2_above(k_nominal[l]);
        v->ring[l].mem = mem;
        v->ring[l].mask = (uint16_t)(size - 1);
        set_tap(&v->ring[l], 0, k_nominal[l]);
        memset(mem, 0, size * sizeof(float));
        mem += size;
    }
    for (size_t i = 0; i < sizeof(k_extra) / sizeof(k_extra[0]); i++)
        set_tap(&v->ring[k_extra[i].line], k_extra[i].tap, k_extra[i].delay);
    /* defaults, verb.cpp:215-221 (preDelay 0.1 is a double literal narrowed to float) */
    verb_set(v, ODT_PREDELAY, (float)0.1);
    verb_set(v, ODT_PREFILTER, (float)0.85);
    verb_set(v, ODT_INPUT_DIFFUSION1, (float)0.75);
    verb_set(v, ODT_INPUT_DIFFUSION2, (float)0.625);
    verb_set(v, ODT_DECAY, (float)0.75);
    verb_set(v, ODT_DECAY_DIFFUSION, (float)0.70);
    verb_set(v, ODT_DAMPING, (float)0.95);
}

static inline float rd(const ring_t *r, int tap, uint16_t t)
{
    return r->mem[(t + r->off[tap]) & r->mask];
}

static inline void wr(ring_t *r, uint16_t t, float x)
{
    r->mem[t & r->mask] = x;
}

/* all-pass section: verb.cpp:123-128 */
static inline float allpass(ring_t *r, uint16_t t, float g, float x)
{
    float d = rd(r, 0, t);
    x += d * -g;
    wr(r, t, x);
    return d + x * g;
}

static void verb_tick(verb_t *v, float in, float *outl, float *outr)
{
    ring_t *R = v->ring;
    const uint16_t t = v->t;

    /* tank-APF tap modulation, verb.cpp:262-270 */
    if ((t & 0x07ff) == 0) {
        if (t < (1 << 15)) { R[L_AP1A].off[0]--; R[L_AP1B].off[0]--; }
        else               { R[L_AP1A].off[0]++; R[L_AP1B].off[0]++; }
    }

    wr(&R[L_PRE], t, in);
    float x = rd(&R[L_PRE], 0, t);
    v->lp_pre += (x - v->lp_pre) * v->a_prefilter;
    x = v->lp_pre;
    x = allpass(&R[L_IN0], t, v->a_in1, x);
    x = allpass(&R[L_IN1], t, v->a_in1, x);
    x = allpass(&R[L_IN2], t, v->a_in2, x);
    x = allpass(&R[L_IN3], t, v->a_in2, x);

    for (int h = 0; h < 2; h++) {
        ring_t *ap1 = &R[h ? L_AP1B : L_AP1A];
        ring_t *dl1 = &R[h ? L_DL1B : L_DL1A];
        ring_t *ap2 = &R[h ? L_AP2B : L_AP2A];
        ring_t *dl2 = &R[h ? L_DL2B : L_DL2A];
        ring_t *fb  = &R[h ? L_DL2A : L_DL2B];
        float y = x + rd(fb, 0, t) * v->a_decay;
        y = allpass(ap1, t, -v->a_dd1, y);
        wr(dl1, t, y);
        y = rd(dl1, 0, t);
        v->lp_damp[h] += (y - v->lp_damp[h]) * v->a_damping;
        y = v->lp_damp[h];
        y *= v->a_decay;
        y = allpass(ap2, t, v->a_dd2, y);
        wr(dl2, t, y);
    }

    const uint16_t tn = (uint16_t)(t + 1);
    v->t = tn;

    /* stereo taps at the incremented t, verb.cpp:302-325 */
    float l = rd(&R[L_DL1B], 1, tn);
    l += rd(&R[L_DL1B], 2, tn);
    l -= rd(&R[L_AP2B], 2, tn);
    l += rd(&R[L_DL2B], 2, tn);
    l -= rd(&R[L_DL1A], 3, tn);
    l -= rd(&R[L_AP2A], 1, tn);
    l += rd(&R[L_DL2A], 1, tn);
    float r = rd(&R[L_DL1A], 1, tn);
    r += rd(&R[L_DL1A], 2, tn);
    r -= rd(&R[L_AP2A], 2, tn);
    r += rd(&R[L_DL2A], 2, tn);
    r -= rd(&R[L_DL1B], 3, tn);
    r -= rd(&R[L_AP2B], 1, tn);
    r += rd(&R[L_DL2B], 1, tn);
    *outl = l;
    *outr = r;
}

oracle_dattorro *oracle_dattorro_create(int n_inst)
{
    if (n_inst <= 0) return NULL;
    oracle_dattorro *o = (oracle_dattorro *)calloc(1, sizeof(*o));
    if (!o) return NULL;
    const size_t per = oracle_dattorro_state_floats();
    o->n = n_inst;
    o->pool = (float *)malloc(per * (size_t)n_inst * sizeof(float));
    o->v = (verb_t *)malloc(sizeof(verb_t) * (size_t)n_inst);
    if (!o->pool || !o->v) { oracle_dattorro_destroy(o); return NULL; }
    for (int i = 0; i < n_inst; i++) verb_init(&o->v[i], o->pool + per * (size_t)i);
    return o;
}

void oracle_dattorro_destroy(oracle_dattorro *o)
{
    if (!o) return;
    free(o->pool);
    free(o->v);
    free(o);
}

int oracle_dattorro_set(oracle_dattorro *o, int inst, int field, float value)
{
    if (!o || inst < 0 || inst >= o->n || field < 0 || field >= ODT_NPARAMS) return -1;
    verb_set(&o->v[inst], field, value);
    return 0;
}

/*
 * in : [in_ch][n_frames][n_inst] (in_ch 1 = the C API's mono input, 2 = fxlib's (l+r)/2)
 * out: [2][n_frames][n_inst]
 * Instances are independent; threads split them statically (OpenMP when built with it).
 */
int oracle_dattorro_process(oracle_dattorro *o, const float *in, int in_ch, float *out,
                            int n_frames, int n_threads)
{
    if (!o || (in_ch != 1 && in_ch != 2) || n_frames < 0) return -1;
    const long n = o->n;
    const long plane = n * (long)n_frames;
    (void)n_threads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
#endif
    for (long i = 0; i < n; i++) {
        verb_t *v = &o->v[i];
        for (int f = 0; f < n_frames; f++) {
            float x = in[(long)f * n + i];
            if (in_ch == 2) x = (x + in[plane + (long)f * n + i]) / 2;
            verb_tick(v, x, &out[(long)f * n + i], &out[plane + (long)f * n + i]);
        }
    }
    return 0;
}

/* ---- KAT helpers ---- */

/* xorshift32 white noise: s ^= s<<13; s ^= s>>17; s ^= s<<5; x = (float)(int32)s / 2^31 * 0.5 */
uint32_t oracle_xorshift_noise(uint32_t seed, float *out, long n, long stride)
{
    uint32_t s = seed;
    for (long k = 0; k < n; k++) {
        s ^= s << 13;
        s ^= s >> 17;
        s ^= s << 5;
        out[k * stride] = (float)((int32_t)s) / 2147483648.0f * 0.5f;
    }
    return s;
}

/* FNV-1a 64 over the little-endian bytes of L[f] then R[f] for every frame */
uint64_t oracle_fnv1a64_lr(const float *l, const float *r, long n_frames, long stride)
{
    uint64_t h = 0xcbf29ce484222325ull;
    for (long f = 0; f < n_frames; f++) {
        const float v[2] = {l[f * stride], r[f * stride]};
        const unsigned char *b = (const unsigned char *)v;
        for (int k = 0; k < 8; k++) { h ^= b[k]; h *= 0x100000001b3ull; }
    }
    return h;
}
