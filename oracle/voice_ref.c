/*
 * oracle/voice_ref.c -- CPU oracle for the synthlib SynthVoice (osc + 2 ADSR + SVF + portamento).
 *
 * TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline).  Never part of the product.
 *
 * Parity status: UNPINNED for the DaisySP arithmetic.  The voice composition is in-tree and
 * restated literally from modules/synthlib/SynthVoice.h:31-53 (Init/Process), :55-98
 * (UpdateConfig/Update), :245-256 (NoteOn/NoteOff), Portamento.h:12-42 (in-tree daisysp::Port
 * stub), but the primitives are the third-party module DaisySP (pinned only as "commit": "master"
 * in submodules.json:74-80, fork URL .gitmodules:4-6), which is not vendored and not in this
 * container.  Its published algorithm is restated here:
 *   daisysp::Oscillator (WAVE_POLYBLEP_SAW, normalised phase, amp 0.5),
 *   daisysp::Adsr (Init(sr, 1), SetAttackTime(t, shape), SetTimeConstant, Process(gate), Retrigger),
 *   daisysp::Svf (double-sampled Chamberlin, SetFreq/SetRes/SetDrive, Low()),
 *   daisysp::mtof,
 *   daisysp::LadderFilter (the MoogFilter voice of the Daisy synth firmware, Filter.h:35-63,
 *   ol_daisy/app/synth/main.cpp:49-52): Huovilainen-style 4-pole ladder, 4x linear-interpolated
 *   oversampling, Pade tanh on the feedback sum, one-zero/one-pole stages (0.3/1.3 zero), the
 *   polynomial alpha/Qadjust fit of the normalised cutoff, LP24 output.  [unverified] against the
 *   DaisySP source, like the rest of this file.
 * The only reference pins at this boundary are qualitative (synth_test.cpp:102-148: first sample
 * after NoteOn/NoteOff/NoteOn is exactly 0, later != 0 and != 1; amp_env_amount 0 -> 0) and are
 * reproduced by tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

enum { SEG_IDLE = 0, SEG_ATTACK = 1, SEG_DECAY = 2, SEG_RELEASE = 3 };

typedef struct {
    float x, atk_d0, atk_tgt, dec_d0, rel_d0, sus;
    int mode, gate_prev;
} adsr_t;

typedef struct {
    /* oscillator */
    float phase, sr_recip;
    /* svf */
    float sr, fc_max, res, pre_drive, drive, low, band;
    /* ladder (daisysp::LadderFilter, MoogFilter voices only) */
    float lz0[4], lz1[4], l_old, alpha_scratch, l_k, l_pbg, l_drive_scaled, l_sr_int_recip;
    int model;                      /* 0: SvfFilter (SynthVoice default), 1: MoogFilter */
    /* port */
    float port_coef, port_z;
    adsr_t amp_env, filt_env;
    /* voice members (SynthVoice.h:276-315) */
    float freq, amp_env_amount, filter_cutoff, filter_env_amount;
    int gate;
} voice_t;

struct oracle_voice {
    int n;
    float sr;
    int arith;        /* 0: the restatement (unfused, glibc sinf); 1: the kernels' arithmetic (below) */
    voice_t *v;
    float *params;    /* [n][OVC_NPARAMS] SynthVoice members (Config order) */
};

/* daisysp::Adsr setters */
static void adsr_attack(adsr_t *e, float T, float shape, float sr)
{
    float target = 9.f * powf(shape, 10.f) + 0.3f * shape + 1.01f;
    e->atk_tgt = target;
    if (T > 0.f) {
        float logTarget = logf(1.f - (1.f / target));
        e->atk_d0 = 1.f - expf(logTarget / (T * sr));
    } else {
        e->atk_d0 = 1.f;
    }
}
static float adsr_tc(float T, float sr)
{
    if (T > 0.f) {
        const float target = logf((float)(1. / M_E));
        return 1.f - expf(target / (T * sr));
    }
    return 1.f;
}
static float adsr_sus(float s) { return (s <= 0.f) ? -0.01f : (s > 1.f ? 1.f : s); }

static void adsr_init(adsr_t *e, float sr)
{
    memset(e, 0, sizeof(*e));
    e->sus = 0.7f;
    e->mode = SEG_IDLE;
    adsr_attack(e, 0.1f, 0.0f, sr);
    e->dec_d0 = adsr_tc(0.1f, sr);
    e->rel_d0 = adsr_tc(0.1f, sr);
}

static float adsr_process(adsr_t *e, int gate)
{
    if (gate && !e->gate_prev) e->mode = SEG_ATTACK;
    else if (!gate && e->gate_prev) e->mode = SEG_RELEASE;
    e->gate_prev = gate;
    float d0 = e->atk_d0;
    if (e->mode == SEG_DECAY) d0 = e->dec_d0;
    else if (e->mode == SEG_RELEASE) d0 = e->rel_d0;
    float target = e->mode == SEG_DECAY ? e->sus : -0.01f;
    float out = 0.0f;
    switch (e->mode) {
    case SEG_ATTACK:
        e->x += d0 * (e->atk_tgt - e->x);
        out = e->x;
        if (out > 1.f) { e->x = out = 1.f; e->mode = SEG_DECAY; }
        break;
    case SEG_DECAY:
    case SEG_RELEASE:
        e->x += d0 * (target - e->x);
        out = e->x;
        if (out < 0.0f) { e->x = out = 0.f; e->mode = SEG_IDLE; }
        break;
    default: break;
    }
    return out;
}

static float polyblep(float dt, float t)
{
    if (t < dt) { t /= dt; return t + t - t * t - 1.0f; }
    else if (t > 1.0f - dt) { t = (t - 1.0f) / dt; return t * t + t + t + 1.0f; }
    return 0.0f;
}

static float fclampf(float in, float mn, float mx) { return fminf(fmaxf(in, mn), mx); }
#define MINF(a, b) ((a) < (b) ? (a) : (b))

/* daisysp::LadderFilter::Init(sr): SetPassbandGain(0.5), SetInputDrive(0.5), SetFreq(5000),
 * SetRes(0.2).  SetFreq is re-issued every sample by SynthVoice::Process, so only K, pbg and the
 * input drive persist. */
#define LADDER_OS 4
static void ladder_init(voice_t *v, float sr)
{
    memset(v->lz0, 0, sizeof(v->lz0));
    memset(v->lz1, 0, sizeof(v->lz1));
    v->l_old = 0.f;
    v->l_sr_int_recip = 1.0f / (sr * LADDER_OS);
    v->l_pbg = 0.5f;
    v->l_drive_scaled = 0.5f;           /* SetInputDrive(0.5): drive <= 1 -> drive_scaled = drive */
    v->l_k = 4.0f * 0.2f;               /* SetRes(0.2) */
}

/* LadderFilter::SetRes: K = 4 * clamp(res, 0, kMaxResonance = 1.8) */
static float ladder_k(float res) { return 4.0f * fminf(fmaxf(res, 0.0f), 1.8f); }

/* Pade tanh, saturating at |x| > 3 */
static float ladder_tanh(float x)
{
    if (x > 3.0f) return 1.0f;
    if (x < -3.0f) return -1.0f;
    const float x2 = x * x;
    return x * (27.0f + x2) / (27.0f + 9.0f * x2);
}

static float ladder_lpf(voice_t *v, float s, int i)
{
    float ft = s * (1.0f / 1.3f) + (0.3f / 1.3f) * v->lz0[i] - v->lz1[i];
    ft = ft * v->alpha_scratch + v->lz1[i];
    v->lz1[i] = ft;
    v->lz0[i] = s;
    return ft;
}

/* LadderFilter::SetFreq(fc) -> SetAlpha, then LadderFilter::Process(in), LP24 */
static float ladder_process(voice_t *v, float fc, float in)
{
    const float wc = fc * 2.0f * 3.1415927410125732f * v->l_sr_int_recip;
    const float wc2 = wc * wc;
    v->alpha_scratch = 0.9892f * wc - 0.4324f * wc2 + 0.1381f * wc * wc2 - 0.0202f * wc2 * wc2;
    const float qadj = 1.006f + 0.0536f * wc - 0.095f * wc2 - 0.05f * wc2 * wc2;
    const float input = in * v->l_drive_scaled;
    float total = 0.0f, interp = 0.0f;
    for (int os = 0; os < LADDER_OS; os++) {
        float u = (interp * v->l_old + (1.0f - interp) * input) - (v->lz1[3] - v->l_pbg * input) * v->l_k * qadj;
        u = ladder_tanh(u);
        const float s1 = ladder_lpf(v, u, 0);
        const float s2 = ladder_lpf(v, s1, 1);
        const float s3 = ladder_lpf(v, s2, 2);
        const float s4 = ladder_lpf(v, s3, 3);
        total += s4 * (1.0f / LADDER_OS);
        interp += 1.0f / LADDER_OS;
    }
    v->l_old = input;
    return total;
}

static void voice_init(voice_t *v, float sr, int model)
{
    memset(v, 0, sizeof(*v));
    v->model = model;
    ladder_init(v, sr);
    v->sr_recip = 1.0f / sr;                        /* Oscillator::Init */
    v->sr = sr; v->fc_max = sr / 3.f;               /* Svf::Init */
    v->res = 0.5f; v->pre_drive = 0.5f; v->drive = 0.5f;
    adsr_init(&v->amp_env, sr);                     /* SynthVoice::Init: Init(sr, 1) x2 */
    adsr_init(&v->filt_env, sr);
    v->port_coef = expf(-1.0f / (0.0f * sr));       /* Port::Init(sr, portamento_htime = 0, the member default) */
    v->amp_env_amount = 0.8f;
    v->filter_cutoff = 0.0f;
    v->filter_env_amount = 1.0f;
}

/* SynthVoice::UpdateConfig -> Update (SynthVoice.h:55-98) */
static void voice_update(voice_t *v, const float *p, float sr)
{
    v->filter_cutoff = p[OVC_FILTER_CUTOFF];
    v->filter_env_amount = p[OVC_FILTER_ENV_AMOUNT];
    v->amp_env_amount = p[OVC_AMP_ENV_AMOUNT];
    /* MoogFilter::SetRes -> LadderFilter::SetRes; MoogFilter::SetDrive is a no-op */
    v->l_k = ladder_k(p[OVC_FILTER_RESONANCE]);
    /* Svf::SetRes, Svf::SetDrive */
    v->res = fclampf(p[OVC_FILTER_RESONANCE], 0.f, 1.f);
    v->drive = v->pre_drive * v->res;
    v->pre_drive = fclampf(p[OVC_FILTER_DRIVE] * 0.1f, 0.f, 1.f);
    v->drive = v->pre_drive * v->res;
    adsr_attack(&v->filt_env, p[OVC_FILTER_ATTACK], p[OVC_FILTER_ATTACK_SHAPE], sr);
    v->filt_env.dec_d0 = adsr_tc(p[OVC_FILTER_DECAY], sr);
    v->filt_env.sus = adsr_sus(p[OVC_FILTER_SUSTAIN]);
    v->filt_env.rel_d0 = adsr_tc(p[OVC_FILTER_RELEASE], sr);
    adsr_attack(&v->amp_env, p[OVC_AMP_ATTACK], p[OVC_AMP_ATTACK_SHAPE], sr);
    v->amp_env.dec_d0 = adsr_tc(p[OVC_AMP_DECAY], sr);
    v->amp_env.sus = adsr_sus(p[OVC_AMP_SUSTAIN]);
    v->amp_env.rel_d0 = adsr_tc(p[OVC_AMP_RELEASE], sr);
    v->port_coef = expf(-1.0f / (p[OVC_PORTAMENTO] * sr));
}

static float voice_tick(voice_t *v)
{
    float amp = adsr_process(&v->amp_env, v->gate);
    amp *= v->amp_env_amount;
    /* Port::Process, Oscillator::SetFreq */
    v->port_z = v->freq + v->port_coef * (v->port_z - v->freq);
    const float inc = v->port_z * v->sr_recip;
    /* Oscillator::Process (WAVE_POLYBLEP_SAW) */
    float o = (2.0f * v->phase) - 1.0f;
    o -= polyblep(inc, v->phase);
    o *= -1.0f;
    v->phase += inc;
    if (v->phase > 1.0f) v->phase -= 1.0f;
    const float src = o * 0.5f;
    /* filter envelope -> Filter::SetFreq */
    const float fc_in = v->filter_cutoff + ((adsr_process(&v->filt_env, v->gate) * 20000) * v->filter_env_amount);
    /* MoogFilter: Process() is a no-op, Low(frame) = LadderFilter::Process(frame); the frequency
     * reaches SetAlpha unclamped */
    if (v->model == 1) return ladder_process(v, fc_in, src) * amp;
    const float fc = fclampf(fc_in, 1.0e-6f, v->fc_max);
    const float fq = 2.0f * sinf(3.1415927410125732f * MINF(0.25f, fc / (v->sr * 2.0f)));
    const float damp = MINF(2.0f * (1.0f - powf(v->res, 0.25f)), MINF(2.0f, 2.0f / fq - fq * 0.5f));
    /* Svf::Process + Low() */
    float notch = src - damp * v->band;
    v->low = v->low + fq * v->band;
    float high = notch - v->low;
    v->band = fq * high + v->band - v->drive * v->band * v->band * v->band;
    float out_low = 0.5f * v->low;
    notch = src - damp * v->band;
    v->low = v->low + fq * v->band;
    high = notch - v->low;
    v->band = fq * high + v->band - v->drive * v->band * v->band * v->band;
    out_low += 0.5f * v->low;
    return out_low * amp;
}

/* ---------------------------------------------------------------------------------------------
 * The kernels' arithmetic (arith = 1).  The GPU voices (ol_dsp_amd/csrc/voice.hip) compute the same
 * composition with three documented departures from the restatement above, restated here operation
 * for operation so that the GPU output can be checked BIT-EXACTLY (tests/test_gpu_parity.py
 * test_voice_bit_exact_kernel_arith); the restatement above stays the tolerance-based check:
 *   1. contraction into fused multiply-adds (C99 fmaf, correctly rounded like v_fma_f32) at the
 *      sites voice.hip lists under "Contraction": the polyBLEP quadratics and the saw's output, the
 *      sine polynomial and the cutoff sum, the Svf's low/band updates, the ladder's stages, its
 *      oversampling interpolation, feedback sum and SetAlpha polynomials;
 *   2. Svf::SetFreq's sinf as the odd Taylor polynomial to x^9 (voice.hip sin_quarter), its
 *      2/fq - fq/2 as 1/s - s (s = fq/2) and fc / (2 sr) as fc * (1 / (2 sr));
 *   3. divisions by the hardware reciprocal v_rcp_f32 (the polyBLEP's t/dt, 1/s, the Pade tanh's
 *      denominator).  v_rcp_f32 is not correctly rounded: measured on gfx950 over every mantissa of
 *      [1, 2) (tools/rcp_probe.hip), it differs from RN(1/x) on 10.70 % of them, always by one ulp
 *      (the exact quotient within 0.1..0.85 ulp of the floor: an approximation of < 0.4 ulp error,
 *      rounded), and rcp(m 2^e) = rcp(m) 2^-e exactly for every normal result.  Its model here is
 *      that table: oracle_rcp_table_set() takes the 2^23 results (the GPU tests read them from the
 *      device, tests/gpu_probe/rcp_probe.hip), scaled by the exponent.  Without a table the model is
 *      the correctly rounded 1/x.  Inputs whose result is not normal (0, denormals, inf: the voices
 *      never divide by them where the quotient is used) fall back to 1/x.
 * Everything else (envelopes, portamento, phase, notch, the Low() sum) is unfused in both. */
static uint32_t *g_rcp_tab;

int oracle_rcp_table_set(const uint32_t *tab)
{
    free(g_rcp_tab);
    g_rcp_tab = NULL;
    if (!tab) return 0;
    g_rcp_tab = (uint32_t *)malloc(sizeof(uint32_t) << 23);
    if (!g_rcp_tab) return -1;
    memcpy(g_rcp_tab, tab, sizeof(uint32_t) << 23);
    return 0;
}

float oracle_rcp_model(float x)
{
    uint32_t b;
    memcpy(&b, &x, 4);
    const int e = (int)((b >> 23) & 0xffu);
    if (!g_rcp_tab || e == 0 || e == 255) return 1.0f / x;
    const uint32_t r = g_rcp_tab[b & 0x7fffffu];
    const int re = (int)((r >> 23) & 0xffu) - (e - 127);
    if (re <= 0 || re >= 255) return 1.0f / x;
    const uint32_t o = (b & 0x80000000u) | ((uint32_t)re << 23) | (r & 0x7fffffu);
    float y;
    memcpy(&y, &o, 4);
    return y;
}

/* voice.hip polyblep + saw_out: q = (lo ? t : t - 1) rcp(dt); fma(-q, q, 2q) - 1 / fma(q, q, 2q) + 1 */
static float k_saw(float t, float dt)
{
    const int lo = t < dt, hi = t > 1.0f - dt;
    const float q = (lo ? t : t - 1.0f) * oracle_rcp_model(dt);
    const float q2 = q + q;
    const float rlo = fmaf(-q, q, q2) - 1.0f;
    const float rhi = fmaf(q, q, q2) + 1.0f;
    const float blep = lo ? rlo : (hi ? rhi : 0.0f);
    return fmaf(0.5f, blep, 0.5f - t);
}

/* voice.hip sin_quarter */
static float k_sin_quarter(float x)
{
    const float x2 = x * x;
    float p = fmaf(2.7557319e-6f, x2, -1.9841270e-4f);
    p = fmaf(p, x2, 8.3333333e-3f);
    p = fmaf(p, x2, -1.6666667e-1f);
    return fmaf(x * x2, p, x);
}

/* voice.hip voice_block_v4 (MOOG) filter wave: LadderFilter::Process contracted, the Pade tanh as
   r(med3(x, -3, 3)) with v_rcp */
static float k_ladder(voice_t *v, float alpha, float qadj, float input)
{
    const float kq = v->l_k * qadj;
    const float fb0 = -0.5f * input, dold = v->l_old - input;
    float total = 0.0f;
    for (int os = 0; os < LADDER_OS; os++) {
        const float interp = 0.25f * (float)os;
        const float mixin = os == 0 ? input : fmaf(interp, dold, input);
        float x = fmaf(-(v->lz1[3] + fb0), kq, mixin);
        x = fminf(fmaxf(x, -3.0f), 3.0f);
        const float x2 = x * x;
        float u = (x * (27.0f + x2)) * oracle_rcp_model(fmaf(9.0f, x2, 27.0f));
        for (int st = 0; st < 4; st++) {
            float ft = fmaf(u, 1.0f / 1.3f, fmaf(0.3f / 1.3f, v->lz0[st], -v->lz1[st]));
            ft = fmaf(ft, alpha, v->lz1[st]);
            v->lz1[st] = ft;
            v->lz0[st] = u;
            u = ft;
        }
        total = fmaf(u, 0.25f, total);
    }
    v->l_old = input;
    return total;
}

static float voice_tick_k(voice_t *v)
{
    const int moog = v->model == 1;
    /* ENV: the segment machine is adsr_process's (voice.hip Env: identical updates and clamps);
       the Svf voice hands FILT amp * (amp_env_amount / 2) (Low()'s halving folded in, exact) */
    const float env_a = adsr_process(&v->amp_env, v->gate);
    const float amp = env_a * (moog ? v->amp_env_amount : 0.5f * v->amp_env_amount);
    /* OSC */
    v->port_z = v->freq + v->port_coef * (v->port_z - v->freq);
    const float inc = v->port_z * v->sr_recip;
    const float t = v->phase;
    v->phase += inc;
    if (v->phase > 1.0f) v->phase -= 1.0f;
    const float src = k_saw(t, inc);
    const float fe = adsr_process(&v->filt_env, v->gate);
    const float fc_in = fmaf(fe * 20000.0f, v->filter_env_amount, v->filter_cutoff);
    if (moog) {
        const float wc = fc_in * 2.0f * 3.1415927410125732f * v->l_sr_int_recip;
        const float wc2 = wc * wc;
        const float alpha = wc * fmaf(fmaf(fmaf(-0.0202f, wc, 0.1381f), wc, -0.4324f), wc, 0.9892f);
        const float qadj = fmaf(fmaf(-0.05f, wc2, -0.095f), wc2, fmaf(0.0536f, wc, 1.006f));
        return k_ladder(v, alpha, qadj, src * v->l_drive_scaled) * amp;
    }
    /* FREQ: Svf::SetFreq */
    const float fc = fminf(fmaxf(fc_in, 1.0e-6f), v->fc_max);
    const float inv_2sr = 1.0f / (v->sr * 2.0f);
    const float s = k_sin_quarter(3.1415927410125732f * fminf(fc * inv_2sr, 0.25f));
    const float fq = s + s;
    const float lim = oracle_rcp_model(s) - s;
    const float damp_res = 2.0f * (1.0f - powf(v->res, 0.25f));
    const float ndamp = fmaxf(fmaxf(-damp_res, -2.0f), -lim);
    /* FILT: Svf::Process, the notch unfused */
    float notch = src + ndamp * v->band;
    v->low = fmaf(fq, v->band, v->low);
    float high = notch - v->low;
    v->band = fmaf(-((v->drive * v->band) * v->band), v->band, fmaf(fq, high, v->band));
    const float low1 = v->low;
    notch = src + ndamp * v->band;
    v->low = fmaf(fq, v->band, v->low);
    high = notch - v->low;
    v->band = fmaf(-((v->drive * v->band) * v->band), v->band, fmaf(fq, high, v->band));
    return (low1 + v->low) * amp;
}

int oracle_voice_set_arith(oracle_voice *o, int kernel)
{
    if (!o || kernel < 0 || kernel > 1) return -1;
    o->arith = kernel;
    return 0;
}

oracle_voice *oracle_voice_create(int n_inst, float sample_rate)
{
    return oracle_voice_create_model(n_inst, sample_rate, 0);
}

oracle_voice *oracle_voice_create_model(int n_inst, float sample_rate, int model)
{
    if (n_inst <= 0 || model < 0 || model > 1) return NULL;
    oracle_voice *o = (oracle_voice *)calloc(1, sizeof(*o));
    if (!o) return NULL;
    o->n = n_inst;
    o->sr = sample_rate;
    o->v = (voice_t *)calloc((size_t)n_inst, sizeof(voice_t));
    o->params = (float *)calloc((size_t)n_inst * OVC_NPARAMS, sizeof(float));
    if (!o->v || !o->params) { oracle_voice_destroy(o); return NULL; }
    for (int i = 0; i < n_inst; i++) voice_init(&o->v[i], sample_rate, model);
    return o;
}

void oracle_voice_destroy(oracle_voice *o)
{
    if (!o) return;
    free(o->v); free(o->params); free(o);
}

/* values: [OVC_NPARAMS] = a full Voice::Config (UpdateConfig semantics) */
int oracle_voice_config(oracle_voice *o, int inst, const float *values)
{
    if (!o || inst < 0 || inst >= o->n || !values) return -1;
    memcpy(o->params + (size_t)inst * OVC_NPARAMS, values, sizeof(float) * OVC_NPARAMS);
    voice_update(&o->v[inst], values, o->sr);
    return 0;
}

/* Setters called before SynthVoice::Init, then Init (SynthVoice.h:31-39; the Daisy firmware's
   order, ol_daisy/app/synth/main.cpp:114-128, 149): the members hold the values, Init resets the
   components to DaisySP's defaults and hands the member portamento_htime to Port::Init; Process
   reads filter_cutoff, filter_env_amount and amp_env_amount from the members. */
int oracle_voice_init_members(oracle_voice *o, int inst, const float *values)
{
    if (!o || inst < 0 || inst >= o->n || !values) return -1;
    voice_t *v = &o->v[inst];
    voice_init(v, o->sr, v->model);
    memcpy(o->params + (size_t)inst * OVC_NPARAMS, values, sizeof(float) * OVC_NPARAMS);
    v->filter_cutoff = values[OVC_FILTER_CUTOFF];
    v->filter_env_amount = values[OVC_FILTER_ENV_AMOUNT];
    v->amp_env_amount = values[OVC_AMP_ENV_AMOUNT];
    v->port_coef = expf(-1.0f / (values[OVC_PORTAMENTO] * o->sr));
    return 0;
}

int oracle_voice_note(oracle_voice *o, int inst, int on, int note)
{
    if (!o || inst < 0 || inst >= o->n) return -1;
    voice_t *v = &o->v[inst];
    if (on) {
        v->gate = 1;
        v->freq = powf(2.f, ((float)note - 69.0f) / 12.0f) * 440.0f;
        v->amp_env.mode = SEG_ATTACK; v->amp_env.x = 0.f;     /* Retrigger(true) */
        v->filt_env.mode = SEG_ATTACK; v->filt_env.x = 0.f;
    } else {
        v->gate = 0;
    }
    return 0;
}

/* Voice.h:33-57 gate / pitch calls (types as include/olfx.h OLFX_EV_*): 0 NoteOff, 1 NoteOn,
   2 GateOn (SynthVoice.h:231-234), 3 GateOff (:236-239), 4 SetFrequency(value) (:264-267) */
int oracle_voice_event(oracle_voice *o, int inst, int type, int note, float value)
{
    if (!o || inst < 0 || inst >= o->n) return -1;
    voice_t *v = &o->v[inst];
    switch (type) {
    case 0: case 1: return oracle_voice_note(o, inst, type, note);
    case 2: v->gate = 1; return 0;
    case 3: v->gate = 0; return 0;
    case 4: v->freq = value; return 0;
    default: return -1;
    }
}

/* out [n_frames][n] */
int oracle_voice_process(oracle_voice *o, float *out, int n_frames, int n_threads)
{
    if (!o || n_frames < 0) return -1;
    const long n = o->n;
    const int k = o->arith;
    (void)n_threads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
#endif
    for (long i = 0; i < n; i++)
        for (int f = 0; f < n_frames; f++)
            out[(long)f * n + i] = k ? voice_tick_k(&o->v[i]) : voice_tick(&o->v[i]);
    return 0;
}
