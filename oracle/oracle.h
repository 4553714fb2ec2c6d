/*
 * oracle/oracle.h -- C API of the CPU oracle (TEST INFRASTRUCTURE ONLY).
 *
 * Used by tests/ (via ctypes), __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Never linked into the product library (ol_dsp_amd/libolfx.so).
 *
 * Layouts match the product C-ABI (include/olfx.h):
 *   audio in : [in_ch][n_frames][n_inst]   (instance index fastest)
 *   audio out: [out_ch][n_frames][n_inst]
 */
#ifndef OLFX_ORACLE_H
#define OLFX_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* ---- Dattorro plate reverb (bit-exact restatement of libs/dattorro-verb/verb.cpp) ---- */
enum {
    ODT_PREDELAY = 0,          /* DattorroVerb_setPreDelay       verb.cpp:137 */
    ODT_PREFILTER,             /* DattorroVerb_setPreFilter      verb.cpp:142 */
    ODT_INPUT_DIFFUSION1,      /* DattorroVerb_setInputDiffusion1 verb.cpp:147 */
    ODT_INPUT_DIFFUSION2,      /* DattorroVerb_setInputDiffusion2 verb.cpp:152 */
    ODT_DECAY_DIFFUSION,       /* DattorroVerb_setDecayDiffusion verb.cpp:157 */
    ODT_DECAY,                 /* DattorroVerb_setDecay          verb.cpp:162 */
    ODT_DAMPING,               /* DattorroVerb_setDamping        verb.cpp:168 */
    ODT_NPARAMS
};
typedef struct oracle_dattorro oracle_dattorro;
size_t oracle_dattorro_state_floats(void);
oracle_dattorro *oracle_dattorro_create(int n_inst);
void oracle_dattorro_destroy(oracle_dattorro *o);
int oracle_dattorro_set(oracle_dattorro *o, int inst, int field, float value);
int oracle_dattorro_process(oracle_dattorro *o, const float *in, int in_ch, float *out,
                            int n_frames, int n_threads);
/* KAT helpers: xorshift32 noise and FNV-1a-64 over L,R frame bytes */
uint32_t oracle_xorshift_noise(uint32_t seed, float *out, long n, long stride);
uint64_t oracle_fnv1a64_lr(const float *l, const float *r, long n_frames, long stride);

/* ---- RNBO stereo chorus / gen~ pitch-shift (spec oracle, parity unpinned) ---- */
enum {
    OCH_PITCH = 0, OCH_MIX, OCH_Q, OCH_CUTOFF, OCH_PHASE, OCH_DEPTH, OCH_RATE, OCH_WINDOW,
    OCH_NPARAMS
};
typedef struct oracle_chorus oracle_chorus;
float oracle_cos2pi(float x);
double oracle_cos2pi_d(double x);
void oracle_win_gains(float p, float *g0, float *g1);
/* mode 0 = full chorus, 1 = pitch-shift stage only (params OCH_PITCH = shift Hz, OCH_WINDOW) */
oracle_chorus *oracle_chorus_create(int n_inst, float sample_rate, int mode);
void oracle_chorus_destroy(oracle_chorus *o);
int oracle_chorus_set(oracle_chorus *o, int inst, int field, float value);
int oracle_chorus_process(oracle_chorus *o, const float *in, float *out, int n_frames, int n_threads);
/* config 1: one instance, one core, per-frame calls in fx_test.cpp:45-54's shape */
long oracle_chorus_c1(float sample_rate, const float *params, long n_frames, int block, double *sum_abs);

/* The same chorus / pitch-shift in double precision with double phasors (gen~ / RNBO arithmetic;
   oracle/chorus_ref_f64.c): measures the fp32 spec's arithmetic deviation.  out is double.
   mode: bit 0 as oracle_chorus_create; bit 1 = phasor increments rounded to the spec's 32-bit
   fixed point (isolates the fp32 arithmetic from the increment rounding). */
typedef struct oracle_chorus64 oracle_chorus64;
oracle_chorus64 *oracle_chorus64_create(int n_inst, double sample_rate, int mode);
void oracle_chorus64_destroy(oracle_chorus64 *o);
int oracle_chorus64_set(oracle_chorus64 *o, int inst, int field, double value);
int oracle_chorus64_process(oracle_chorus64 *o, const float *in, double *out, int n_frames);

/* ---- synthlib SynthVoice (DaisySP restatement, parity unpinned) ---- */
enum {  /* Voice::Config order, modules/synthlib/Voice.h:14-31 */
    OVC_FILTER_CUTOFF = 0, OVC_FILTER_RESONANCE, OVC_FILTER_DRIVE, OVC_FILTER_ENV_AMOUNT,
    OVC_FILTER_ATTACK, OVC_FILTER_ATTACK_SHAPE, OVC_FILTER_DECAY, OVC_FILTER_SUSTAIN,
    OVC_FILTER_RELEASE, OVC_AMP_ENV_AMOUNT, OVC_AMP_ATTACK, OVC_AMP_ATTACK_SHAPE,
    OVC_AMP_DECAY, OVC_AMP_SUSTAIN, OVC_AMP_RELEASE, OVC_PORTAMENTO,
    OVC_NPARAMS
};
typedef struct oracle_voice oracle_voice;
oracle_voice *oracle_voice_create(int n_inst, float sample_rate);
/* model 0: SvfFilter voice (SynthVoice default), 1: MoogFilter voice (daisysp::LadderFilter) */
oracle_voice *oracle_voice_create_model(int n_inst, float sample_rate, int model);
void oracle_voice_destroy(oracle_voice *o);
int oracle_voice_config(oracle_voice *o, int inst, const float *values);
/* member values set before Init, then Init (no Update): see voice_ref.c */
int oracle_voice_init_members(oracle_voice *o, int inst, const float *values);
int oracle_voice_note(oracle_voice *o, int inst, int on, int note);
/* 0 NoteOff, 1 NoteOn, 2 GateOn, 3 GateOff, 4 SetFrequency(value Hz) (Voice.h:33-57) */
int oracle_voice_event(oracle_voice *o, int inst, int type, int note, float value);
int oracle_voice_process(oracle_voice *o, float *out, int n_frames, int n_threads);
/* arith 1: the GPU kernels' arithmetic (contractions, sine polynomial, v_rcp model; voice_ref.c),
   0: the unfused restatement (default) */
int oracle_voice_set_arith(oracle_voice *o, int kernel);
/* v_rcp_f32's 2^23 results over the mantissas of [1, 2) (copied); NULL: correctly rounded 1/x */
int oracle_rcp_table_set(const uint32_t *tab);
float oracle_rcp_model(float x);

/* ---- fxlib effect rack ol::fx::FxRack<2> (spec oracle for the DaisySP parts, parity unpinned) ---- */
enum {
    OFR_DELAY_TIME = 0,        /* DelayFx time [0,1] -> SetDelay(time * 48000)          Fx.h:172,214 */
    OFR_DELAY_FEEDBACK,        /* DelayFx feedback                                      Fx.h:173 */
    OFR_DELAY_BALANCE,         /* DelayFx wet/dry balance                               Fx.h:174 */
    OFR_DELAY_CUTOFF,          /* DelayFx filter_ cutoff, Hz                            Fx.h:188 */
    OFR_DELAY_RESONANCE,       /* DelayFx filter_ resonance [0,1]                       Fx.h:189 */
    OFR_REVERB_BALANCE,        /* ReverbFx balance                                      Fx.h:282 */
    OFR_FILTER_CUTOFF,         /* FxRack filter1 cutoff, Hz                             Fx.h:75 */
    OFR_FILTER_RESONANCE,      /* FxRack filter1 resonance [0,1] */
    OFR_FILTER_DRIVE,          /* FxRack filter1 drive [0,1] */
    OFR_FILTER_TYPE,           /* 0 low, 1 band, 2 high, 3 notch, 4 peak                Fx.h:67-73 */
    OFR_MASTER_VOLUME,         /* FxRack master_volume                                  Fx.h:405 */
    OFR_TOPOLOGY,              /* 0 FxRack<2>; 1 the synth firmware callback (main.cpp:78-86); 2 DelayFx<2>,
                                  3 ReverbFx<2>, 4 FilterFx<2> alone (main.cpp:82-85) */
    OFR_NPARAMS
};
typedef struct oracle_fxrack oracle_fxrack;
void oracle_fxrack_defaults(float *p);
oracle_fxrack *oracle_fxrack_create(int n_inst, float sample_rate);
void oracle_fxrack_destroy(oracle_fxrack *o);
int oracle_fxrack_set(oracle_fxrack *o, int inst, int field, float value);
/* in / out: [2][n_frames][n_inst] */
int oracle_fxrack_process(oracle_fxrack *o, const float *in, float *out, int n_frames, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
