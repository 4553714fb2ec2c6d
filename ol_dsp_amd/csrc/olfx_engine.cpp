// ol_dsp_amd/csrc/olfx_engine.cpp -- host side of libolfx.so: the C-ABI of include/olfx.h.
//
// Owns all device state of an engine (SoA rings, recursive scalars, derived coefficients),
// derives per-instance coefficients from the reference's setter semantics on the host (control
// rate), applies parameter changes / note events at block boundaries, and launches the gfx950
// kernels on a HIP stream.  There is no CPU compute path: if no GPU is present olfx_create
// fails with OLFX_E_NODEVICE.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/olfx.h"
#include "olfx_internal.h"

using namespace olfx;

namespace {

std::mutex g_err_mu;
std::string g_err;

void set_global_error(const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_err = buf;
}

}  // namespace

// for the per-sample pool (olfx_sample_pool.cpp): its failures are reported through
// olfx_last_error(NULL) like engine-less errors here
void olfx::internal_set_error(const char *msg) { set_global_error("%s", msg); }

namespace {

uint32_t pow2_at_least(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }

// a fraction of a cycle in [0, 1] as 64-bit fixed point (2^64 = one cycle); 1.0 wraps to 0
uint64_t fix64(double cycles) {
    constexpr double kTwo64 = 18446744073709551616.0;
    const double v = std::floor(cycles * kTwo64 + 0.5);
    return v <= 0 ? 0u : (v >= kTwo64 ? (uint64_t)(v - kTwo64) : (uint64_t)v);
}

uint32_t as_u32(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

// ---------------------------------------------------------------------------------------------
// Per-kind constants
// ---------------------------------------------------------------------------------------------
uint32_t n_params_of(int kind) {
    switch (kind) {
    case OLFX_KIND_DATTORRO: return OLFX_DT_NPARAMS;
    case OLFX_KIND_CHORUS: return OLFX_CH_NPARAMS;
    case OLFX_KIND_PITCHSHIFT: return OLFX_PS_NPARAMS;
    case OLFX_KIND_VOICE:
    case OLFX_KIND_VOICE_MOOG: return OLFX_VC_NPARAMS;
    case OLFX_KIND_CHAIN: return OLFX_CN_NPARAMS;
    case OLFX_KIND_FXRACK: return OLFX_FR_NPARAMS;
    default: return 0;
    }
}

// ol::core::scale (modules/corelib/ol_corelib.h:27-44), t_sample = float
float core_scale(float in, float inlow, float inhigh, float outlow, float outhigh, float power) {
    const float denom = inhigh - inlow;
    const float inscale = denom == 0.f ? 0.f : (float)(1.f / denom);
    const float outdiff = outhigh - outlow;
    float value = (in - inlow) * inscale;
    if (value > 0.0f) value = powf(value, power);
    else if (value < 0.0f) value = -powf(-value, power);
    return (value * outdiff) + outlow;
}

// Reference defaults of the user-facing parameters.
void default_params(int kind, float *p) {
    switch (kind) {
    case OLFX_KIND_DATTORRO:
        // verb.cpp:215-221
        p[OLFX_DT_PREDELAY] = (float)0.1;
        p[OLFX_DT_PREFILTER] = (float)0.85;
        p[OLFX_DT_INPUT_DIFFUSION1] = (float)0.75;
        p[OLFX_DT_INPUT_DIFFUSION2] = (float)0.625;
        p[OLFX_DT_DECAY_DIFFUSION] = (float)0.70;
        p[OLFX_DT_DECAY] = (float)0.75;
        p[OLFX_DT_DAMPING] = (float)0.95;
        break;
    case OLFX_KIND_CHORUS:
        // mono-chorus.rnbopat param boxes (:431,1772,2226,2660,3420,3854,4353)
        p[OLFX_CH_PITCH] = 0.0f;
        p[OLFX_CH_MIX] = 0.5f;
        p[OLFX_CH_Q] = 0.5f;
        p[OLFX_CH_CUTOFF] = 0.3f;
        p[OLFX_CH_PHASE] = 1.0f;
        p[OLFX_CH_DEPTH] = 0.5f;
        p[OLFX_CH_RATE] = 0.2f;
        p[OLFX_CH_WINDOW] = 10.0f;
        break;
    case OLFX_KIND_PITCHSHIFT:
        p[OLFX_PS_SHIFT] = 0.0f;
        p[OLFX_PS_WINDOW] = 10.0f;
        break;
    case OLFX_KIND_VOICE:
    case OLFX_KIND_VOICE_MOOG:
        // SynthVoice member defaults (SynthVoice.h:285-311); Config order (Voice.h:14-31)
        p[OLFX_VC_FILTER_CUTOFF] = 0.0f;
        p[OLFX_VC_FILTER_RESONANCE] = 0.0f;
        p[OLFX_VC_FILTER_DRIVE] = 0.0f;
        p[OLFX_VC_FILTER_ENV_AMOUNT] = 1.0f;
        p[OLFX_VC_FILTER_ATTACK] = 0.0f;
        p[OLFX_VC_FILTER_ATTACK_SHAPE] = 1.0f;
        p[OLFX_VC_FILTER_DECAY] = 0.2f;
        p[OLFX_VC_FILTER_SUSTAIN] = 0.0f;
        p[OLFX_VC_FILTER_RELEASE] = 0.0f;
        p[OLFX_VC_AMP_ENV_AMOUNT] = 0.8f;
        p[OLFX_VC_AMP_ATTACK] = 0.01f;
        p[OLFX_VC_AMP_ATTACK_SHAPE] = 1.0f;
        p[OLFX_VC_AMP_DECAY] = 0.0f;
        p[OLFX_VC_AMP_SUSTAIN] = 1.0f;
        p[OLFX_VC_AMP_RELEASE] = 0.01f;
        p[OLFX_VC_PORTAMENTO] = 0.0f;
        break;
    case OLFX_KIND_CHAIN:
        default_params(OLFX_KIND_CHORUS, p + OLFX_CN_CHORUS0);
        default_params(OLFX_KIND_PITCHSHIFT, p + OLFX_CN_PITCH0);
        default_params(OLFX_KIND_DATTORRO, p + OLFX_CN_VERB0);
        break;
    case OLFX_KIND_FXRACK:
        // Fx.h member defaults; DelayFx::Init sets its filter through UpdateMidiControl(CC, 64 / 24)
        p[OLFX_FR_DELAY_TIME] = 0.5f;
        p[OLFX_FR_DELAY_FEEDBACK] = 0.5f;
        p[OLFX_FR_DELAY_BALANCE] = 0.33f;
        p[OLFX_FR_DELAY_CUTOFF] = core_scale(64.f, 0.f, 127.f, 0.f, 20000.f, 1.f);
        p[OLFX_FR_DELAY_RESONANCE] = core_scale(24.f, 0.f, 127.f, 0.f, 1.f, 1.f);
        p[OLFX_FR_REVERB_BALANCE] = 0.1f;
        p[OLFX_FR_FILTER_CUTOFF] = 20000.f;
        p[OLFX_FR_FILTER_RESONANCE] = 0.f;
        p[OLFX_FR_FILTER_DRIVE] = 0.f;
        p[OLFX_FR_FILTER_TYPE] = 0.f;
        p[OLFX_FR_MASTER_VOLUME] = 0.8f;
        p[OLFX_FR_TOPOLOGY] = 0.f;
        break;
    default: break;
    }
}

// ---------------------------------------------------------------------------------------------
// Coefficient derivation (control rate, host).  These restate the reference setters.
// ---------------------------------------------------------------------------------------------
uint32_t dattorro_predelay_samples(float v) {
    // verb.cpp:137-139: uint16(value * 4800.f) into DelayBuffer_setDelay, whose read offset
    // mask + 1 - delay (verb.cpp:59-61) on the 8192-sample pre-delay ring makes the effective delay
    // uint16(value * 4800) mod 8192 (olfx_set_params accepts value * 4800 in [0, 65536))
    float d = v * 4800.0f;
    return d <= 0.0f ? 0u : ((uint32_t)(uint16_t)d & (kDtSize[DT_PRE] - 1u));
}

void derive_dattorro(const float *p, float *c) {
    c[DTC_PREFILTER] = p[OLFX_DT_PREFILTER];
    c[DTC_IN1] = p[OLFX_DT_INPUT_DIFFUSION1];
    c[DTC_IN2] = p[OLFX_DT_INPUT_DIFFUSION2];
    c[DTC_DD1] = p[OLFX_DT_DECAY_DIFFUSION];
    c[DTC_DAMPING] = p[OLFX_DT_DAMPING];
    c[DTC_DECAY] = p[OLFX_DT_DECAY];
    // verb.cpp:49,162-165: clamp(t_sample x, ...) narrows value+0.15 to float
    float x = (float)((double)p[OLFX_DT_DECAY] + 0.15);
    c[DTC_DD2] = x < 0.25f ? 0.25f : (x > 0.5f ? 0.5f : x);
    c[DTC_PREDELAY] = (float)dattorro_predelay_samples(p[OLFX_DT_PREDELAY]);
}

// chorus: p = [OLFX_CH_*], c = [CHC_*] (u32 words)
void derive_chorus(const float *p, double sr, uint32_t *c) {
    const double pitch = clampf(p[OLFX_CH_PITCH], 0.0f, 3.0f);
    const double mix = clampf(p[OLFX_CH_MIX], 0.0f, 1.0f);
    const double q = clampf(p[OLFX_CH_Q], 0.0f, 1.0f);
    const double cutoff = clampf(p[OLFX_CH_CUTOFF], 0.0f, 1.0f);
    const double phase = clampf(p[OLFX_CH_PHASE], 0.0f, 1.0f);
    const double depth = clampf(p[OLFX_CH_DEPTH], 0.08f, 1.0f);
    const double rate = clampf(p[OLFX_CH_RATE], 0.01f, 1.0f);
    const double window = clampf(p[OLFX_CH_WINDOW], 4.0f, 10.0f);

    const double rate_hz = 0.01 + rate * (0.5 - 0.01);           // scale 0 1 0.01 0.5 (:3935)
    const double depth_ms = 1.0 + depth * (12.0 - 1.0);          // scale 0 1 1 12 1   (:3436)
    const double fc = 300.0 + cutoff * (15000.0 - 300.0);         // scale 0 1 300 15000 1 (:2242)
    // 64-bit phasors: the increment rounding drifts a phase by < 2^-64 cycle per sample
    const uint64_t lfo_inc = fix64(rate_hz / sr), lfo_off = fix64(phase), ps_inc = fix64(pitch / sr);
    c[CHC_LFO_INC] = (uint32_t)(lfo_inc >> 32);
    c[CHC_LFO_INC_LO] = (uint32_t)lfo_inc;
    c[CHC_LFO_OFF] = (uint32_t)(lfo_off >> 32);                   // phase 1.0 wraps to 0
    c[CHC_LFO_OFF_LO] = (uint32_t)lfo_off;
    c[CHC_PS_INC] = (uint32_t)(ps_inc >> 32);
    c[CHC_PS_INC_LO] = (uint32_t)ps_inc;
    // D = mstosamps (:3897) as a double; W = mstosamps(window) in 32.32 fixed point (spec v2,
    // olfx_internal.h pitch_split / chorus_split)
    const double D = depth_ms * sr / 1000.0;
    uint64_t Dbits;
    std::memcpy(&Dbits, &D, 8);
    c[CHC_DEPTH] = (uint32_t)(Dbits >> 32);
    c[CHC_DEPTH_LO] = (uint32_t)Dbits;
    const uint64_t Wfix = (uint64_t)std::floor(window * sr / 1000.0 * 4294967296.0 + 0.5);
    c[CHC_WINDOW] = (uint32_t)(Wfix >> 32);
    c[CHC_WINDOW_LO] = (uint32_t)Wfix;
    // lores~ -> RBJ biquad low-pass, Q = 1/sqrt(2) + 20 q^3 (declared)
    const double Q = 0.70710678118654752 + 20.0 * q * q * q;
    const double w0 = 2.0 * 3.14159265358979323846 * fc / sr;
    const double cw = std::cos(w0), sw = std::sin(w0);
    const double alpha = sw / (2.0 * Q);
    const double a0 = 1.0 + alpha;
    c[CHC_B0] = as_u32((float)((1.0 - cw) * 0.5 / a0));
    c[CHC_B1] = as_u32((float)((1.0 - cw) / a0));
    c[CHC_B2] = as_u32((float)((1.0 - cw) * 0.5 / a0));
    c[CHC_A1] = as_u32((float)(-2.0 * cw / a0));
    c[CHC_A2] = as_u32((float)((1.0 - alpha) / a0));
    const float mixf = (float)mix;
    c[CHC_MIX] = as_u32(mixf);
    c[CHC_DRY] = as_u32(1.0f - mixf);                             // !- 1 (:1176)
}

// pitch-shift stage only: reuse the chorus coefficient block (mode 1 ignores the rest)
void derive_pitchshift(const float *p, double sr, uint32_t *c) {
    float cp[OLFX_CH_NPARAMS];
    default_params(OLFX_KIND_CHORUS, cp);
    cp[OLFX_CH_PITCH] = p[OLFX_PS_SHIFT];
    cp[OLFX_CH_WINDOW] = p[OLFX_PS_WINDOW];
    derive_chorus(cp, sr, c);
}

// DaisySP Adsr coefficient setters (restated; DaisySP is absent from the reference tree, see
// DESIGN.md "parity unpinned"): SetAttackTime / SetTimeConstant.
float adsr_attack_d0(float T, float shape, float sr, float *target_out) {
    float target = 9.f * powf(shape, 10.f) + 0.3f * shape + 1.01f;
    *target_out = target;
    if (T > 0.f) {
        float logTarget = logf(1.f - (1.f / target));
        return 1.f - expf(logTarget / (T * sr));
    }
    return 1.f;
}
float adsr_time_d0(float T, float sr) {
    if (T > 0.f) {
        const float target = logf((float)(1. / M_E));
        return 1.f - expf(target / (T * sr));
    }
    return 1.f;
}
float adsr_sustain(float s) { return (s <= 0.f) ? -0.01f : (s > 1.f ? 1.f : s); }

// Voice: `configured` = false reproduces SynthVoice::Init without any Update()
// (SynthVoice.h:31-39): DaisySP Init defaults in the envelopes and the Svf.
// FxRack<2> (modules/fxlib/Fx.h:398-492): DelayLine::SetDelay(scale(time, 0,1, 0,48000, 1)),
// and FilterFx::Update = Svf SetFreq, SetRes, SetDrive (DaisySP restated, as oracle/fxrack_ref.c)
void svf_coef(float cutoff, float res_in, float drive_in, float sr, float *freq, float *damp, float *drive) {
    const float fc = clampf(cutoff, 1.0e-6f, sr / 3.f);
    const float f = 2.0f * sinf(3.1415927410125732f * std::min(0.25f, fc / (sr * 2.0f)));
    const float res = clampf(res_in, 0.f, 1.f);
    *freq = f;
    *damp = std::min(2.0f * (1.0f - powf(res, 0.25f)), std::min(2.0f, 2.0f / f - f * 0.5f));
    *drive = clampf(drive_in * 0.1f, 0.f, 1.f) * res;
}

void derive_fxrack(const float *p, float sr, uint32_t *c) {
    auto put = [&](int k, float v) { std::memcpy(&c[k], &v, 4); };
    const float dly = core_scale(p[OLFX_FR_DELAY_TIME], 0.f, 1.f, 0.f, (float)kFrMaxDelay, 1.f);
    const int32_t id = (int32_t)dly;
    c[FRC_DELAY] = (uint32_t)id < kFrMaxDelay ? (uint32_t)id : kFrMaxDelay - 1;
    put(FRC_FRAC, dly - (float)id);
    put(FRC_FEEDBACK, p[OLFX_FR_DELAY_FEEDBACK]);
    put(FRC_DBAL, p[OLFX_FR_DELAY_BALANCE]);
    float f, d, dr;
    svf_coef(p[OLFX_FR_DELAY_CUTOFF], p[OLFX_FR_DELAY_RESONANCE], 0.f, sr, &f, &d, &dr);
    put(FRC_DFREQ, f); put(FRC_DDAMP, d); put(FRC_DDRIVE, dr);
    put(FRC_RBAL, p[OLFX_FR_REVERB_BALANCE]);
    svf_coef(p[OLFX_FR_FILTER_CUTOFF], p[OLFX_FR_FILTER_RESONANCE], p[OLFX_FR_FILTER_DRIVE], sr, &f, &d, &dr);
    put(FRC_FFREQ, f); put(FRC_FDAMP, d); put(FRC_FDRIVE, dr);
    c[FRC_FTYPE] = (uint32_t)(int32_t)p[OLFX_FR_FILTER_TYPE];
    const uint32_t topo = (uint32_t)p[OLFX_FR_TOPOLOGY];     // 0..4 (validated by olfx_set_params)
    c[FRC_TOPO] = topo;
    put(FRC_MASTER, topo ? 1.0f : p[OLFX_FR_MASTER_VOLUME]);   // x 1.0f is exact: no FxRack, no master
}

void derive_voice(const float *p, bool configured, bool moog, float sr, float *c) {
    float tgt;
    if (!configured) {
        // daisysp::Adsr::Init: attack 0.1 s shape 0, decay 0.1 s, release 0.1 s, sustain 0.7
        c[VCC_ATK_D0A] = adsr_attack_d0(0.1f, 0.0f, sr, &tgt); c[VCC_ATK_TGT_A] = tgt;
        c[VCC_DEC_D0A] = adsr_time_d0(0.1f, sr);
        c[VCC_REL_D0A] = adsr_time_d0(0.1f, sr);
        c[VCC_SUS_A] = 0.7f;
        c[VCC_ATK_D0F] = c[VCC_ATK_D0A]; c[VCC_ATK_TGT_F] = tgt;
        c[VCC_DEC_D0F] = c[VCC_DEC_D0A];
        c[VCC_REL_D0F] = c[VCC_REL_D0A];
        c[VCC_SUS_F] = 0.7f;
        // daisysp::Svf::Init: res 0.5, drive 0.5
        c[VCC_DAMP_RES] = 2.0f * (1.0f - powf(0.5f, 0.25f));
        c[VCC_DRIVE] = 0.5f;
    } else {
        c[VCC_ATK_D0A] = adsr_attack_d0(p[OLFX_VC_AMP_ATTACK], p[OLFX_VC_AMP_ATTACK_SHAPE], sr, &tgt);
        c[VCC_ATK_TGT_A] = tgt;
        c[VCC_DEC_D0A] = adsr_time_d0(p[OLFX_VC_AMP_DECAY], sr);
        c[VCC_REL_D0A] = adsr_time_d0(p[OLFX_VC_AMP_RELEASE], sr);
        c[VCC_SUS_A] = adsr_sustain(p[OLFX_VC_AMP_SUSTAIN]);
        c[VCC_ATK_D0F] = adsr_attack_d0(p[OLFX_VC_FILTER_ATTACK], p[OLFX_VC_FILTER_ATTACK_SHAPE], sr, &tgt);
        c[VCC_ATK_TGT_F] = tgt;
        c[VCC_DEC_D0F] = adsr_time_d0(p[OLFX_VC_FILTER_DECAY], sr);
        c[VCC_REL_D0F] = adsr_time_d0(p[OLFX_VC_FILTER_RELEASE], sr);
        c[VCC_SUS_F] = adsr_sustain(p[OLFX_VC_FILTER_SUSTAIN]);
        // Svf::SetRes then Svf::SetDrive (SynthVoice::Update, SynthVoice.h:82-83)
        float res = fminf(fmaxf(p[OLFX_VC_FILTER_RESONANCE], 0.f), 1.f);
        float pre_drive = fminf(fmaxf(p[OLFX_VC_FILTER_DRIVE] * 0.1f, 0.f), 1.f);
        c[VCC_DAMP_RES] = 2.0f * (1.0f - powf(res, 0.25f));
        c[VCC_DRIVE] = pre_drive * res;
    }
    c[VCC_AMP_AMT] = p[OLFX_VC_AMP_ENV_AMOUNT];
    c[VCC_CUTOFF] = p[OLFX_VC_FILTER_CUTOFF];
    c[VCC_FENV_AMT] = p[OLFX_VC_FILTER_ENV_AMOUNT];
    // daisysp::Port (in-tree stub, Portamento.h:223-226): SynthVoice::Init passes the member
    // portamento_htime (SynthVoice.h:37), Update SetHtime(portamento_htime): either way the member
    float htime = p[OLFX_VC_PORTAMENTO];
    c[VCC_PORT_COEF] = expf(-1.0f / (htime * sr));
    c[VCC_FC_MAX] = sr / 3.f;
    c[VCC_SR] = sr;
    c[VCC_INV_SR] = 1.0f / sr;
    if (moog) {
        // daisysp::LadderFilter: Init -> SetRes(0.2), SetInputDrive(0.5) (drive <= 1: drive_scaled =
        // drive), sr_int_recip_ = 1 / (sr * 4); Update -> MoogFilter::SetRes -> SetRes(res):
        // K = 4 * clamp(res, 0, kMaxResonance 1.8); MoogFilter::SetDrive is a no-op
        const float res = configured ? p[OLFX_VC_FILTER_RESONANCE] : 0.2f;
        c[VCC_LADDER_K] = 4.0f * fminf(fmaxf(res, 0.0f), 1.8f);
        c[VCC_LADDER_DRIVE] = 0.5f;
        c[VCC_LADDER_WREC] = 1.0f / (sr * 4);
    }
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Engine
// ---------------------------------------------------------------------------------------------
struct olfx_engine {
    int kind = 0;
    int device = 0;
    uint32_t n = 0;
    uint32_t block = 0;
    float sr = 48000.f;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;    // copies of large control packets
    uint64_t frames = 0;
    std::string err;

    // user parameters [n_params][n] (host shadow) and device coefficient blocks
    uint32_t n_params = 0;
    std::vector<float> params;
    std::vector<uint8_t> configured;     // voice: UpdateConfig seen
    // instances whose coefficients must be re-derived at the next block (each listed once)
    std::vector<uint32_t> dirty_list;
    std::vector<uint8_t> dirty_mark;
    int cus = 0;                          // compute units (the chain's persistent grid)
    int64_t n_components = 0;             // rack instances with OLFX_FR_TOPOLOGY >= 2

    // control packets: a block's changed coefficients and folded note events, in pinned host
    // slots the block's kernels read (submit_control).  A slot is rewritten only after the
    // kernels that read it are done (consumed).
    // 16 slots in groups of 4: one `consumed` marker per group (each marker is a command-processor
    // packet between two blocks' kernels), recorded after the group's last packet or when the
    // caller switches streams; a slot's guard is its group's marker
    static constexpr int kSlots = 16, kGroup = 4, kBig = 2;
    static constexpr size_t kCopyBytes = 64 * 1024;   // packets from this size on are copied
    size_t copy_bytes = kCopyBytes;                  // OLFX_COPY_BYTES overrides (A/B diagnostic)
    struct Slot {
        uint32_t *h = nullptr, *hd = nullptr;   // pinned host half and its device address
        uint32_t *d = nullptr;                  // device half (large packets), allocated on first need
        size_t cap = 0, dcap = 0;               // words
        hipEvent_t copied = nullptr, consumed = nullptr;
        hipEvent_t guard = nullptr;             // the marker after this slot's last readers
        bool used = false;
    } slot[kSlots], big[kBig];                  // small packets (zero-copy) / large ones (copied)
    int slot_next = 0, big_next = 0;
    template <class F>
    void each_slot(F &&f) {
        for (Slot &x : slot) f(x);
        for (Slot &x : big) f(x);
    }
    int pending[kGroup] = {};                   // slots used since the last marker, all on pending_stream
    int n_pending = 0;
    hipStream_t pending_stream = nullptr;
    // the stream of the engine's latest launch (olfx_process / olfx_mix): what reset, sync and
    // destroy wait for (engine-scoped; the caller keeps that stream alive until then, olfx.h).  A
    // block on another stream is ordered after it through `switched` (recorded on the old stream at
    // the switch only: an event per block would cost a command-processor packet per block)
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    hipEvent_t switched = nullptr;
    std::vector<int32_t> ev_slot;         // voice -> its record in `folded` during fold_events, else -1
    struct Folded { uint32_t inst, op, freq, pad; };
    std::vector<Folded> folded;
    // per workgroup: records, first overflow record (crowded groups), records written so far
    std::vector<uint32_t> ev_count, ev_more, ev_fill;
    uint32_t n_more = 0;                  // overflow records
    std::vector<uint32_t> h_words;        // scratch for a record
    // OLFX_TRACE_CONTROL=1 (read at create): host time of each control-path step, summed and
    // printed to stderr at destroy (tracing)
    bool trace = false;
    double tr[6] = {0, 0, 0, 0, 0, 0};
    uint64_t tr_calls = 0;

    // device memory: one allocation per engine, carved
    void *d_mem = nullptr;
    size_t d_bytes = 0;

    // dattorro (also the chain's reverb stage)
    // fx rack
    float *fr_ring = nullptr;
    uint32_t *fr_state = nullptr, *fr_coef = nullptr;
    uint32_t n_dt = 0;           // reverb-stage instances: n, or n rounded up to 64 for the chain
    float *dt_rings = nullptr;
    // standalone reverb: the network (dattorro.hip dattorro_rows) and so its pre-delay ring's layout
    float *dt_pre_tmp = nullptr; // a copy of the pre-delay ring while its layout changes
    int dt_net = DT_NET_V4;      // the network of the last block; its pre-delay ring layout: rows unless v4
    bool dt_pre_check = true;    // a pre-delay changed: re-decide the network at the next block
    float *dt_state = nullptr;
    float *dt_coef = nullptr;

    // chorus / pitch-shift (also the chain's first two stages)
    uint32_t psize = 0, csize = 0;
    float *ch_pring = nullptr, *ch_cring = nullptr;
    uint32_t *ch_state = nullptr, *ch_coef = nullptr;
    float *ps_pring = nullptr, *ps_cring = nullptr;      // chain stage 2
    uint32_t *ps_state = nullptr, *ps_coef = nullptr;

    // voice
    float *vc_state = nullptr, *vc_coef = nullptr;
    std::vector<olfx_voice_event> events;
    // voice buses (olfx_mix_config): [n_buses + 1] offsets, then the voice lists
    uint32_t *mix_dev = nullptr;
    uint32_t mix_quad = 0;                  // contiguous buses on multiples of 4 voices (voice_mix_v4)
    hipEvent_t mix_done = nullptr;          // recorded after every olfx_mix launch
    uint32_t n_buses = 0;

    // host-pointer I/O staging
    float *h_in = nullptr, *h_out = nullptr, *d_in = nullptr, *d_out = nullptr;
    size_t stage_floats_in = 0, stage_floats_out = 0;
    // device staging of frame tiles whose channel planes are too far apart for the kernels'
    // 32-bit buffer offsets (olfx_process on > 4 GiB planes), allocated on first need
    float *tile_in = nullptr, *tile_out = nullptr;
    size_t tile_floats = 0;

    int fail(int code, const char *fmt, ...) {
        char buf[512];
        va_list ap;
        va_start(ap, fmt);
        vsnprintf(buf, sizeof buf, fmt, ap);
        va_end(ap);
        err = buf;
        set_global_error("%s", buf);
        return code;
    }
    int hip_fail(hipError_t e, const char *what) {
        return fail(OLFX_E_HIP, "%s: %s", what, hipGetErrorString(e));
    }
};

#define HIPCHK(e, call)                                          \
    do {                                                         \
        hipError_t _r = (call);                                  \
        if (_r != hipSuccess) return (e)->hip_fail(_r, #call);   \
    } while (0)

namespace {

size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Carve {
    size_t off = 0;
    size_t take(size_t bytes) {
        size_t o = off;
        off = align_up(off + bytes, 256);
        return o;
    }
};

void chorus_sizes(float sr, uint32_t *psize, uint32_t *csize) {
    // pitch ring: delays up to W = 10 ms plus the interpolation neighbour
    *psize = pow2_at_least((uint32_t)std::ceil(10.0 * sr / 1000.0) + 2);
    // chorus ring: delays up to 2 D, D <= 12 ms (delay~ @maxsize samplerate*2 is never reached)
    *csize = pow2_at_least(2u * (uint32_t)std::ceil(12.0 * sr / 1000.0) + 2);
}

uint64_t state_bytes(int kind, uint32_t n, float sr) {
    uint32_t ps, cs;
    chorus_sizes(sr, &ps, &cs);
    const uint64_t dt = (uint64_t)dt_total_floats() * 4 + DTS_N * 4 + DTC_N * 4;
    const uint64_t ch = (uint64_t)2 * (ps + cs) * 4 + CHS_N * 4 + CHC_N * 4;
    const uint64_t vc = (uint64_t)VCS_N * 4 + VCC_N * 4;
    switch (kind) {
    case OLFX_KIND_DATTORRO: return dt * n;
    case OLFX_KIND_CHORUS:
    case OLFX_KIND_PITCHSHIFT: return ch * n;
    case OLFX_KIND_VOICE: return vc * n;
    case OLFX_KIND_VOICE_MOOG: return vc * n + (uint64_t)(VCS_N_MOOG - VCS_N) * 4 * n;
    case OLFX_KIND_CHAIN: return (dt + 2 * ch) * n;
    case OLFX_KIND_FXRACK: return ((uint64_t)kFrMaxDelay * 2 * 4 + FRS_N * 4 + FRC_N * 4) * n;
    default: return 0;
    }
}

// ---------------------------------------------------------------------------------------------
// Control path (parameters and note events at the block boundary; JUCE-host pattern,
// modules/juce/host/host.cpp:646-653): O(changed), asynchronous, no host<->device round trip.
// ---------------------------------------------------------------------------------------------

// Coefficient words per instance and their destination arrays (field-major, CoefScatterArgs).
uint32_t coef_segments(const olfx_engine *e, CoefScatterArgs *a) {
    auto seg = [&](void *dst, uint32_t words, uint32_t stride) {
        a->dst[a->nseg] = (uint32_t *)dst;
        a->words[a->nseg] = words;
        a->stride[a->nseg] = stride;
        ++a->nseg;
    };
    a->nseg = 0;
    switch (e->kind) {
    case OLFX_KIND_DATTORRO: seg(e->dt_coef, DTC_N, e->n_dt); break;
    case OLFX_KIND_CHORUS:
    case OLFX_KIND_PITCHSHIFT: seg(e->ch_coef, CHC_N, e->n); break;
    case OLFX_KIND_CHAIN:       // padding reverb instances keep their zeroed coefficients
        seg(e->ch_coef, CHC_N, e->n);
        seg(e->ps_coef, CHC_N, e->n);
        seg(e->dt_coef, DTC_N, e->n_dt);
        break;
    case OLFX_KIND_FXRACK: seg(e->fr_coef, FRC_N, e->n); break;
    case OLFX_KIND_VOICE:
    case OLFX_KIND_VOICE_MOOG: seg(e->vc_coef, VCC_N, e->n); break;
    default: break;
    }
    uint32_t w = 0;
    for (uint32_t k = 0; k < a->nseg; ++k) w += a->words[k];
    return w;
}

// The coefficient record of instance i from its current parameters (the reference setters'
// arithmetic, derive_*), in the word order of coef_segments.
void derive_record(olfx_engine *e, uint32_t i, uint32_t *w) {
    const uint32_t n = e->n, np = e->n_params;
    float p[OLFX_CN_NPARAMS > OLFX_VC_NPARAMS ? OLFX_CN_NPARAMS : OLFX_VC_NPARAMS];
    for (uint32_t f = 0; f < np; ++f) p[f] = e->params[(size_t)f * n + i];
    float fc[VCC_N > DTC_N ? VCC_N : DTC_N];
    switch (e->kind) {
    case OLFX_KIND_DATTORRO:
        derive_dattorro(p, fc);
        std::memcpy(w, fc, DTC_N * 4);
        break;
    case OLFX_KIND_CHORUS: derive_chorus(p, e->sr, w); break;
    case OLFX_KIND_PITCHSHIFT: derive_pitchshift(p, e->sr, w); break;
    case OLFX_KIND_CHAIN:
        derive_chorus(p + OLFX_CN_CHORUS0, e->sr, w);
        derive_pitchshift(p + OLFX_CN_PITCH0, e->sr, w + CHC_N);
        derive_dattorro(p + OLFX_CN_VERB0, fc);
        std::memcpy(w + 2 * CHC_N, fc, DTC_N * 4);
        break;
    case OLFX_KIND_FXRACK: derive_fxrack(p, e->sr, w); break;
    case OLFX_KIND_VOICE:
    case OLFX_KIND_VOICE_MOOG:
        derive_voice(p, e->configured[i] != 0, e->kind == OLFX_KIND_VOICE_MOOG, e->sr, fc);
        std::memcpy(w, fc, VCC_N * 4);
        break;
    default: break;
    }
}

void mark_dirty(olfx_engine *e, uint32_t first, uint32_t count) {
    for (uint32_t k = first; k < first + count; ++k)
        if (!e->dirty_mark[k]) {
            e->dirty_mark[k] = 1;
            e->dirty_list.push_back(k);
        }
}

// The block's note events, one record per voice, in voice order (VEV_*, olfx_internal.h).
// Calls on one voice compose field by field, as their in-order application does
// (SynthVoice.h:231-268): NoteOn = GateOn + freq_ = mtof(note) + Retrigger(true) on both
// envelopes (:245-251); NoteOff / GateOff = gate off (:236-239, :253-256); GateOn = gate on
// (:231-234); SetFrequency = freq_ (:264-267).  The last gate call decides the gate, any NoteOn
// retriggers (gate calls do not touch the envelope modes), the last NoteOn / SetFrequency the pitch.
// daisysp::mtof of a MIDI note, from a table of the same expression (notes are 0..127; one powf
// per NoteOn had been the largest host cost of a block with note events)
float mtof_note(uint8_t note) {
    static const std::array<float, 128> t = [] {
        std::array<float, 128> r{};
        for (int k = 0; k < 128; ++k) r[(size_t)k] = powf(2.f, ((float)k - 69.0f) / 12.0f) * 440.0f;
        return r;
    }();
    return t[note & 127u];
}

void fold_events(olfx_engine *e) {
    e->folded.clear();
    for (const olfx_voice_event &ev : e->events) {
        int32_t &k = e->ev_slot[ev.inst];
        if (k < 0) {
            k = (int32_t)e->folded.size();
            e->folded.push_back(olfx_engine::Folded{ev.inst, 0u, 0u, 0u});
        }
        olfx_engine::Folded &r = e->folded[(size_t)k];
        switch (ev.type) {
        case OLFX_EV_NOTE_ON: {
            r.op |= VEV_GATE_SET | VEV_GATE_ON | VEV_RETRIGGER | VEV_FREQ;
            const float hz = mtof_note(ev.note);                              // daisysp::mtof
            std::memcpy(&r.freq, &hz, 4);
            break;
        }
        case OLFX_EV_GATE_ON: r.op |= VEV_GATE_SET | VEV_GATE_ON; break;
        case OLFX_EV_SET_FREQUENCY:
            r.op |= VEV_FREQ;
            std::memcpy(&r.freq, &ev.value, 4);
            break;
        default: r.op = (r.op | VEV_GATE_SET) & ~VEV_GATE_ON; break;   // NoteOff / GateOff
        }
    }
    e->events.clear();
    // records per workgroup (64 voices); crowded workgroups (more than kVevCap records) get a run
    // of the overflow list each, in group order
    const uint32_t groups = (e->n + 63u) / 64u;
    e->ev_count.assign(groups, 0u);
    for (const olfx_engine::Folded &r : e->folded) {
        e->ev_count[r.inst >> 6]++;
        e->ev_slot[r.inst] = -1;
    }
    e->ev_more.assign(groups, 0u);
    e->n_more = 0;
    for (uint32_t g = 0; g < groups; ++g)
        if (e->ev_count[g] > kVevCap) {
            e->ev_more[g] = e->n_more;
            e->n_more += e->ev_count[g];
        }
}

// The folded records into a packet's event section (VoiceArgs::ev layout, olfx_internal.h):
// `fix` = [groups][kVevCap] 8-B slots, then the overflow list.
void write_events(olfx_engine *e, uint32_t *fix) {
    const uint32_t groups = (e->n + 63u) / 64u;
    std::memset(fix, 0, (size_t)groups * kVevCap * 8);
    uint32_t *more = fix + (size_t)groups * kVevCap * 2;
    e->ev_fill.assign(groups, 0u);
    for (const olfx_engine::Folded &r : e->folded) {
        const uint32_t g = r.inst >> 6;
        const uint32_t k = e->ev_fill[g]++;
        uint32_t *rec = e->ev_count[g] <= kVevCap ? fix + 2 * ((size_t)g * kVevCap + k) : more + 2 * ((size_t)e->ev_more[g] + k);
        rec[0] = (r.inst & 63u) | r.op << 8;
        rec[1] = r.freq;
    }
    for (uint32_t g = 0; g < groups; ++g)
        if (e->ev_count[g] > kVevCap) {
            fix[2 * (size_t)g * kVevCap] = VEV_MORE << 8 | e->ev_count[g] << 16;
            fix[2 * (size_t)g * kVevCap + 1] = e->ev_more[g];
        }
}

// Record one marker after the pending slots' kernels (on their stream) and make it their guard.
hipError_t flush_markers(olfx_engine *e) {
    if (!e->n_pending) return hipSuccess;
    hipEvent_t m = e->slot[e->pending[e->n_pending - 1]].consumed;
    const hipError_t r = hipEventRecord(m, e->pending_stream);
    for (int k = 0; k < e->n_pending; ++k) e->slot[e->pending[k]].guard = r == hipSuccess ? m : nullptr;
    e->n_pending = 0;
    return r;
}

// A block's kernels that read slot `sl` are queued on `s`: a big slot gets its own marker, a small
// one joins the pending group.
hipError_t slot_queued(olfx_engine *e, olfx_engine::Slot *sl, hipStream_t s) {
    if (sl >= e->big && sl < e->big + olfx_engine::kBig) {
        const hipError_t r = hipEventRecord(sl->consumed, s);
        sl->guard = r == hipSuccess ? sl->consumed : nullptr;
        return r;
    }
    hipError_t r = hipSuccess;
    if (e->n_pending && e->pending_stream != s) r = flush_markers(e);
    e->pending[e->n_pending++] = (int)(sl - e->slot);
    e->pending_stream = s;
    if (e->n_pending == olfx_engine::kGroup) {
        const hipError_t r2 = flush_markers(e);
        if (r == hipSuccess) r = r2;
    }
    return r;
}

// A slot's pinned half (and, for copied packets, its device half) of at least `words` words.
int grow_slot(olfx_engine *e, olfx_engine::Slot &sl, size_t words, bool device_half) {
    if (sl.cap < words) {
        if (sl.h) (void)hipHostFree(sl.h);
        sl.h = nullptr; sl.hd = nullptr; sl.cap = 0;
        const size_t cap = std::max<size_t>(words, 4096);
        // zero-copy slots (read by the kernels over the host link, rewritten 16 blocks later) are
        // coherent: no GPU cache may hold a stale line of them whatever HIP_HOST_COHERENT says;
        // copied slots are only a copy source
        HIPCHK(e, hipHostMalloc((void **)&sl.h, cap * 4,
                                device_half ? hipHostMallocDefault : (hipHostMallocMapped | hipHostMallocCoherent)));
        void *dp = nullptr;
        HIPCHK(e, hipHostGetDevicePointer(&dp, sl.h, 0));
        sl.hd = (uint32_t *)dp;
        sl.cap = cap;
    }
    if (device_half && sl.dcap < sl.cap) {
        if (sl.d) (void)hipFree(sl.d);
        sl.d = nullptr; sl.dcap = 0;
        HIPCHK(e, hipMalloc((void **)&sl.d, sl.cap * 4));
        sl.dcap = sl.cap;
    }
    return OLFX_OK;
}

// The largest control packet an engine can produce: every instance's coefficients and, for voices,
// an event for every voice (submit_control's layout, rounded up).
size_t max_packet_words(const olfx_engine *e) {
    CoefScatterArgs ca{};
    const size_t n = e->n, W = coef_segments(e, &ca);
    const size_t ev = is_voice_kind(e->kind) ? 2 * ((n + 63) / 64 * kVevCap + n) : 0;
    return n + W * n + ev + 16;
}

// This block's control packet -- the changed instances' coefficient records and the folded note
// events -- in a pinned host slot that the block's kernels read directly over the host link
// (zero-copy: no copy command, no second stream, no host wait on the device).  The coefficients are
// scattered on `s` ahead of the block's kernel; the voice kernel reads its events itself.  A slot is
// rewritten only after the kernels that read it are done (its `consumed` event, recorded by the
// caller after them: *used_slot).  Packet layout (u32 words, 16-B aligned sections): instance list
// (absent when every instance changed) | coefficient records [W][m] | event slots [groups][kVevCap]
// and the overflow list, 8-B records (write_events).
int submit_control(olfx_engine *e, hipStream_t s, VoiceArgs *va, olfx_engine::Slot **used_slot) {
    *used_slot = nullptr;
    const bool voice = is_voice_kind(e->kind);
    const size_t m = e->dirty_list.size();
    if (!m && !(voice && !e->events.empty())) return OLFX_OK;
    using clk = std::chrono::steady_clock;
    auto t_prev = clk::now();
    auto lap = [&](int k) {
        if (!e->trace) return;
        const auto t = clk::now();
        e->tr[k] += std::chrono::duration<double, std::micro>(t - t_prev).count();
        t_prev = t;
    };
    e->tr_calls++;
    const bool evs = voice && !e->events.empty();
    if (evs) fold_events(e);
    lap(0);
    CoefScatterArgs ca{};
    const uint32_t W = coef_segments(e, &ca);
    const bool dense = m == e->n;                        // every instance: no instance list
    const uint32_t groups = (e->n + 63u) / 64u;
    auto up4 = [](size_t x) { return (x + 3) & ~(size_t)3; };
    const size_t o_inst = 0;
    const size_t o_val = o_inst + (dense ? 0 : up4(m));
    const size_t o_ev = up4(o_val + (size_t)W * m);
    const size_t words = o_ev + (evs ? 2 * ((size_t)groups * kVevCap + e->n_more) : 0);

    // Delivery: a small packet (a block's CCs / notes) is read by the kernels straight from a pinned
    // slot -- no copy command: ~2 us of host time, a host-link round trip or two inside the kernel.
    // A large one (the first block's full upload, an all-voices note-off) goes to one of two big
    // slots and is copied into its device half on the engine's copy stream, which the caller's
    // stream waits for: ~20 us of host API time, but no 512-KB read over the host link on the
    // kernel's critical path.
    const bool copy = words * 4 >= e->copy_bytes;
    olfx_engine::Slot &sl = copy ? e->big[e->big_next] : e->slot[e->slot_next];
    if (copy) e->big_next = (e->big_next + 1) % olfx_engine::kBig;
    else e->slot_next = (e->slot_next + 1) % olfx_engine::kSlots;
    // the slot is free once the kernels that read it are done (both halves)
    if (sl.used) {
        if (!sl.guard) HIPCHK(e, flush_markers(e));
        if (sl.guard) HIPCHK(e, hipEventSynchronize(sl.guard));
        else HIPCHK(e, hipDeviceSynchronize());     // its marker failed to record: wait for everything
    }
    lap(1);
    if (const int rc = grow_slot(e, sl, words, copy)) return rc;
    uint32_t *const dev = copy ? sl.d : sl.hd;      // what the kernels read
    lap(2);
    // coefficient records, field-major [W][m]
    uint32_t *val = sl.h + o_val;
    e->h_words.resize(W);
    for (size_t r = 0; r < m; ++r) {
        const uint32_t i = dense ? (uint32_t)r : e->dirty_list[r];
        if (!dense) sl.h[o_inst + r] = i;
        derive_record(e, i, e->h_words.data());
        for (uint32_t w = 0; w < W; ++w) val[(size_t)w * m + r] = e->h_words[w];
    }
    for (const uint32_t i : e->dirty_list) e->dirty_mark[i] = 0;
    e->dirty_list.clear();
    lap(3);
    if (evs) write_events(e, sl.h + o_ev);
    if (copy) {
        // the copy stream waits for nothing on the device: the host made sure above that the slot's
        // previous readers are done (a device-side wait there serialised the copy behind them)
        HIPCHK(e, hipMemcpyAsync(sl.d, sl.h, words * 4, hipMemcpyHostToDevice, e->copy_stream));
        HIPCHK(e, hipEventRecord(sl.copied, e->copy_stream));
        HIPCHK(e, hipStreamWaitEvent(s, sl.copied, 0));
    } else {
        std::atomic_thread_fence(std::memory_order_seq_cst);     // the packet's stores before the launch
    }
    sl.used = true;
    sl.guard = nullptr;
    *used_slot = &sl;
    lap(4);
    if (m) {
        ca.inst = dense ? nullptr : dev + o_inst;
        ca.val = dev + o_val;
        ca.m = (uint32_t)m;
        ca.W = W;
        const hipError_t r = launch_coef_scatter(ca, s);
        if (r != hipSuccess) return e->hip_fail(r, "coefficient scatter launch");
    }
    if (evs) {
        va->ev = reinterpret_cast<const uint2 *>(dev + o_ev);
        va->ev_more = va->ev + (size_t)groups * kVevCap;
    }
    lap(5);
    return OLFX_OK;
}

// Wait for this engine's queued work only -- not the device: its latest launch stream (the caller
// orders its own streams, so that covers every earlier block), its own stream, and every control
// slot's marker.  A slot whose marker failed to record falls back to a device-wide wait.
int wait_engine(olfx_engine *e) {
    HIPCHK(e, flush_markers(e));
    bool unmarked = false;
    e->each_slot([&](olfx_engine::Slot &sl) {
        if (!sl.used) return;
        if (sl.guard) {
            if (hipEventSynchronize(sl.guard) != hipSuccess) unmarked = true;
        } else {
            unmarked = true;
        }
        if (sl.d && sl.copied && hipEventSynchronize(sl.copied) != hipSuccess) unmarked = true;
    });
    if (e->mix_done) HIPCHK(e, hipEventSynchronize(e->mix_done));
    if (e->have_last) HIPCHK(e, hipStreamSynchronize(e->last_stream));
    if (e->stream) HIPCHK(e, hipStreamSynchronize(e->stream));
    if (e->copy_stream) HIPCHK(e, hipStreamSynchronize(e->copy_stream));
    if (unmarked) HIPCHK(e, hipDeviceSynchronize());
    return OLFX_OK;
}

// Every instance back to the freshly created state.  The caller has made sure that none of the
// engine's work is still queued (olfx_create: none was; olfx_reset: wait_engine).
int init_state(olfx_engine *e) {
    e->n_pending = 0;
    e->each_slot([](olfx_engine::Slot &sl) { sl.used = false; sl.guard = nullptr; });
    HIPCHK(e, hipMemsetAsync(e->d_mem, 0, e->d_bytes, e->stream));
    // voices: daisysp Oscillator::Init phase 0; Svf::Init states 0; Adsr idle; freq_ = 0
    // (SynthVoice.h:276); Port z1 = 0 -- all zeros
    HIPCHK(e, hipStreamSynchronize(e->stream));
    e->params.assign((size_t)e->n_params * e->n, 0.f);
    std::vector<float> d(e->n_params);
    default_params(e->kind, d.data());
    for (uint32_t f = 0; f < e->n_params; ++f)
        std::fill(e->params.begin() + (size_t)f * e->n, e->params.begin() + (size_t)(f + 1) * e->n, d[f]);
    e->configured.assign(e->n, 0);
    e->n_components = 0;
    e->dt_net = DT_NET_V4;         // the zeroed ring is valid in either layout: decided at the next block
    e->dt_pre_check = true;
    e->events.clear();
    e->ev_slot.assign(e->n, -1);
    e->frames = 0;
    e->dirty_list.clear();
    e->dirty_mark.assign(e->n, 0);
    mark_dirty(e, 0, e->n);                  // every coefficient is derived at the first block
    return OLFX_OK;
}

int ensure_staging(olfx_engine *e, size_t fin, size_t fout) {
    if (fin > e->stage_floats_in) {
        if (e->h_in) (void)hipHostFree(e->h_in);
        if (e->d_in) (void)hipFree(e->d_in);
        e->h_in = nullptr; e->d_in = nullptr;
        HIPCHK(e, hipHostMalloc((void **)&e->h_in, fin * 4, hipHostMallocDefault));
        HIPCHK(e, hipMalloc((void **)&e->d_in, fin * 4));
        e->stage_floats_in = fin;
    }
    if (fout > e->stage_floats_out) {
        if (e->h_out) (void)hipHostFree(e->h_out);
        if (e->d_out) (void)hipFree(e->d_out);
        e->h_out = nullptr; e->d_out = nullptr;
        HIPCHK(e, hipHostMalloc((void **)&e->h_out, fout * 4, hipHostMallocDefault));
        HIPCHK(e, hipMalloc((void **)&e->d_out, fout * 4));
        e->stage_floats_out = fout;
    }
    return OLFX_OK;
}


// One launch over frames [e->frames, e->frames + n_frames) of every instance: in / out hold those
// frames with channel planes `plane` floats apart.  `ev` carries the block's note events (voices).
int launch(olfx_engine *e, const float *din, float *dout, uint32_t n_frames, uint64_t plane, hipStream_t s,
           const VoiceArgs &ev) {
    hipError_t r = hipSuccess;
    const uint32_t t0 = (uint32_t)(e->frames & 0xFFFFFFFFu);
    auto dt_args = [&](const float *in, float *out) {
        DattorroArgs a{};
        size_t off = 0;
        for (int l = 0; l < DT_NLINES; ++l) {
            a.ring[l] = e->dt_rings + off;
            off += (size_t)kDtSize[l] * e->n_dt;
        }
        a.state = e->dt_state;
        a.coef = e->dt_coef;
        a.in = in;
        a.out = out;
        a.plane = plane;
        a.n = e->n_dt;
        a.n_frames = n_frames;
        a.t0 = t0 & 0xFFFFu;
        a.in_ch = 2;
        a.cus = (uint32_t)e->cus;
        return a;
    };
    auto ch_args = [&](float *pr, float *cr, uint32_t *st, const uint32_t *cf, const float *in,
                       float *out, uint32_t mode) {
        ChorusArgs a{};
        a.pitch_ring = pr;
        a.chorus_ring = cr;
        a.state = st;
        a.coef = cf;
        a.in = in;
        a.out = out;
        a.plane = plane;
        a.n = e->n;
        a.n_frames = n_frames;
        a.t0 = t0;
        a.psize = e->psize;
        a.csize = e->csize;
        a.mode = mode;
        return a;
    };
    switch (e->kind) {
    case OLFX_KIND_DATTORRO: {
        if (e->dt_pre_check) {
            // one pre-delay for all instances or several: the network (dattorro.hip dattorro_rows)
            // and so the pre-delay ring's layout; its content is converted when that changes
            e->dt_pre_check = false;
            const float *pd = e->params.data() + (size_t)OLFX_DT_PREDELAY * e->n;
            const uint32_t d0 = dattorro_predelay_samples(pd[0]);
            bool uniform = true;
            for (uint32_t i = 1; i < e->n && uniform; ++i) uniform = dattorro_predelay_samples(pd[i]) == d0;
            const int net = dattorro_network(e->n_dt, (uint32_t)e->cus, uniform);
            const bool rows = net != DT_NET_V4;
            if (rows != (e->dt_net != DT_NET_V4) && e->frames > 0) {   // a fresh (zeroed) ring needs no conversion
                if (!e->dt_pre_tmp) HIPCHK(e, hipMalloc((void **)&e->dt_pre_tmp, (size_t)kDtSize[DT_PRE] * e->n_dt * 4));
                r = launch_dattorro_pre_layout(dt_args(nullptr, nullptr), e->dt_pre_tmp, rows, s);
                if (r != hipSuccess) return e->hip_fail(r, "pre-delay ring layout");
            }
            e->dt_net = net;
        }
        r = launch_dattorro(dt_args(din, dout), e->dt_net, s);
        break;
    }
    case OLFX_KIND_CHORUS:
        r = launch_chorus(ch_args(e->ch_pring, e->ch_cring, e->ch_state, e->ch_coef, din, dout, 0), s);
        break;
    case OLFX_KIND_PITCHSHIFT:
        r = launch_chorus(ch_args(e->ch_pring, e->ch_cring, e->ch_state, e->ch_coef, din, dout, 1), s);
        break;
    case OLFX_KIND_VOICE:
    case OLFX_KIND_VOICE_MOOG: {
        VoiceArgs a{};
        a.state = e->vc_state;
        a.coef = e->vc_coef;
        a.out = dout;
        a.n = e->n;
        a.n_frames = n_frames;
        a.moog = e->kind == OLFX_KIND_VOICE_MOOG;
        a.ev_more = ev.ev_more;
        a.ev = ev.ev;
        r = launch_voice(a, s);
        break;
    }
    case OLFX_KIND_FXRACK: {
        FxRackArgs a{};
        a.ring = e->fr_ring;
        a.state = e->fr_state;
        a.coef = e->fr_coef;
        a.in = din;
        a.out = dout;
        a.plane = plane;
        a.n = e->n;
        a.n_frames = n_frames;
        a.t0 = (uint32_t)(e->frames % kFrMaxDelay);
        a.components = e->n_components > 0;
        r = launch_fxrack(a, s);
        break;
    }
    case OLFX_KIND_CHAIN: {
        // one fused launch: chorus and pitch-shift waves feed the reverb wave through LDS
        ChainArgs a{};
        a.c1 = ch_args(e->ch_pring, e->ch_cring, e->ch_state, e->ch_coef, nullptr, nullptr, 0);
        a.c2 = ch_args(e->ps_pring, e->ps_cring, e->ps_state, e->ps_coef, nullptr, nullptr, 1);
        a.d = dt_args(nullptr, nullptr);
        a.in = din;
        a.out = dout;
        a.plane = plane;
        a.n = e->n;
        a.n_frames = n_frames;
        a.cus = (uint32_t)e->cus;
        r = launch_chain(a, s);
        break;
    }
    default: return e->fail(OLFX_E_KIND, "unknown kind");
    }
    if (r != hipSuccess) return e->hip_fail(r, "kernel launch");
    return OLFX_OK;
}

uint32_t in_channels(int kind) { return is_voice_kind(kind) ? 0u : 2u; }
uint32_t out_channels(int kind) { return is_voice_kind(kind) ? 1u : 2u; }

// Kinds whose kernels address the audio planes with 32-bit buffer offsets from `in` / `out`.
bool planes_32bit(int kind) {
    return kind == OLFX_KIND_CHORUS || kind == OLFX_KIND_PITCHSHIFT || kind == OLFX_KIND_CHAIN ||
           kind == OLFX_KIND_FXRACK;
}

// All n_frames of a call, as frame tiles where a launch's planes would leave the kernels' 32-bit
// offset range (planes_32bit): a tile is frames [f0, f0 + F) at in + f0 n with the caller's
// plane distance, so the launch spans plane + F n floats (< 4 GiB); when the caller's planes alone
// are >= 4 GiB apart, tiles are staged through a compact device buffer.  Frames run in order and
// the state carries between launches, so tiles compute exactly what one launch would.  The note
// events apply before the first tile (the block's start).
int run_frames(olfx_engine *e, const float *in, float *out, uint32_t n_frames, hipStream_t s, const VoiceArgs &ev) {
    const uint64_t n = e->n, plane = (uint64_t)n_frames * n;
    const uint64_t lim = (1ull << 30) - 1;                     // floats addressable in 32-bit bytes
    const VoiceArgs none{};
    if (!planes_32bit(e->kind) || plane + plane <= lim) {
        const int rc = launch(e, in, out, n_frames, plane, s, ev);
        if (rc) return rc;
        e->frames += n_frames;
        return OLFX_OK;
    }
    if (plane + 4 * n <= lim) {
        const uint32_t F = (uint32_t)std::min<uint64_t>(n_frames, ((lim - plane) / n) & ~3ull);
        for (uint32_t f0 = 0; f0 < n_frames; f0 += F) {
            const uint32_t Ft = std::min(F, n_frames - f0);
            const int rc = launch(e, in ? in + (size_t)f0 * n : nullptr, out + (size_t)f0 * n, Ft, plane, s,
                                  f0 ? none : ev);
            if (rc) return rc;
            e->frames += Ft;
        }
        return OLFX_OK;
    }
    // staged: tiles of up to 256 MiB per direction, compact [ch][F][n]
    const uint32_t ich = in_channels(e->kind), och = out_channels(e->kind);
    const uint32_t F = (uint32_t)std::max<uint64_t>(4, std::min<uint64_t>(n_frames, ((1ull << 26) / (2 * n)) & ~3ull));
    if (e->tile_floats < (size_t)2 * F * n) {
        if (e->tile_in) (void)hipFree(e->tile_in);
        if (e->tile_out) (void)hipFree(e->tile_out);
        e->tile_in = e->tile_out = nullptr;
        e->tile_floats = 0;
        HIPCHK(e, hipMalloc((void **)&e->tile_in, (size_t)2 * F * n * 4));
        HIPCHK(e, hipMalloc((void **)&e->tile_out, (size_t)2 * F * n * 4));
        e->tile_floats = (size_t)2 * F * n;
    }
    for (uint32_t f0 = 0; f0 < n_frames; f0 += F) {
        const uint32_t Ft = std::min(F, n_frames - f0);
        const size_t bytes = (size_t)Ft * n * 4;
        for (uint32_t c = 0; c < ich; ++c)
            HIPCHK(e, hipMemcpyAsync(e->tile_in + (size_t)c * Ft * n, in + c * plane + (size_t)f0 * n, bytes,
                                     hipMemcpyDeviceToDevice, s));
        const int rc = launch(e, e->tile_in, e->tile_out, Ft, (uint64_t)Ft * n, s, f0 ? none : ev);
        if (rc) return rc;
        for (uint32_t c = 0; c < och; ++c)
            HIPCHK(e, hipMemcpyAsync(out + c * plane + (size_t)f0 * n, e->tile_out + (size_t)c * Ft * n, bytes,
                                     hipMemcpyDeviceToDevice, s));
        e->frames += Ft;
    }
    return OLFX_OK;
}

}  // namespace

// =============================================================================================
// C-ABI
// =============================================================================================
extern "C" {

int olfx_abi_version(void) { return OLFX_ABI_VERSION; }

int olfx_kind_info_get(int kind, float sample_rate, olfx_kind_info *info) {
    if (!info) return OLFX_E_ARG;
    const uint32_t np = n_params_of(kind);
    if (!np) return OLFX_E_KIND;
    info->kind = kind;
    info->n_params = np;
    info->in_channels = in_channels(kind);
    info->out_channels = out_channels(kind);
    info->state_bytes_per_instance = state_bytes(kind, 1, sample_rate);
    return OLFX_OK;
}

int olfx_create(int kind, int device, uint32_t n_inst, float sample_rate, uint32_t block,
                olfx_engine **out) {
    if (!out) return OLFX_E_ARG;
    *out = nullptr;
    if (!n_params_of(kind)) {
        set_global_error("olfx_create: unknown kind %d", kind);
        return OLFX_E_KIND;
    }
    if (n_inst == 0 || !(sample_rate > 1000.f && sample_rate <= 384000.f) || block == 0 || (block & 3u)) {
        set_global_error("olfx_create: bad argument (n_inst=%u sr=%g block=%u)", n_inst, sample_rate, block);
        return OLFX_E_ARG;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_global_error("olfx_create: no HIP device visible (this library has no CPU path)");
        return OLFX_E_NODEVICE;
    }
    if (device < 0 || device >= ndev) {
        set_global_error("olfx_create: device %d out of range (%d devices)", device, ndev);
        return OLFX_E_NODEVICE;
    }
    olfx_engine *e = new (std::nothrow) olfx_engine();
    if (!e) return OLFX_E_NOMEM;
    e->kind = kind;
    e->device = device;
    e->n = n_inst;
    e->block = block;
    e->sr = sample_rate;
    e->n_params = n_params_of(kind);
    e->trace = std::getenv("OLFX_TRACE_CONTROL") && std::getenv("OLFX_TRACE_CONTROL")[0] == '1';
    if (const char *cb = std::getenv("OLFX_COPY_BYTES"))
        e->copy_bytes = std::min<size_t>((size_t)std::strtoull(cb, nullptr, 10), olfx_engine::kCopyBytes);
    chorus_sizes(sample_rate, &e->psize, &e->csize);
    e->n_dt = kind == OLFX_KIND_CHAIN ? (n_inst + 63u) & ~63u : n_inst;

    hipError_t r = hipSetDevice(device);
    if (r == hipSuccess) r = hipDeviceGetAttribute(&e->cus, hipDeviceAttributeMultiprocessorCount, device);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (r == hipSuccess) r = hipStreamCreateWithFlags(&e->copy_stream, hipStreamNonBlocking);
    if (r == hipSuccess) r = hipEventCreateWithFlags(&e->switched, hipEventDisableTiming);
    e->each_slot([&](olfx_engine::Slot &x) {
        if (r == hipSuccess) r = hipEventCreateWithFlags(&x.copied, hipEventDisableTiming);
        if (r == hipSuccess) r = hipEventCreateWithFlags(&x.consumed, hipEventDisableTiming);
    });
    if (r != hipSuccess) {
        int rc = e->hip_fail(r, "olfx_create: stream / events");
        olfx_destroy(e);
        return rc;
    }

    // carve one allocation
    const size_t n = n_inst;
    Carve cv;
    size_t o_dt_r = 0, o_dt_s = 0, o_dt_c = 0, o_ch_p = 0, o_ch_c = 0, o_ch_s = 0, o_ch_k = 0;
    size_t o_ps_p = 0, o_ps_c = 0, o_ps_s = 0, o_ps_k = 0, o_vc_s = 0, o_vc_c = 0;
    const bool has_dt = kind == OLFX_KIND_DATTORRO || kind == OLFX_KIND_CHAIN;
    const bool has_ch = kind == OLFX_KIND_CHORUS || kind == OLFX_KIND_PITCHSHIFT || kind == OLFX_KIND_CHAIN;
    const bool has_ps = kind == OLFX_KIND_CHAIN;
    const bool has_vc = is_voice_kind(kind);
    const bool has_fr = kind == OLFX_KIND_FXRACK;
    size_t o_fr_r = 0, o_fr_s = 0, o_fr_c = 0;
    if (has_fr) {
        o_fr_r = cv.take((size_t)kFrMaxDelay * 2 * n * 4);
        o_fr_s = cv.take((size_t)FRS_N * n * 4);
        o_fr_c = cv.take((size_t)FRC_N * n * 4);
    }
    if (has_dt) {
        o_dt_r = cv.take((size_t)dt_total_floats() * e->n_dt * 4);
        o_dt_s = cv.take((size_t)DTS_N * e->n_dt * 4);
        o_dt_c = cv.take((size_t)DTC_N * e->n_dt * 4);
    }
    if (has_ch) {
        o_ch_p = cv.take((size_t)2 * e->psize * n * 4);
        o_ch_c = cv.take((size_t)2 * e->csize * n * 4);
        o_ch_s = cv.take((size_t)CHS_N * n * 4);
        o_ch_k = cv.take((size_t)CHC_N * n * 4);
    }
    if (has_ps) {
        o_ps_p = cv.take((size_t)2 * e->psize * n * 4);
        o_ps_c = cv.take(256);
        o_ps_s = cv.take((size_t)CHS_N * n * 4);
        o_ps_k = cv.take((size_t)CHC_N * n * 4);
    }
    if (has_vc) {
        o_vc_s = cv.take((size_t)voice_state_slots(kind) * n * 4);
        o_vc_c = cv.take((size_t)VCC_N * n * 4);
    }
    e->d_bytes = cv.off;
    r = hipMalloc(&e->d_mem, e->d_bytes);
    if (r != hipSuccess) {
        int rc = e->fail(OLFX_E_NOMEM, "olfx_create: hipMalloc(%zu bytes): %s", e->d_bytes, hipGetErrorString(r));
        e->d_mem = nullptr;
        olfx_destroy(e);
        return rc;
    }
    char *base = (char *)e->d_mem;
    if (has_dt) {
        e->dt_rings = (float *)(base + o_dt_r);
        e->dt_state = (float *)(base + o_dt_s);
        e->dt_coef = (float *)(base + o_dt_c);
    }
    if (has_ch) {
        e->ch_pring = (float *)(base + o_ch_p);
        e->ch_cring = (float *)(base + o_ch_c);
        e->ch_state = (uint32_t *)(base + o_ch_s);
        e->ch_coef = (uint32_t *)(base + o_ch_k);
    }
    if (has_ps) {
        e->ps_pring = (float *)(base + o_ps_p);
        e->ps_cring = (float *)(base + o_ps_c);
        e->ps_state = (uint32_t *)(base + o_ps_s);
        e->ps_coef = (uint32_t *)(base + o_ps_k);
    }
    if (has_fr) {
        e->fr_ring = (float *)(base + o_fr_r);
        e->fr_state = (uint32_t *)(base + o_fr_s);
        e->fr_coef = (uint32_t *)(base + o_fr_c);
    }
    if (has_vc) {
        e->vc_state = (float *)(base + o_vc_s);
        e->vc_coef = (float *)(base + o_vc_c);
    }
    int rc = init_state(e);
    // slots allocated now, so that no block -- an all-voices note-off in the middle of a stream,
    // say -- pays a pinned / device allocation: the small ones at the copy threshold, the big ones
    // for the largest packet this engine can produce (up to 256 MiB each; larger on first need)
    const size_t maxw = max_packet_words(e);
    for (olfx_engine::Slot &sl : e->slot)
        if (!rc) rc = grow_slot(e, sl, olfx_engine::kCopyBytes / 4, false);
    if (maxw * 4 >= e->copy_bytes && maxw * 4 <= ((size_t)256 << 20))
        for (olfx_engine::Slot &sl : e->big)
            if (!rc) rc = grow_slot(e, sl, maxw, true);
    if (rc) {
        olfx_destroy(e);
        return rc;
    }
    *out = e;
    return OLFX_OK;
}

int olfx_destroy(olfx_engine *e) {
    if (!e) return OLFX_E_ARG;
    if (e->trace && e->tr_calls)
        std::fprintf(stderr, "olfx control trace (kind %d, %llu packets, mean us): fold %.2f slot-free %.2f "
                     "alloc %.2f coefficients %.2f events+deliver %.2f scatter %.2f\n", e->kind,
                     (unsigned long long)e->tr_calls, e->tr[0] / e->tr_calls, e->tr[1] / e->tr_calls,
                     e->tr[2] / e->tr_calls, e->tr[3] / e->tr_calls, e->tr[4] / e->tr_calls, e->tr[5] / e->tr_calls);
    (void)hipSetDevice(e->device);
    // the engine's own work only (its latest launch stream, its streams, its slots' markers): other
    // engines and the host application's kernels keep running
    if (wait_engine(e) != OLFX_OK) (void)hipDeviceSynchronize();
    e->each_slot([](olfx_engine::Slot &sl) {
        if (sl.h) (void)hipHostFree(sl.h);
        if (sl.d) (void)hipFree(sl.d);
        if (sl.copied) (void)hipEventDestroy(sl.copied);
        if (sl.consumed) (void)hipEventDestroy(sl.consumed);
    });
    if (e->copy_stream) (void)hipStreamDestroy(e->copy_stream);
    if (e->dt_pre_tmp) (void)hipFree(e->dt_pre_tmp);
    if (e->tile_in) (void)hipFree(e->tile_in);
    if (e->tile_out) (void)hipFree(e->tile_out);
    if (e->d_mem) (void)hipFree(e->d_mem);
    if (e->h_in) (void)hipHostFree(e->h_in);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->d_in) (void)hipFree(e->d_in);
    if (e->d_out) (void)hipFree(e->d_out);
    if (e->mix_dev) (void)hipFree(e->mix_dev);
    if (e->mix_done) (void)hipEventDestroy(e->mix_done);
    if (e->switched) (void)hipEventDestroy(e->switched);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return OLFX_OK;
}

int olfx_reset(olfx_engine *e) {
    if (!e) return OLFX_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    if (const int rc = wait_engine(e)) return rc;               // the last block, engine-scoped
    return init_state(e);
}

}  // extern "C"

namespace {
// A parameter value the reference's setter gives a meaning to (nullptr) or why not.
const char *bad_value(const olfx_engine *e, uint32_t field, float v) {
    if (!std::isfinite(v)) return "non-finite value";
    // the reference converts value * MAX_PREDELAY (4800) to uint16 (verb.cpp:137-139): values whose
    // product leaves [0, 65536) have no defined meaning there
    const bool predelay = (e->kind == OLFX_KIND_DATTORRO && field == OLFX_DT_PREDELAY) ||
                          (e->kind == OLFX_KIND_CHAIN && field == OLFX_CN_VERB0 + OLFX_DT_PREDELAY);
    if (predelay && !(v >= 0.f && v * 4800.0f < 65536.0f)) return "pre-delay outside [0, 65536/4800)";
    if (e->kind == OLFX_KIND_FXRACK && field == OLFX_FR_TOPOLOGY && !(v >= 0.f && v <= 4.f && v == (float)(int)v))
        return "rack topology must be 0, 1, 2, 3 or 4";
    return nullptr;
}

// One parameter of one instance; the rack's count of standalone components (topology >= 2, the
// kernel variant that serves them) follows its topology field.
void store_param(olfx_engine *e, uint32_t field, uint32_t inst, float v) {
    float &slot = e->params[(size_t)field * e->n + inst];
    if (e->kind == OLFX_KIND_DATTORRO && field == OLFX_DT_PREDELAY) e->dt_pre_check = true;
    if (e->kind == OLFX_KIND_FXRACK && field == OLFX_FR_TOPOLOGY)
        e->n_components += (v >= 2.f ? 1 : 0) - (slot >= 2.f ? 1 : 0);
    slot = v;
}
}  // namespace

extern "C" {

int olfx_set_params(olfx_engine *e, uint32_t first, uint32_t count, uint32_t field0, uint32_t n_fields,
                    const float *values) {
    if (!e) return OLFX_E_ARG;
    if (!values || (uint64_t)first + count > e->n || (uint64_t)field0 + n_fields > e->n_params)
        return e->fail(OLFX_E_ARG, "olfx_set_params: range out of bounds");
    // validate everything first: a rejected call changes nothing
    for (uint32_t f = 0; f < n_fields; ++f)
        for (uint32_t k = 0; k < count; ++k)
            if (const char *why = bad_value(e, field0 + f, values[(size_t)f * count + k]))
                return e->fail(OLFX_E_ARG, "olfx_set_params: %s", why);
    for (uint32_t f = 0; f < n_fields; ++f)
        for (uint32_t k = 0; k < count; ++k) store_param(e, field0 + f, first + k, values[(size_t)f * count + k]);
    if (is_voice_kind(e->kind))
        for (uint32_t k = 0; k < count; ++k) e->configured[first + k] = 1;
    mark_dirty(e, first, count);
    return OLFX_OK;
}

int olfx_set_param_list(olfx_engine *e, uint32_t field, const uint32_t *inst, const float *values, uint32_t count) {
    if (!e) return OLFX_E_ARG;
    if (count && (!inst || !values)) return e->fail(OLFX_E_ARG, "olfx_set_param_list: null list");
    if (field >= e->n_params) return e->fail(OLFX_E_ARG, "olfx_set_param_list: field out of range");
    for (uint32_t k = 0; k < count; ++k) {
        if (inst[k] >= e->n) return e->fail(OLFX_E_ARG, "olfx_set_param_list: instance %u out of range", inst[k]);
        if (const char *why = bad_value(e, field, values[k]))
            return e->fail(OLFX_E_ARG, "olfx_set_param_list: %s", why);
    }
    for (uint32_t k = 0; k < count; ++k) {
        store_param(e, field, inst[k], values[k]);
        if (is_voice_kind(e->kind)) e->configured[inst[k]] = 1;
        mark_dirty(e, inst[k], 1);
    }
    return OLFX_OK;
}

// ---- control changes (corelib/cc_map.h) ----
namespace {
enum : uint8_t {
    CC_CTL_PORTAMENTO = 5, CC_CTL_VOLUME = 7,
    CC_REVERB_BALANCE = 34,
    CC_DELAY_TIME = 35, CC_DELAY_FEEDBACK = 36, CC_DELAY_CUTOFF = 37, CC_DELAY_RESONANCE = 38,
    CC_DELAY_BALANCE = 39,
    CC_FILTER_CUTOFF = 41, CC_FILTER_RESONANCE = 42, CC_FILTER_DRIVE = 44,
    CC_FX_FILTER_CUTOFF = 45, CC_FX_FILTER_RESONANCE = 46, CC_FX_FILTER_TYPE = 47, CC_FX_FILTER_DRIVE = 48,
    CC_ENV_FILT_AMT = 73, CC_ENV_FILT_A = 74, CC_ENV_FILT_D = 75, CC_ENV_FILT_S = 76, CC_ENV_FILT_R = 77,
    CC_ENV_AMP_A = 108, CC_ENV_AMP_D = 109, CC_ENV_AMP_S = 110, CC_ENV_AMP_R = 111,
    CC_OSC_1_VOLUME = 114,
};
}  // namespace

int olfx_control_map(int kind, uint8_t control, int source, float value, uint32_t *field, float *param_value) {
    if (!field || !param_value || (source != OLFX_CTL_MIDI && source != OLFX_CTL_HARDWARE)) return OLFX_E_ARG;
    const bool midi = source == OLFX_CTL_MIDI;
    // MIDI: ol::core::scale(val, 0, 127, lo, hi, power); hardware: scale(value, 0, 1, ...) or raw
    auto sc = [&](float hi, float power) {
        return midi ? core_scale(value, 0.f, 127.f, 0.f, hi, power) : core_scale(value, 0.f, 1.f, 0.f, hi, power);
    };
    const float unit = midi ? core_scale(value, 0.f, 127.f, 0.f, 1.f, 1.f) : value;   // `scaled` / raw value
    auto put = [&](uint32_t f, float v) { *field = f; *param_value = v; return OLFX_OK; };
    if (is_voice_kind(kind)) {                     // SynthVoice.h:100-229
        switch (control) {
        case CC_CTL_VOLUME: return put(OLFX_VC_AMP_ENV_AMOUNT, unit);
        case CC_CTL_PORTAMENTO: return put(OLFX_VC_PORTAMENTO, sc(1.f, 4.f));
        case CC_FILTER_CUTOFF: return put(OLFX_VC_FILTER_CUTOFF, sc(20000.f, 2.5f));
        case CC_FILTER_RESONANCE: return put(OLFX_VC_FILTER_RESONANCE, unit);
        case CC_FILTER_DRIVE: return put(OLFX_VC_FILTER_DRIVE, unit);
        case CC_ENV_FILT_AMT: return put(OLFX_VC_FILTER_ENV_AMOUNT, unit);
        case CC_ENV_FILT_A: return put(OLFX_VC_FILTER_ATTACK, unit);
        case CC_ENV_FILT_D: return put(OLFX_VC_FILTER_DECAY, sc(1.f, 3.f));
        case CC_ENV_FILT_S: return put(OLFX_VC_FILTER_SUSTAIN, unit);
        case CC_ENV_FILT_R: return put(OLFX_VC_FILTER_RELEASE, unit);
        case CC_ENV_AMP_A: return put(OLFX_VC_AMP_ATTACK, unit);
        case CC_ENV_AMP_D: return put(OLFX_VC_AMP_DECAY, unit);
        case CC_ENV_AMP_S: return put(OLFX_VC_AMP_SUSTAIN, unit);
        case CC_ENV_AMP_R: return put(OLFX_VC_AMP_RELEASE, unit);
        case CC_OSC_1_VOLUME: return put(OLFX_FIELD_UPDATE_ONLY, unit);   // osc_1_mix: unused by Process
        default: return OLFX_IGNORED;
        }
    }
    if (kind == OLFX_KIND_FXRACK) {                // FxRack -> FilterFx / DelayFx / ReverbFx
        switch (control) {
        case CC_FX_FILTER_CUTOFF: return put(OLFX_FR_FILTER_CUTOFF, midi ? sc(20000.f, 1.f) : sc(20000.f, 1.02f));
        case CC_FX_FILTER_RESONANCE: return put(OLFX_FR_FILTER_RESONANCE, unit);
        case CC_FX_FILTER_DRIVE: return put(OLFX_FR_FILTER_DRIVE, unit);
        case CC_FX_FILTER_TYPE: return put(OLFX_FR_FILTER_TYPE, (float)(int32_t)sc(5.f, 1.f));   // FilterType(float)
        case CC_DELAY_TIME: return put(OLFX_FR_DELAY_TIME, unit);
        case CC_DELAY_FEEDBACK: return put(OLFX_FR_DELAY_FEEDBACK, unit);
        case CC_DELAY_BALANCE: return put(OLFX_FR_DELAY_BALANCE, unit);
        case CC_DELAY_CUTOFF:                      // DelayFx handles these in MIDI only (Fx.h:253-260)
            return midi ? put(OLFX_FR_DELAY_CUTOFF, sc(20000.f, 1.f)) : OLFX_IGNORED;
        case CC_DELAY_RESONANCE: return midi ? put(OLFX_FR_DELAY_RESONANCE, unit) : OLFX_IGNORED;
        case CC_REVERB_BALANCE: return put(OLFX_FR_REVERB_BALANCE, unit);
        case CC_CTL_VOLUME: return put(OLFX_FR_MASTER_VOLUME, unit);
        default: return OLFX_IGNORED;              // incl. the reverb CCs that reach only the ReverbSc stub
        }
    }
    return n_params_of(kind) ? OLFX_IGNORED : OLFX_E_KIND;
}

int olfx_control(olfx_engine *e, const olfx_control_event *ev, uint32_t n) {
    if (!e) return OLFX_E_ARG;
    if (n && !ev) return e->fail(OLFX_E_ARG, "olfx_control: null events");
    for (uint32_t k = 0; k < n; ++k) {
        if (ev[k].inst >= e->n) return e->fail(OLFX_E_ARG, "olfx_control: event %u: instance out of range", k);
        uint32_t field;
        float v;
        uint8_t control = ev[k].control;
        const float topo = e->kind == OLFX_KIND_FXRACK ? e->params[(size_t)OLFX_FR_TOPOLOGY * e->n + ev[k].inst] : 0.f;
        if (topo != 0.f) {
            // No FxRack around these instances (ol_daisy/app/synth/main.cpp:201-207 sends every CC to
            // delay_fx, reverb_fx and filter_fx directly): CC_FILTER_* (41-44) reach a FilterFx's own
            // handler (Fx.h:116-139), which the rack field map reaches as CC_FX_FILTER_* (45-48);
            // FxRack's own CC_FX_FILTER_* and master volume (CC 7) reach nothing.  A component alone
            // takes only its own controls: DelayFx 35-39 (Fx.h:218-267), ReverbFx the reverb CCs (of
            // which only the balance, 34, is audible through the ReverbSc stub), FilterFx 41-44.
            const bool filter_cc = control >= CC_FILTER_CUTOFF && control <= CC_FILTER_DRIVE;
            const bool delay_cc = control >= CC_DELAY_TIME && control <= CC_DELAY_BALANCE;
            const bool takes = topo == 1.f ? (filter_cc || delay_cc || control == CC_REVERB_BALANCE)
                             : topo == 2.f ? delay_cc : topo == 3.f ? control == CC_REVERB_BALANCE : filter_cc;
            if (!takes) continue;
            if (filter_cc) control = (uint8_t)(control - CC_FILTER_CUTOFF + CC_FX_FILTER_CUTOFF);
        }
        const int rc = olfx_control_map(e->kind, control, ev[k].source, ev[k].value, &field, &v);
        if (rc == OLFX_IGNORED) continue;
        if (rc != OLFX_OK) return e->fail(rc, "olfx_control: event %u", k);
        if (field == OLFX_FIELD_UPDATE_ONLY) {    // Update() with unchanged members
            if (is_voice_kind(e->kind)) e->configured[ev[k].inst] = 1;
            mark_dirty(e, ev[k].inst, 1);
            continue;
        }
        const int r2 = olfx_set_params(e, ev[k].inst, 1, field, 1, &v);
        if (r2 != OLFX_OK) return r2;
    }
    return OLFX_OK;
}

int olfx_set_param(olfx_engine *e, uint32_t inst, uint32_t field, float value) {
    return olfx_set_params(e, inst, 1, field, 1, &value);
}

int olfx_set_member(olfx_engine *e, uint32_t inst, uint32_t field, float value) {
    if (!e) return OLFX_E_ARG;
    if (!is_voice_kind(e->kind)) return olfx_set_params(e, inst, 1, field, 1, &value);
    if (inst >= e->n || field >= e->n_params) return e->fail(OLFX_E_ARG, "olfx_set_member: out of range");
    if (const char *why = bad_value(e, field, value)) return e->fail(OLFX_E_ARG, "olfx_set_member: %s", why);
    // SynthVoice::Process reads filter_cutoff, filter_env_amount and amp_env_amount itself every
    // sample (SynthVoice.h:42-52): writing them takes effect at once, Update()d or not.  Re-deriving
    // at the next block changes nothing else, since every other member still holds the value the
    // last Update() saw (they change only through olfx_set_params, i.e. with an Update()).
    const bool process_reads = field == OLFX_VC_FILTER_CUTOFF || field == OLFX_VC_FILTER_ENV_AMOUNT ||
                               field == OLFX_VC_AMP_ENV_AMOUNT;
    // the other members feed the components only through Update() (SynthVoice.h:66-98); written
    // after the first Update() they would take effect at the next block as if Update() had run,
    // which SynthVoice does not do: refused instead of silently diverging
    if (e->configured[inst] && !process_reads)
        return e->fail(OLFX_E_STATE, "olfx_set_member: instance %u is already Update()d (use olfx_set_params)", inst);
    store_param(e, field, inst, value);                 // no Update(): `configured` unchanged
    mark_dirty(e, inst, 1);
    return OLFX_OK;
}

int olfx_get_param(olfx_engine *e, uint32_t inst, uint32_t field, float *value) {
    if (!e || !value || inst >= e->n || field >= e->n_params) return OLFX_E_ARG;
    *value = e->params[(size_t)field * e->n + inst];
    return OLFX_OK;
}

int olfx_note_events(olfx_engine *e, const olfx_event *ev, uint32_t n) {
    if (!e) return OLFX_E_ARG;
    if (!is_voice_kind(e->kind)) return e->fail(OLFX_E_STATE, "olfx_note_events: not a voice engine");
    if (n && !ev) return e->fail(OLFX_E_ARG, "olfx_note_events: null events");
    for (uint32_t k = 0; k < n; ++k) {
        if (ev[k].inst >= e->n || ev[k].note > 127 || ev[k].type > OLFX_EV_GATE_OFF)
            return e->fail(OLFX_E_ARG, "olfx_note_events: bad event %u", k);
    }
    for (uint32_t k = 0; k < n; ++k)
        e->events.push_back(olfx_voice_event{ev[k].inst, ev[k].type, ev[k].note, ev[k].velocity, 0, 0.f});
    return OLFX_OK;
}

int olfx_voice_events(olfx_engine *e, const olfx_voice_event *ev, uint32_t n) {
    if (!e) return OLFX_E_ARG;
    if (!is_voice_kind(e->kind)) return e->fail(OLFX_E_STATE, "olfx_voice_events: not a voice engine");
    if (n && !ev) return e->fail(OLFX_E_ARG, "olfx_voice_events: null events");
    for (uint32_t k = 0; k < n; ++k) {
        if (ev[k].inst >= e->n || ev[k].note > 127 || ev[k].type > OLFX_EV_SET_FREQUENCY ||
            (ev[k].type == OLFX_EV_SET_FREQUENCY && !std::isfinite(ev[k].value)))
            return e->fail(OLFX_E_ARG, "olfx_voice_events: bad event %u", k);
    }
    e->events.insert(e->events.end(), ev, ev + n);
    return OLFX_OK;
}

int olfx_update(olfx_engine *e, uint32_t first, uint32_t count) {
    if (!e) return OLFX_E_ARG;
    if ((uint64_t)first + count > e->n) return e->fail(OLFX_E_ARG, "olfx_update: range out of bounds");
    if (is_voice_kind(e->kind))
        for (uint32_t k = 0; k < count; ++k) e->configured[first + k] = 1;
    mark_dirty(e, first, count);
    return OLFX_OK;
}

int olfx_process(olfx_engine *e, const float *in, float *out, uint32_t n_frames, int io_flags, void *stream) {
    if (!e) return OLFX_E_ARG;
    if (n_frames == 0) return OLFX_OK;
    if ((n_frames & 3u) || !out || (in_channels(e->kind) && !in))
        return e->fail(OLFX_E_ARG, "olfx_process: bad argument (n_frames=%u must be a multiple of 4)", n_frames);
    if (io_flags != OLFX_IO_DEVICE && io_flags != OLFX_IO_HOST)
        return e->fail(OLFX_E_ARG, "olfx_process: bad io_flags");
    HIPCHK(e, hipSetDevice(e->device));
    hipStream_t s = (hipStream_t)stream;   // NULL = the HIP default (null) stream
    const size_t fin = (size_t)in_channels(e->kind) * n_frames * e->n;
    const size_t fout = (size_t)out_channels(e->kind) * n_frames * e->n;
    // a stream switch: this block's work (the control scatter included) after the previous launch
    if (e->have_last && s != e->last_stream) {
        HIPCHK(e, hipEventRecord(e->switched, e->last_stream));
        HIPCHK(e, hipStreamWaitEvent(s, e->switched, 0));
    }
    int rc = OLFX_OK;
    if (io_flags == OLFX_IO_HOST) {
        rc = ensure_staging(e, fin ? fin : 1, fout);
        if (rc) return rc;
    }
    // the block's parameter changes and note events: asynchronous, O(changed)
    VoiceArgs ev{};
    olfx_engine::Slot *sl = nullptr;
    rc = submit_control(e, s, &ev, &sl);
    if (rc) return rc;
    if (io_flags == OLFX_IO_HOST) {
        hipError_t r = hipSuccess;
        if (fin) {
            std::memcpy(e->h_in, in, fin * 4);
            r = hipMemcpyAsync(e->d_in, e->h_in, fin * 4, hipMemcpyHostToDevice, s);
        }
        rc = r == hipSuccess ? run_frames(e, fin ? e->d_in : nullptr, e->d_out, n_frames, s, ev)
                             : e->hip_fail(r, "olfx_process: input copy");
    } else {
        rc = run_frames(e, in, out, n_frames, s, ev);
    }
    e->last_stream = s;
    e->have_last = true;
    // the slot is free again once whatever was queued on `s` (the scatter, the kernels) is done --
    // recorded on the error paths too, so a later block never overwrites a packet still being read
    if (sl) {
        const hipError_t r = slot_queued(e, sl, s);
        if (!rc && r != hipSuccess) rc = e->hip_fail(r, "hipEventRecord(consumed)");
    }
    if (rc) return rc;
    if (io_flags == OLFX_IO_HOST) {
        HIPCHK(e, hipMemcpyAsync(e->h_out, e->d_out, fout * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipStreamSynchronize(s));
        std::memcpy(out, e->h_out, fout * 4);
    }
    return OLFX_OK;
}

// ---- voice buses: Polyvoice::Process / VoiceMap::Process (Polyvoice.h:28-33, VoiceMap.h:64-73) ----
int olfx_mix_config(olfx_engine *e, uint32_t n_buses, const uint32_t *offsets, const uint32_t *order) {
    if (!e) return OLFX_E_ARG;
    if (!is_voice_kind(e->kind)) return e->fail(OLFX_E_STATE, "olfx_mix_config: not a voice engine");
    std::vector<uint32_t> h;
    if (n_buses) {
        if (!offsets || offsets[0] != 0) return e->fail(OLFX_E_ARG, "olfx_mix_config: offsets must start at 0");
        for (uint32_t b = 0; b < n_buses; ++b)
            if (offsets[b + 1] < offsets[b])
                return e->fail(OLFX_E_ARG, "olfx_mix_config: offsets decrease at bus %u", b);
        const uint32_t len = offsets[n_buses];
        if (len > e->n)
            return e->fail(OLFX_E_ARG, "olfx_mix_config: %u entries for %u voices (each voice at most once)", len, e->n);
        if (len && !order) return e->fail(OLFX_E_ARG, "olfx_mix_config: null order");
        std::vector<uint8_t> seen(e->n, 0);
        for (uint32_t k = 0; k < len; ++k) {
            if (order[k] >= e->n)
                return e->fail(OLFX_E_ARG, "olfx_mix_config: order[%u] = %u out of range", k, order[k]);
            // listed twice, the reference would run the voice twice per frame (Polyvoice.h:28-33)
            if (seen[order[k]]++) return e->fail(OLFX_E_ARG, "olfx_mix_config: voice %u listed twice", order[k]);
        }
        h.assign(offsets, offsets + n_buses + 1);
        h.insert(h.end(), order, order + len);
    }
    HIPCHK(e, hipSetDevice(e->device));
    // the new lists first: a failed allocation leaves the current configuration in place
    uint32_t *fresh = nullptr;
    if (n_buses) {
        HIPCHK(e, hipMalloc((void **)&fresh, h.size() * 4));
        const hipError_t r = hipMemcpy(fresh, h.data(), h.size() * 4, hipMemcpyHostToDevice);
        if (r != hipSuccess) {
            (void)hipFree(fresh);
            return e->hip_fail(r, "olfx_mix_config upload");
        }
    }
    if (e->mix_dev) {   // the last mix launched (on any stream) may still read the old lists
        hipError_t r = e->mix_done ? hipEventSynchronize(e->mix_done) : hipSuccess;
        if (r == hipSuccess) r = hipFree(e->mix_dev);
        if (r != hipSuccess) {          // the current configuration stays; the new lists are dropped
            if (fresh) (void)hipFree(fresh);
            return e->hip_fail(r, "olfx_mix_config: releasing the previous lists");
        }
    }
    e->mix_dev = fresh;
    e->n_buses = n_buses;
    // buses that are contiguous voice runs in voice order, on multiples of 4 voices, take
    // voice_mix_v4 (float4 runs)
    e->mix_quad = 0;
    if (n_buses) {
        const uint32_t len = offsets[n_buses];
        bool quad = true;
        for (uint32_t k = 0; k < len && quad; ++k) quad = order[k] == k;
        for (uint32_t b = 0; b <= n_buses && quad; ++b) quad = (offsets[b] & 3u) == 0;
        e->mix_quad = quad ? 1u : 0u;
    }
    return OLFX_OK;
}

int olfx_mix(olfx_engine *e, const float *voice_out, float *bus_out, uint32_t n_frames, int io_flags, void *stream) {
    if (!e) return OLFX_E_ARG;
    if (!e->n_buses) return e->fail(OLFX_E_STATE, "olfx_mix: no buses (olfx_mix_config)");
    if (n_frames == 0) return OLFX_OK;
    if (!voice_out || !bus_out) return e->fail(OLFX_E_ARG, "olfx_mix: null buffer");
    if (io_flags != OLFX_IO_DEVICE && io_flags != OLFX_IO_HOST) return e->fail(OLFX_E_ARG, "olfx_mix: bad io_flags");
    HIPCHK(e, hipSetDevice(e->device));
    if (!e->mix_done) HIPCHK(e, hipEventCreateWithFlags(&e->mix_done, hipEventDisableTiming));
    hipStream_t s = (hipStream_t)stream;
    // a stream switch, as in olfx_process: the mix after the engine's previous launch, and the next
    // launch (on whichever stream) after the mix
    if (e->have_last && s != e->last_stream) {
        HIPCHK(e, hipEventRecord(e->switched, e->last_stream));
        HIPCHK(e, hipStreamWaitEvent(s, e->switched, 0));
    }
    MixArgs a{};
    a.off = e->mix_dev;
    a.order = e->mix_dev + e->n_buses + 1;
    a.quad = e->mix_quad;
    a.n = e->n;
    a.n_buses = e->n_buses;
    a.n_frames = n_frames;
    const size_t fin = (size_t)n_frames * e->n, fout = (size_t)n_frames * e->n_buses;
    hipError_t r;
    if (io_flags == OLFX_IO_HOST) {
        const int rc = ensure_staging(e, fin, fout);
        if (rc) return rc;
        std::memcpy(e->h_in, voice_out, fin * 4);
        std::memcpy(e->h_out, bus_out, fout * 4);
        HIPCHK(e, hipMemcpyAsync(e->d_in, e->h_in, fin * 4, hipMemcpyHostToDevice, s));
        HIPCHK(e, hipMemcpyAsync(e->d_out, e->h_out, fout * 4, hipMemcpyHostToDevice, s));
        a.in = e->d_in;
        a.out = e->d_out;
        if ((r = launch_mix(a, s)) != hipSuccess) return e->hip_fail(r, "mix launch");
        HIPCHK(e, hipEventRecord(e->mix_done, s));
        HIPCHK(e, hipMemcpyAsync(e->h_out, e->d_out, fout * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(e, hipStreamSynchronize(s));
        std::memcpy(bus_out, e->h_out, fout * 4);
        e->last_stream = s;
        e->have_last = true;
        return OLFX_OK;
    }
    a.in = voice_out;
    a.out = bus_out;
    if ((r = launch_mix(a, s)) != hipSuccess) return e->hip_fail(r, "mix launch");
    HIPCHK(e, hipEventRecord(e->mix_done, s));
    e->last_stream = s;
    e->have_last = true;
    return OLFX_OK;
}

int olfx_sync(olfx_engine *e) {
    if (!e) return OLFX_E_ARG;
    HIPCHK(e, hipSetDevice(e->device));
    return wait_engine(e);
}

void *olfx_stream(const olfx_engine *e) { return e ? (void *)e->stream : nullptr; }

uint32_t olfx_num_instances(const olfx_engine *e) { return e ? e->n : 0; }
int olfx_kind(const olfx_engine *e) { return e ? e->kind : 0; }
uint64_t olfx_frames_processed(const olfx_engine *e) { return e ? e->frames : 0; }
uint32_t olfx_num_buses(const olfx_engine *e) { return e ? e->n_buses : 0; }

double olfx_algorithmic_bytes_per_frame(const olfx_engine *e) {
    if (!e) return 0.0;
    // DESIGN.md section 4 / SURVEY.md section 8d, B = 256: compulsory ring traffic + I/O
    switch (e->kind) {
    case OLFX_KIND_DATTORRO: return 164.6;     // 148.6 state + 8 in + 8 out (stereo in)
    case OLFX_KIND_CHORUS: return 56.0;        // 2 x (pitch w + 2 taps + chorus w + tap) x 4 + 16 I/O
    case OLFX_KIND_PITCHSHIFT: return 40.0;    // 2 x (w + 2 taps) x 4 + 16 I/O
    case OLFX_KIND_VOICE: return 5.4;          // 4 B out + per-block state
    case OLFX_KIND_VOICE_MOOG: return 5.7;     // 4 B out + per-block state (9 more state words)
    case OLFX_KIND_CHAIN: return 228.6;
    case OLFX_KIND_FXRACK: return 32.0;       // ring write 8 + ring read 8 + I/O 16 per stereo frame
    default: return 0.0;
    }
}

double olfx_algorithmic_read_bytes_per_frame(const olfx_engine *e) {
    if (!e) return 0.0;
    // the read share of the figures above (the north star's "HBM-read roofline"): every tap read
    // of data older than the block, counted once, plus the input
    switch (e->kind) {
    case OLFX_KIND_DATTORRO: return 6445.0 * 4.0 / 256.0 + 8.0;   // 27 taps: sum min(d, 256) = 6,445 floats; + 8 in
    case OLFX_KIND_CHORUS: return 32.0;        // 2 x (2 pitch taps + chorus tap) x 4 + 8 in
    case OLFX_KIND_PITCHSHIFT: return 24.0;    // 2 x 2 taps x 4 + 8 in
    case OLFX_KIND_VOICE: return 0.7;          // per-block state and coefficients
    case OLFX_KIND_VOICE_MOOG: return 0.85;
    case OLFX_KIND_CHAIN: return 8.0 + 24.0 + 16.0 + 6445.0 * 4.0 / 256.0;   // 148.7
    case OLFX_KIND_FXRACK: return 16.0;        // ring read 8 + in 8
    default: return 0.0;
    }
}

const char *olfx_kernel_name(const olfx_engine *e) {
    if (!e) return "";
    switch (e->kind) {
    case OLFX_KIND_DATTORRO:   // the network of the last block (dattorro.hip dattorro_rows)
        return dattorro_network_name(e->dt_net);
    case OLFX_KIND_CHORUS:
    case OLFX_KIND_PITCHSHIFT: return "chorus_block_v11";
    case OLFX_KIND_VOICE: return "voice_block_v5";
    case OLFX_KIND_VOICE_MOOG: return "voice_block_v4";
    case OLFX_KIND_CHAIN: return "chain_block_v5";
    case OLFX_KIND_FXRACK: return "fxrack_block_v3";
    default: return "";
    }
}

const char *olfx_last_error(const olfx_engine *e) {
    if (e) return e->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    static thread_local std::string copy;
    copy = g_err;
    return copy.c_str();
}

}  // extern "C"
