// ol_dsp_amd/csrc/voice.hip -- synthlib SynthVoice, one lane per voice, state in registers.
//
// Reference call sequence per sample: modules/synthlib/SynthVoice.h:41-53
//   amp = ampEnv.Process(gate) * amp_env_amount
//   osc.SetFreq(port.Process(freq)); s = osc.Process()          (WAVE_POLYBLEP_SAW, amp 0.5)
//   fc = cutoff + ((filtEnv.Process(gate) * 20000) * filter_env_amount)
//   svf.SetFreq(fc); svf.Process(s); out = svf.Low() * amp
// DaisySP (Oscillator, Adsr, Svf) is not in the reference tree: the arithmetic restates its
// published algorithm ("parity unpinned").  Setter-side transcendentals
// (expf/logf/powf in Adsr/Svf/Port setters, mtof) run on the host; the per-sample sinf of
// Svf::SetFreq runs here.  VALU-bound: ~5 B of HBM traffic per sample.
#include "olfx_internal.h"

namespace olfx {

namespace {

enum { SEG_IDLE = 0, SEG_ATTACK = 1, SEG_DECAY = 2, SEG_RELEASE = 3 };

// daisysp::Adsr::Process(gate)
__device__ __forceinline__ float adsr(bool gate, uint32_t &mode, bool &gprev, float &x, float atk_d0,
                                      float atk_tgt, float dec_d0, float rel_d0, float sus) {
    if (gate && !gprev) mode = SEG_ATTACK;
    else if (!gate && gprev) mode = SEG_RELEASE;
    gprev = gate;
    float d0 = atk_d0;
    if (mode == SEG_DECAY) d0 = dec_d0;
    else if (mode == SEG_RELEASE) d0 = rel_d0;
    const float target = mode == SEG_DECAY ? sus : -0.01f;
    float out = 0.0f;
    if (mode == SEG_ATTACK) {
        x += d0 * (atk_tgt - x);
        out = x;
        if (out > 1.f) { x = out = 1.f; mode = SEG_DECAY; }
    } else if (mode == SEG_DECAY || mode == SEG_RELEASE) {
        x += d0 * (target - x);
        out = x;
        if (out < 0.0f) { x = out = 0.f; mode = SEG_IDLE; }
    }
    return out;
}

__device__ __forceinline__ float polyblep(float dt, float t) {
    if (t < dt) { t /= dt; return t + t - t * t - 1.0f; }
    else if (t > 1.0f - dt) { t = (t - 1.0f) / dt; return t * t + t + t + 1.0f; }
    return 0.0f;
}

}  // namespace

__global__ __launch_bounds__(256) void voice_block_v1(VoiceArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;
    const float *c = a.coef;
    const float atk_d0a = c[VCC_ATK_D0A * n + i], atk_tga = c[VCC_ATK_TGT_A * n + i];
    const float dec_d0a = c[VCC_DEC_D0A * n + i], rel_d0a = c[VCC_REL_D0A * n + i], sus_a = c[VCC_SUS_A * n + i];
    const float atk_d0f = c[VCC_ATK_D0F * n + i], atk_tgf = c[VCC_ATK_TGT_F * n + i];
    const float dec_d0f = c[VCC_DEC_D0F * n + i], rel_d0f = c[VCC_REL_D0F * n + i], sus_f = c[VCC_SUS_F * n + i];
    const float amp_amt = c[VCC_AMP_AMT * n + i], cutoff = c[VCC_CUTOFF * n + i], fenv_amt = c[VCC_FENV_AMT * n + i];
    const float damp_res = c[VCC_DAMP_RES * n + i], drive = c[VCC_DRIVE * n + i];
    const float port_c = c[VCC_PORT_COEF * n + i], fc_max = c[VCC_FC_MAX * n + i];
    const float sr = c[VCC_SR * n + i], inv_sr = c[VCC_INV_SR * n + i];

    float *s = a.state;
    float phase = s[VCS_PHASE * n + i];
    float port_z = s[VCS_PORT_Z * n + i];
    float xa = s[VCS_ENVA_X * n + i];
    float xf = s[VCS_ENVF_X * n + i];
    float low = s[VCS_LOW * n + i];
    float band = s[VCS_BAND * n + i];
    const float freq = s[VCS_FREQ * n + i];
    uint32_t flags = __float_as_uint(s[VCS_FLAGS * n + i]);
    uint32_t mode_a = flags & 7u, mode_f = (flags >> 3) & 7u;
    bool gprev_a = (flags >> 6) & 1u, gprev_f = (flags >> 7) & 1u;
    const bool gate = (flags >> 8) & 1u;

    for (uint32_t f = 0; f < a.n_frames; ++f) {
        float amp = adsr(gate, mode_a, gprev_a, xa, atk_d0a, atk_tga, dec_d0a, rel_d0a, sus_a);
        amp *= amp_amt;
        // Port::Process (Portamento.h:218-221), Oscillator::SetFreq: phase_inc = f * sr_recip
        port_z = freq + port_c * (port_z - freq);
        const float inc = port_z * inv_sr;
        // Oscillator::Process, WAVE_POLYBLEP_SAW
        float o = (2.0f * phase) - 1.0f;
        o -= polyblep(inc, phase);
        o *= -1.0f;
        phase += inc;
        if (phase > 1.0f) phase -= 1.0f;
        const float src = o * 0.5f;
        // filter envelope -> Svf::SetFreq
        const float fe = adsr(gate, mode_f, gprev_f, xf, atk_d0f, atk_tgf, dec_d0f, rel_d0f, sus_f);
        const float fc_in = cutoff + ((fe * 20000.0f) * fenv_amt);
        const float fc = fminf(fmaxf(fc_in, 1.0e-6f), fc_max);
        const float arg = 0.25f < fc / (sr * 2.0f) ? 0.25f : fc / (sr * 2.0f);
        const float fq = 2.0f * sinf(3.1415927410125732f * arg);
        const float dlim = 2.0f < 2.0f / fq - fq * 0.5f ? 2.0f : 2.0f / fq - fq * 0.5f;
        const float damp = damp_res < dlim ? damp_res : dlim;
        // Svf::Process: two passes, Low() = average of the two low outputs
        float notch = src - damp * band;
        low = low + fq * band;
        float high = notch - low;
        band = fq * high + band - drive * band * band * band;
        float out_low = 0.5f * low;
        notch = src - damp * band;
        low = low + fq * band;
        high = notch - low;
        band = fq * high + band - drive * band * band * band;
        out_low += 0.5f * low;
        a.out[(size_t)f * n + i] = out_low * amp;
    }

    flags = mode_a | (mode_f << 3) | ((uint32_t)gprev_a << 6) | ((uint32_t)gprev_f << 7) | ((uint32_t)gate << 8);
    s[VCS_PHASE * n + i] = phase;
    s[VCS_PORT_Z * n + i] = port_z;
    s[VCS_ENVA_X * n + i] = xa;
    s[VCS_ENVF_X * n + i] = xf;
    s[VCS_LOW * n + i] = low;
    s[VCS_BAND * n + i] = band;
    s[VCS_FLAGS * n + i] = __uint_as_float(flags);
}

hipError_t launch_voice(const VoiceArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t threads = 256;
    hipLaunchKernelGGL(voice_block_v1, dim3((a.n + threads - 1) / threads), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
