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
//
// MOOG = true is the Daisy synth firmware's voice, SynthVoice(OscillatorSoundSource, MoogFilter)
// (ol_daisy/app/synth/main.cpp:49-52, Filter.h:35-63): MoogFilter::Process is a no-op and
// Low(frame) = daisysp::LadderFilter::Process(frame) with SetFreq(fc) (-> SetAlpha) every sample,
// unclamped.  LadderFilter: 4x linear-interpolated oversampling, Pade tanh of the feedback sum,
// four one-zero/one-pole stages, LP24 output (restated, [unverified] like the rest of DaisySP;
// oracle/voice_ref.c ladder_process).  ~4x the Svf voice's VALU work per sample.
#include "olfx_internal.h"

namespace olfx {

namespace {

enum { SEG_IDLE = 0, SEG_ATTACK = 1, SEG_DECAY = 2, SEG_RELEASE = 3 };

// daisysp::Adsr::Process(gate), branch-free: every lane evaluates the segment step and selects
// (same operations and order as the branchy form, so the same bits).
__device__ __forceinline__ float adsr(bool gate, uint32_t &mode, bool &gprev, float &x, float atk_d0,
                                      float atk_tgt, float dec_d0, float rel_d0, float sus) {
    mode = (gate && !gprev) ? (uint32_t)SEG_ATTACK : ((!gate && gprev) ? (uint32_t)SEG_RELEASE : mode);
    gprev = gate;
    const bool atk = mode == SEG_ATTACK, dec = mode == SEG_DECAY, idle = mode == SEG_IDLE;
    const float d0 = atk ? atk_d0 : (dec ? dec_d0 : rel_d0);
    const float target = atk ? atk_tgt : (dec ? sus : -0.01f);
    const float xn = x + d0 * (target - x);
    const bool top = atk && xn > 1.f, bottom = !atk && xn < 0.0f;
    const float out = idle ? 0.0f : (top ? 1.0f : (bottom ? 0.0f : xn));
    x = idle ? x : out;
    mode = top ? (uint32_t)SEG_DECAY : (bottom && !idle ? (uint32_t)SEG_IDLE : mode);
    return out;
}

// polyBLEP residual with one division: t/dt near the wrap start, (t-1)/dt near its end -- the
// same quotients as the two-branch form
__device__ __forceinline__ float polyblep(float dt, float t) {
    const bool lo = t < dt, hi = !lo && t > 1.0f - dt;
    const float q = (lo ? t : t - 1.0f) * __builtin_amdgcn_rcpf(dt);   // v_rcp: ~1 ulp
    const float rlo = q + q - q * q - 1.0f;
    const float rhi = q * q + q + q + 1.0f;
    return lo ? rlo : (hi ? rhi : 0.0f);
}

// sin(x) for x in [0, pi/4] (Svf::SetFreq's argument pi * min(0.25, fc / 2sr)): odd Taylor
// polynomial to x^9, truncation < 2e-9, i.e. within an ulp of sinf; branch-free.  The voice's
// parity tolerance (1e-5 of max(|ref|, rms), tests/test_gpu_parity.py) covers ulp-level
// differences from the host's sinf.
__device__ __forceinline__ float sin_quarter(float x) {
    const float x2 = x * x;
    float p = 2.7557319e-6f;                 // 1/9!
    p = p * x2 + -1.9841270e-4f;             // -1/7!
    p = p * x2 + 8.3333333e-3f;              // 1/5!
    p = p * x2 + -1.6666667e-1f;             // -1/3!
    return x + (x * x2) * p;
}

// daisysp::LadderFilter's tanh: Pade approximant, saturating beyond |x| > 3 (the exact division
// keeps it bit-identical with the oracle)
__device__ __forceinline__ float ladder_tanh(float x) {
    const float x2 = x * x;
    const float r = x * (27.0f + x2) / (27.0f + 9.0f * x2);
    return x > 3.0f ? 1.0f : (x < -3.0f ? -1.0f : r);
}

// LadderFilter::LPF stage i: one zero at -0.3 (0.3/1.3 feed-forward of the previous input), one pole
__device__ __forceinline__ float ladder_lpf(float s, float alpha, float &z0, float &z1) {
    float ft = s * (1.0f / 1.3f) + (0.3f / 1.3f) * z0 - z1;
    ft = ft * alpha + z1;
    z1 = ft;
    z0 = s;
    return ft;
}

struct Ladder {
    float z0[4], z1[4], old;
};

// LadderFilter::SetFreq(fc) (SetAlpha) then Process(in), LP24
__device__ __forceinline__ float ladder_process(Ladder &L, float fc, float in, float k, float drive_scaled,
                                                float wrec) {
    const float wc = fc * 2.0f * 3.1415927410125732f * wrec;
    const float wc2 = wc * wc;
    const float alpha = 0.9892f * wc - 0.4324f * wc2 + 0.1381f * wc * wc2 - 0.0202f * wc2 * wc2;
    const float qadj = 1.006f + 0.0536f * wc - 0.095f * wc2 - 0.05f * wc2 * wc2;
    const float input = in * drive_scaled;
    float total = 0.0f, interp = 0.0f;
#pragma unroll
    for (int os = 0; os < 4; ++os) {
        float u = (interp * L.old + (1.0f - interp) * input) - (L.z1[3] - 0.5f * input) * k * qadj;
        u = ladder_tanh(u);
        const float s1 = ladder_lpf(u, alpha, L.z0[0], L.z1[0]);
        const float s2 = ladder_lpf(s1, alpha, L.z0[1], L.z1[1]);
        const float s3 = ladder_lpf(s2, alpha, L.z0[2], L.z1[2]);
        const float s4 = ladder_lpf(s3, alpha, L.z0[3], L.z1[3]);
        total += s4 * (1.0f / 4);
        interp += 1.0f / 4;
    }
    L.old = input;
    return total;
}

}  // namespace

template <bool MOOG>
__global__ __launch_bounds__(64) void voice_block_v2(VoiceArgs a) {
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
    const float inv_2sr = 1.0f / (sr * 2.0f);

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
    Ladder L;
    if (MOOG) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            L.z0[k] = s[(VCS_LZ0 + k) * n + i];
            L.z1[k] = s[(VCS_LZ1 + k) * n + i];
        }
        L.old = s[VCS_LOLD * n + i];
    }

#pragma unroll 2
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
        if (MOOG) {
            // LadderFilter slots: VCC_LADDER_K = damp_res, VCC_LADDER_DRIVE = drive,
            // VCC_LADDER_WREC = fc_max
            a.out[(size_t)f * n + i] = ladder_process(L, fc_in, src, damp_res, drive, fc_max) * amp;
            continue;
        }
        const float fc = fminf(fmaxf(fc_in, 1.0e-6f), fc_max);
        // the three per-sample divisions of Svf::SetFreq / polyBLEP use the hardware reciprocal
        // (~1 ulp; within the voice tolerance, like sin_quarter)
        const float fcn = fc * inv_2sr;
        const float arg = 0.25f < fcn ? 0.25f : fcn;
        const float fq = 2.0f * sin_quarter(3.1415927410125732f * arg);
        const float lim = 2.0f * __builtin_amdgcn_rcpf(fq) - fq * 0.5f;
        const float dlim = 2.0f < lim ? 2.0f : lim;
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
    if (MOOG) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[(VCS_LZ0 + k) * n + i] = L.z0[k];
            s[(VCS_LZ1 + k) * n + i] = L.z1[k];
        }
        s[VCS_LOLD * n + i] = L.old;
    }
}

hipError_t launch_voice(const VoiceArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t threads = 64;       // one wave per workgroup: 32,768 voices spread over every CU
    const dim3 grid((a.n + threads - 1) / threads);
    if (a.moog) hipLaunchKernelGGL(voice_block_v2<true>, grid, dim3(threads), 0, s, a);
    else hipLaunchKernelGGL(voice_block_v2<false>, grid, dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
