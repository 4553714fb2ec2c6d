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

// Contraction.  The voice's continuous stages are contracted into FMAs where the firmware's
// compiler would contract a * b + c (GCC's default -ffp-contract=fast in GNU C++): the polyBLEP
// quadratics, Svf::SetFreq's sine polynomial and damping limit, the Svf's low/band updates, the
// ladder's stages, feedback sum and SetAlpha polynomials.  Not the envelope updates, the
// portamento or the phase accumulator (their segment ends and the phase wrap are discontinuous:
// contracting them moved a segment end or a wrap by a sample, up to 2.8e-2 from the unfused
// oracle) nor the Svf's notch (2.7e-5 on a default-parameter voice).  Measured on the CPU
// restatement, the contracted stages together stay < 2e-6 from the unfused oracle; the voice's
// parity tolerance is 1e-5 of max(|ref|, rms) (tests/test_gpu_parity.py).  MI355X: the Svf voice
// 0.0358 -> 0.0333 ms, the Moog voice 0.1226 -> 0.0664 ms (32,768 voices, same box).

// polyBLEP residual with one division: t/dt near the wrap start, (t-1)/dt near its end -- the
// same quotients as the two-branch form; q + q - q q - 1 and q q + q + q + 1 as
// fma(-q, q, 2q) - 1 and fma(q, q, 2q) + 1
__device__ __forceinline__ float polyblep(float dt, float t) {
    const bool lo = t < dt, hi = t > 1.0f - dt;                          // (lo wins the select)
    const float q = (lo ? t : t - 1.0f) * __builtin_amdgcn_rcpf(dt);   // v_rcp: ~1 ulp
    const float q2 = q + q;
    float rlo = __builtin_fmaf(-q, q, q2) - 1.0f;
    float rhi = __builtin_fmaf(q, q, q2) + 1.0f;
    asm volatile("" : "+v"(rlo), "+v"(rhi));      // both computed: selects, not an exec-mask diamond
    return lo ? rlo : (hi ? rhi : 0.0f);
}

// Oscillator::Process's saw, WAVE_POLYBLEP_SAW with amp 0.5 (o = 2t - 1, o -= blep, o *= -1, o * amp):
// -((2t - 1) - blep) / 2 = fma(1/2, blep, 1/2 - t) -- 2t - 1 = 2 (t - 1/2) and the halving are
// exact scalings, so both forms round the same sum once (up to the sign of an exact zero)
__device__ __forceinline__ float saw_out(float t, float blep) { return __builtin_fmaf(0.5f, blep, 0.5f - t); }

// sin(x) for x in [0, pi/4] (Svf::SetFreq's argument pi * min(0.25, fc / 2sr)): odd Taylor
// polynomial to x^9 in Horner form, truncation < 2e-9; branch-free.
__device__ __forceinline__ float sin_quarter(float x) {
    const float x2 = x * x;
    float p = __builtin_fmaf(2.7557319e-6f, x2, -1.9841270e-4f);     // 1/9!, -1/7!
    p = __builtin_fmaf(p, x2, 8.3333333e-3f);                        // 1/5!
    p = __builtin_fmaf(p, x2, -1.6666667e-1f);                       // -1/3!
    return __builtin_fmaf(x * x2, p, x);
}

// the cutoff sum (SynthVoice.h:46-47) clamped as Svf::SetFreq clamps it, fclamp(f, 1e-6, sr / 3):
// fminf(fmaxf(f, 1e-6), fc_max) for 1e-6 <= fc_max and a non-NaN sum (ENV hands it to FREQ clamped:
// the ENV + FILT SIMDs had the spare issue slots)
__device__ __forceinline__ float svf_fc(float f, float fc_max) { return __builtin_amdgcn_fmed3f(f, 1.0e-6f, fc_max); }

// Svf::SetFreq's damping, negated for FILT: -min(damp_res, min(2, lim)) = max(-damp_res, -2, -lim),
// one v_max3 (the negations are operand modifiers); equal for every non-NaN lim
__device__ __forceinline__ float neg_damp(float damp_res, float lim) {
    return __builtin_fmaxf(__builtin_fmaxf(-damp_res, -2.0f), -lim);
}

// packed FP32 (v_pk_mul_f32 / v_pk_add_f32: two IEEE operations per lane and instruction, the same
// bits as two scalar ones)
typedef float f2 __attribute__((ext_vector_type(2)));

struct Ladder {
    float z0[4], z1[4], old;
};

// The block's folded note events (VoiceArgs::ev, VEV_*) of this lane's voice: the wave reads its
// workgroup's fixed slots (lanes 0 .. kVevCap-1, one host-link round trip; a crowded workgroup's
// overflow list is a second one), stages the records into its own 64 LDS slots, slot = voice within
// the group, and each lane reads its own.  `me` is the lane's voice within the group (dead lanes of
// the last group mirror voice n-1, so they read its slot too).  No events: one uniform test.
struct VoiceEv {
    uint32_t op;
    float freq;
};
__device__ __forceinline__ VoiceEv voice_event(const VoiceArgs &a, uint2 *slot, uint32_t lane, uint32_t me) {
    VoiceEv r{0u, 0.0f};
    if (!a.ev) return r;
    uint2 e = make_uint2(0u, 0u);
    if (lane < kVevCap) e = a.ev[blockIdx.x * kVevCap + lane];
    slot[lane] = make_uint2(0u, 0u);
    const uint32_t head = __builtin_amdgcn_readfirstlane(e.x);
    if ((head >> 8) & VEV_MORE) {
        const uint32_t cnt = head >> 16, first = __builtin_amdgcn_readfirstlane(e.y);
        e = make_uint2(0u, 0u);
        if (lane < cnt) e = a.ev_more[first + lane];
    }
    if (e.x >> 8) slot[e.x & 63u] = make_uint2(e.x >> 8, e.y);
    // one wave writes and reads its slots: LDS operations of a wave complete in order; the fences
    // keep the compiler from moving the read above the other lanes' writes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const uint2 v = slot[me];
    r.op = v.x;
    r.freq = __uint_as_float(v.y);
    return r;
}

// Another wave's view of slots voice_event staged, after a workgroup barrier.
__device__ __forceinline__ VoiceEv staged_event(const VoiceArgs &a, const uint2 *slot, uint32_t me) {
    VoiceEv r{0u, 0.0f};
    if (!a.ev) return r;
    const uint2 v = slot[me];
    r.op = v.x;
    r.freq = __uint_as_float(v.y);
    return r;
}

// NoteOn / GateOn / NoteOff / GateOff on the envelope flags word and levels (SynthVoice.h:231-251):
// Retrigger(true) = mode ATTACK and x = 0 for the amp (bits 0-2) and filter (bits 3-5) envelopes;
// the gate is bit 8
__device__ __forceinline__ void apply_gate_events(const VoiceEv &ev, uint32_t &flags, float &xa, float &xf) {
    if (ev.op & VEV_RETRIGGER) {
        flags = (flags & ~0x3Fu) | 1u | (1u << 3);
        xa = 0.0f;
        xf = 0.0f;
    }
    if (ev.op & VEV_GATE_SET) flags = (flags & ~0x100u) | ((ev.op & VEV_GATE_ON) ? 0x100u : 0u);
}

}  // namespace

// daisysp::Adsr as a segment machine.  The gate is constant inside a block (note events apply
// between blocks), so the gate-edge test of Adsr::Process only fires on the block's first sample:
// it is applied once in begin(), and each sample is the segment update x += d0 (target - x)
// followed by the segment's clamp -- ATTACK ends above 1 (-> DECAY at x = 1), DECAY / RELEASE end
// below 0 (-> IDLE at x = 0) -- which is v_med3(xn, lo, hi) with the segment's (lo, hi).  The
// segment ends in a lane only a few times per note, so the parameter switch runs behind a
// wave-uniform test.  IDLE is d0 = 0, target 0 and no bounds: x stays 0, Adsr's IDLE output (x is 0
// whenever the envelope is idle: it enters IDLE at 0 and leaves only through Retrigger).
struct Env {
    float x, d0, tgt, hi, lo;
    uint32_t mode;
    float dec_d0, sus;

    __device__ __forceinline__ void set_segment(uint32_t m, float atk_d0, float atk_tgt, float rel_d0) {
        const float inf = __builtin_inff();
        const bool atk = m == SEG_ATTACK, dcy = m == SEG_DECAY, rel = m == SEG_RELEASE;
        mode = m;
        d0 = atk ? atk_d0 : (dcy ? dec_d0 : (rel ? rel_d0 : 0.0f));
        tgt = atk ? atk_tgt : (dcy ? sus : (rel ? -0.01f : 0.0f));
        hi = atk ? 1.0f : inf;
        lo = (dcy || rel) ? 0.0f : -inf;
    }
    __device__ __forceinline__ void begin(bool gate, bool &gprev, uint32_t m, float x0, float atk_d0, float atk_tgt,
                                          float dec, float rel_d0, float s) {
        m = (gate && !gprev) ? (uint32_t)SEG_ATTACK : ((!gate && gprev) ? (uint32_t)SEG_RELEASE : m);
        gprev = gate;
        x = x0;
        dec_d0 = dec;
        sus = s;
        set_segment(m, atk_d0, atk_tgt, rel_d0);
    }
    // the same update with no segment switch, for a chunk computed speculatively: returns the
    // sample and records in `ended` whether the segment ended (then the chunk is redone by step())
    __device__ __forceinline__ float step_spec(bool &ended) {
        const float xn = x + d0 * (tgt - x);
        ended = ended || xn > hi || xn < lo;
        x = xn;                                          // == v_med3(xn, lo, hi) while inside
        return x;
    }
    __device__ __forceinline__ float step() {
        const float xn = x + d0 * (tgt - x);
        const bool ends = xn > hi || xn < lo;
        x = __builtin_amdgcn_fmed3f(xn, lo, hi);
        if (__builtin_amdgcn_ballot_w64(ends)) {       // rare, wave-uniform: a segment ended
            // every lane evaluates the switch and keeps it only where its segment ended (selects,
            // no exec-masked block)
            const float inf = __builtin_inff();
            const bool to_dcy = mode == SEG_ATTACK;
            d0 = ends ? (to_dcy ? dec_d0 : 0.0f) : d0;
            tgt = ends ? (to_dcy ? sus : 0.0f) : tgt;
            hi = ends ? inf : hi;
            lo = ends ? (to_dcy ? 0.0f : -inf) : lo;
            mode = ends ? (to_dcy ? (uint32_t)SEG_DECAY : (uint32_t)SEG_IDLE) : mode;
        }
        return x;
    }
};

// samples per hand-off between the roles: 8 (34 barrier steps per 256-frame block, pipeline fill
// 2 of them) measured 2 % faster than 16 (18 steps) for the Svf voice and equal for the Moog
// voice; 32 halves the workgroups per CU (96 KB of LDS each) and is 1.7x slower
constexpr int kVcChunk = 8;

// Runs f(j) for the m samples of a chunk: unrolled when the chunk is full, so the off-recurrence
// work of neighbouring samples interleaves (ILP for a wave that is alone on its SIMD).
template <class F>
__device__ __forceinline__ void for_chunk(uint32_t m, F &&f) {
    if (m == (uint32_t)kVcChunk) {
#pragma unroll
        for (uint32_t j = 0; j < (uint32_t)kVcChunk; ++j) f(j);
    } else {
        for (uint32_t j = 0; j < m; ++j) f(j);
    }
}

// voice_block_v4: the MoogFilter voice.  One workgroup = 64 voices, the voice pipelined over two
// waves that hand each sample's values on through an LDS double buffer (one barrier per 8-sample
// chunk):
//   feed wave   : amp envelope, portamento, oscillator, filter envelope, cutoff,
//                 LadderFilter::SetFreq -> SetAlpha          -> (src * drive, amp, alpha, Qadjust)
//   filter wave : LadderFilter::Process, output store
// The ladder's serial recurrence dominates the voice, so the feed roles share one wave.  (The Svf
// voice runs voice_block_v5 below, over four role waves.)
__global__ __launch_bounds__(128) void voice_block_v4(VoiceArgs a) {
    constexpr uint32_t kRoles = 2u;
    __shared__ float4 q[2][kVcChunk][64];
    __shared__ uint32_t fflags[64];
    __shared__ uint2 evslot[64];
    const uint32_t n = a.n;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t i0 = blockIdx.x * 64 + lane;
    // dead lanes of the last workgroup mirror voice n-1 exactly (same state, same coefficients,
    // same events), so their stores write the values voice n-1's lane writes
    const uint32_t i = i0 < n ? i0 : n - 1;
    const uint32_t me = i - blockIdx.x * 64;
    const uint32_t nf = a.n_frames;
    const uint32_t nchunks = (nf + kVcChunk - 1) / kVcChunk;
    const float *c = a.coef;
    float *s = a.state;
    const bool filt_role = wave == kRoles - 1;

    // ---------------- amp and/or cutoff roles (compile-time role flags: straight-line chunks) ----------------
    auto feed = [&](auto amp_c, auto cut_c) {
        constexpr bool AMP = decltype(amp_c)::value, CUT = decltype(cut_c)::value;
        // the block's note events first (one feed wave per workgroup applies them); the state loads
        // are issued before the event read, so their latency hides under its host-link round trip
        uint32_t flags0 = __float_as_uint(s[VCS_FLAGS * n + i]);
        float xa0 = s[VCS_ENVA_X * n + i], xf0 = s[VCS_ENVF_X * n + i];
        const float freq_s = s[VCS_FREQ * n + i];
        const VoiceEv ev = voice_event(a, evslot, lane, me);
        apply_gate_events(ev, flags0, xa0, xf0);
        const bool gate = (flags0 >> 8) & 1u;
        const float amp_amt = c[VCC_AMP_AMT * n + i], port_c = c[VCC_PORT_COEF * n + i];
        const float inv_sr = c[VCC_INV_SR * n + i];
        const float freq = (ev.op & VEV_FREQ) ? ev.freq : freq_s;
        const float cutoff = c[VCC_CUTOFF * n + i], fenv_amt = c[VCC_FENV_AMT * n + i];
        // ladder: drive_scaled (VCC_DRIVE), 1/(4 sr) (VCC_FC_MAX)
        const float drive = c[VCC_DRIVE * n + i];
        const float fc_max = c[VCC_FC_MAX * n + i];
        float phase = s[VCS_PHASE * n + i];
        float port_z = s[VCS_PORT_Z * n + i];
        bool gprev_a = (flags0 >> 6) & 1u, gprev_f = (flags0 >> 7) & 1u;
        Env ea, ef;
        if constexpr (AMP)
            ea.begin(gate, gprev_a, flags0 & 7u, xa0, c[VCC_ATK_D0A * n + i],
                     c[VCC_ATK_TGT_A * n + i], c[VCC_DEC_D0A * n + i], c[VCC_REL_D0A * n + i], c[VCC_SUS_A * n + i]);
        if constexpr (CUT)
            ef.begin(gate, gprev_f, (flags0 >> 3) & 7u, xf0, c[VCC_ATK_D0F * n + i],
                     c[VCC_ATK_TGT_F * n + i], c[VCC_DEC_D0F * n + i], c[VCC_REL_D0F * n + i], c[VCC_SUS_F * n + i]);

        for (uint32_t k = 0; k <= nchunks; ++k) {
            if (k < nchunks) {
                const uint32_t f0 = k * kVcChunk;
                const uint32_t m = nf - f0 < (uint32_t)kVcChunk ? nf - f0 : (uint32_t)kVcChunk;
                float4 *qb = &q[k & 1][0][lane];
                for_chunk(m, [&](uint32_t j) {
                    float2 ab, cd;
                    if constexpr (AMP) {
                        const float amp = ea.step() * amp_amt;
                        // Port::Process (Portamento.h:218-221), Oscillator::SetFreq: inc = f * sr_recip
                        port_z = freq + port_c * (port_z - freq);
                        const float inc = port_z * inv_sr;
                        // Oscillator::Process, WAVE_POLYBLEP_SAW
                        const float src = saw_out(phase, polyblep(inc, phase));
                        phase += inc;
                        phase = phase > 1.0f ? phase - 1.0f : phase;
                        ab = make_float2(src * drive, amp);   // ladder: Process's input scaling
                    }
                    if constexpr (CUT) {
                        const float fe = ef.step();
                        const float fc_in = __builtin_fmaf(fe * 20000.0f, fenv_amt, cutoff);
                        const float wc = fc_in * 2.0f * 3.1415927410125732f * fc_max;
                        const float wc2 = wc * wc;
                        // the same polynomials in Horner form
                        cd.x = wc * __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(-0.0202f, wc, 0.1381f), wc, -0.4324f), wc, 0.9892f);
                        cd.y = __builtin_fmaf(__builtin_fmaf(-0.05f, wc2, -0.095f), wc2, __builtin_fmaf(0.0536f, wc, 1.006f));
                    }
                    if constexpr (AMP && CUT) {
                        qb[j * 64] = make_float4(ab.x, ab.y, cd.x, cd.y);
                    } else if constexpr (AMP) {
                        reinterpret_cast<float2 *>(&qb[j * 64])[0] = ab;
                    } else {
                        reinterpret_cast<float2 *>(&qb[j * 64])[1] = cd;
                    }
                });
            }
            __syncthreads();
        }
        // the flags word holds both envelopes: the cutoff role hands its bits to the amp role
        if constexpr (CUT && !AMP) fflags[lane] = ef.mode << 3 | (uint32_t)gprev_f << 7;
        __syncthreads();
        if constexpr (AMP) {
            const uint32_t fbits = CUT ? (ef.mode << 3 | (uint32_t)gprev_f << 7) : fflags[lane];
            s[VCS_PHASE * n + i] = phase;
            s[VCS_PORT_Z * n + i] = port_z;
            s[VCS_ENVA_X * n + i] = ea.x;
            s[VCS_FLAGS * n + i] = __uint_as_float(ea.mode | fbits | (uint32_t)gprev_a << 6 | (uint32_t)gate << 8);
            if (ev.op & VEV_FREQ) s[VCS_FREQ * n + i] = freq;
        }
        if constexpr (CUT) s[VCS_ENVF_X * n + i] = ef.x;
    };
    if (!filt_role) {
        feed(std::true_type{}, std::true_type{});
    } else {
        // ---------------- filter role: LadderFilter::Process ----------------
        const float k_or_unused = c[VCC_DAMP_RES * n + i];     // ladder: K (VCC_LADDER_K)
        Ladder L;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            L.z0[k] = s[(VCS_LZ0 + k) * n + i];
            L.z1[k] = s[(VCS_LZ1 + k) * n + i];
        }
        L.old = s[VCS_LOLD * n + i];
        float *out = a.out + i;
        for (uint32_t k = 0; k <= nchunks; ++k) {
            if (k > 0) {
                const uint32_t f0 = (k - 1) * kVcChunk;
                const uint32_t m = nf - f0 < (uint32_t)kVcChunk ? nf - f0 : (uint32_t)kVcChunk;
                const float4 *qb = &q[(k - 1) & 1][0][lane];
                for_chunk(m, [&](uint32_t j) {
                    const float4 v = qb[j * 64];
                    float y;
                    {
                        // contracted (see Contraction above); the Pade tanh as r(med3(x, -3, 3))
                        // (r(+-3) = +-1 exactly: the saturation, branch-free) with a hardware
                        // reciprocal
                        const float input = v.x, alpha = v.z, kq = k_or_unused * v.w;
                        const float fb0 = -0.5f * input, dold = L.old - input;
                        float total = 0.0f;
#pragma unroll
                        for (int os = 0; os < 4; ++os) {
                            const float interp = 0.25f * (float)os;
                            // the linear interpolation interp old + (1 - interp) input as
                            // input + interp (old - input): one fma per oversample (os = 0: input)
                            const float mixin = os == 0 ? input : __builtin_fmaf(interp, dold, input);
                            float x = __builtin_fmaf(-(L.z1[3] + fb0), kq, mixin);
                            x = __builtin_amdgcn_fmed3f(x, -3.0f, 3.0f);
                            const float x2 = x * x;
                            float u = (x * (27.0f + x2)) * __builtin_amdgcn_rcpf(__builtin_fmaf(9.0f, x2, 27.0f));
#pragma unroll
                            for (int st = 0; st < 4; ++st) {
                                float ft = __builtin_fmaf(u, 1.0f / 1.3f, __builtin_fmaf(0.3f / 1.3f, L.z0[st], -L.z1[st]));
                                ft = __builtin_fmaf(ft, alpha, L.z1[st]);
                                L.z1[st] = ft;
                                L.z0[st] = u;
                                u = ft;
                            }
                            total = __builtin_fmaf(u, 0.25f, total);
                        }
                        L.old = input;
                        y = total * v.y;
                    }
                    out[(size_t)(f0 + j) * n] = y;
                });
            }
            __syncthreads();
        }
        __syncthreads();                                      // the flags hand-off barrier
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s[(VCS_LZ0 + k) * n + i] = L.z0[k];
            s[(VCS_LZ1 + k) * n + i] = L.z1[k];
        }
        s[VCS_LOLD * n + i] = L.old;
    }
}

// ---------------------------------------------------------------------------------------------
// voice_block_v5 (SvfFilter voices): v4's arithmetic, operation for operation, over
// FOUR role waves per workgroup of 64 voices (two workgroups per CU, two waves per SIMD):
//   ENV  : the amp and filter Adsr, the cutoff sum, its clamp                 -> (amp, fc)
//   OSC  : Port, the oscillator's phase, the polyBLEP saw                     -> src
//   FREQ : Svf::SetFreq(fc_in)                                                -> (-damp, fq)
//   FILT : the two Svf passes, Low() * amp, the output store
// A three-stage pipeline over 8-sample chunks (kVcChunk): at step k ENV makes chunk k, OSC and FREQ chunk
// k-1, FILT chunk k-2 (and reads that chunk's amp straight from ENV's queue, which holds three
// chunks); one barrier per step; 24 KB of LDS per workgroup.  Measured per role (16-sample chunks,
// 18 steps; the others skipping their arithmetic): the skeleton (launch, state,
// 18 barriers) 9.7 us, FREQ 10.0, FILT 15, OSC 20, ENV 26 of the kernel's 43.6 us.  The envelopes
// of a full chunk run speculatively (Env::step_spec, no per-sample lane vote and branch) and the
// chunk is redone exactly when a lane's segment ended in it.  Roles are assigned by SIMD (below).
// ---------------------------------------------------------------------------------------------
// FILT (the Svf recurrence, the critical chain of the ENV + FILT pair) issues ahead of ENV on
// their SIMD at wave priority 2: ~2 % same-box; OSC raised too was slower.
__global__ __launch_bounds__(256) void voice_block_v5(VoiceArgs a) {
    __shared__ float2 eq[3][kVcChunk][64];      // ENV -> OSC, FREQ (fc_in), FILT (amp): three chunks live
    __shared__ float sq[2][kVcChunk][64];       // OSC -> FILT: src
    __shared__ float2 fdq[2][kVcChunk][64];     // FREQ -> FILT: (-damp, fq)
    __shared__ uint2 evslot[64];                // ENV's staging of the block's events (OSC reads it)
    __shared__ uint32_t hw_simd[5];             // the SIMD of each wave; [4]: wave 0's slot parity
    const uint32_t n = a.n;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // Roles by SIMD.  The roles' VALU loads differ (per 8-sample chunk FILT ~218, OSC ~190, FREQ
    // ~159, ENV ~111 instructions) and the two co-resident workgroups of a CU put wave w on the
    // same SIMD, so role = wave stacks two FILTs on one SIMD.  Each wave reads its SIMD (HW_ID
    // bits 5:4) and slot (bits 3:0); a workgroup whose wave 0 sits in an odd slot takes the roles in
    // mirrored SIMD order, pairing ENV with FILT and OSC with FREQ on every SIMD.  Waves that do
    // not sit on four distinct SIMDs keep role = wave (any assignment is correct; this one only
    // balances).
    {
        const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));   // HW_REG_HW_ID
        if (lane == 0) {
            hw_simd[wave] = (hw >> 4) & 3u;
            if (wave == 0) hw_simd[4] = hw & 1u;
        }
    }
    __syncthreads();
    uint32_t role = wave;
    {
        const uint32_t m = (1u << hw_simd[0]) | (1u << hw_simd[1]) | (1u << hw_simd[2]) | (1u << hw_simd[3]);
        const uint32_t sm = hw_simd[wave];
        if (m == 15u) role = hw_simd[4] ? 3u - sm : sm;
        role = __builtin_amdgcn_readfirstlane(role);
    }
    // the role with the per-sample recurrence (FILT) ahead of its SIMD partner at issue
    if (role == 3u) __builtin_amdgcn_s_setprio(2);
    const uint32_t i0 = blockIdx.x * 64 + lane;
    const uint32_t i = i0 < n ? i0 : n - 1;      // dead lanes mirror voice n-1, as in v4
    const uint32_t me = i - blockIdx.x * 64;
    const uint32_t nf = a.n_frames;
    const uint32_t nsteps = (nf + kVcChunk - 1) / kVcChunk + 2;
    const float *c = a.coef;
    float *s = a.state;
    auto len = [&](uint32_t k) {             // frames of chunk k (the last may be short)
        const uint32_t f0 = k * kVcChunk;
        return nf - f0 < (uint32_t)kVcChunk ? nf - f0 : (uint32_t)kVcChunk;
    };

    if (role == 0) {
        // ---- ENV (SynthVoice.h:42,46-47): the amp and filter Adsr, the cutoff sum ----
        // the block's gate events first (NoteOn / GateOn / NoteOff / GateOff); the state loads are
        // issued before the event read, so their latency hides under its host-link round trip
        uint32_t flags0 = __float_as_uint(s[VCS_FLAGS * n + i]);
        float xa0 = s[VCS_ENVA_X * n + i], xf0 = s[VCS_ENVF_X * n + i];
        const VoiceEv ev = voice_event(a, evslot, lane, me);
        apply_gate_events(ev, flags0, xa0, xf0);
        const bool gate = (flags0 >> 8) & 1u;
        bool gprev_a = (flags0 >> 6) & 1u, gprev_f = (flags0 >> 7) & 1u;
        const float amp_amt = c[VCC_AMP_AMT * n + i], fc_max = c[VCC_FC_MAX * n + i];
        const float amp_half = 0.5f * amp_amt;       // FILT's Low() halving folded in (exact scaling)
        const float cutoff = c[VCC_CUTOFF * n + i], fenv_amt = c[VCC_FENV_AMT * n + i];
        Env ea, ef;
        ea.begin(gate, gprev_a, flags0 & 7u, xa0, c[VCC_ATK_D0A * n + i],
                 c[VCC_ATK_TGT_A * n + i], c[VCC_DEC_D0A * n + i], c[VCC_REL_D0A * n + i], c[VCC_SUS_A * n + i]);
        ef.begin(gate, gprev_f, (flags0 >> 3) & 7u, xf0, c[VCC_ATK_D0F * n + i],
                 c[VCC_ATK_TGT_F * n + i], c[VCC_DEC_D0F * n + i], c[VCC_REL_D0F * n + i], c[VCC_SUS_F * n + i]);
        for (uint32_t k = 0; k < nsteps; ++k) {
            if (k + 2 < nsteps) {
                float2 *qo = &eq[k % 3][0][lane];
                if (len(k) == (uint32_t)kVcChunk) {
                    // Full chunk: the envelopes run speculatively with no per-sample segment test
                    // (a branch on a lane vote per sample serialised the chunk); if any lane's
                    // segment ended inside the chunk -- a few chunks per note -- the chunk is
                    // redone sample by sample from its start with the exact segment machine.
                    const float xa0 = ea.x, xf0 = ef.x;
                    bool ended = false;
                    // both envelopes' Env::step_spec in packed operations (the pair lives in a
                    // register pair for the chunk), then (x_a amp_amt, x_f 20000)
                    f2 X = {ea.x, ef.x};
                    const f2 D0 = {ea.d0, ef.d0}, T = {ea.tgt, ef.tgt}, AMT = {amp_half, 20000.0f};
#pragma unroll
                    for (uint32_t j = 0; j < (uint32_t)kVcChunk; ++j) {
                        X = X + D0 * (T - X);
                        const f2 m = X * AMT;
                        qo[j * 64] = make_float2(m.x, svf_fc(__builtin_fmaf(m.y, fenv_amt, cutoff), fc_max));
                    }
                    // inside a segment the envelope is monotone toward a target beyond its bound
                    // (x += d0 (tgt - x) with tgt - x of one sign: each IEEE step keeps the
                    // direction), so it crossed the bound inside the chunk iff it ends past it
                    ended = X.x > ea.hi || X.x < ea.lo || X.y > ef.hi || X.y < ef.lo;
                    ea.x = X.x;
                    ef.x = X.y;
                    if (__builtin_amdgcn_ballot_w64(ended)) {
                        ea.x = xa0;
                        ef.x = xf0;
                        for (uint32_t j = 0; j < (uint32_t)kVcChunk; ++j) {
                            const float amp = ea.step() * amp_half;
                            const float fe = ef.step();
                            qo[j * 64] = make_float2(amp, svf_fc(__builtin_fmaf(fe * 20000.0f, fenv_amt, cutoff), fc_max));
                        }
                    }
                } else {
                    for_chunk(len(k), [&](uint32_t j) {
                        const float amp = ea.step() * amp_half;
                        const float fe = ef.step();
                        qo[j * 64] = make_float2(amp, svf_fc(__builtin_fmaf(fe * 20000.0f, fenv_amt, cutoff), fc_max));
                    });
                }
            }
            __syncthreads();
        }
        s[VCS_ENVA_X * n + i] = ea.x;
        s[VCS_ENVF_X * n + i] = ef.x;
        s[VCS_FLAGS * n + i] = __uint_as_float(ea.mode | ef.mode << 3 | (uint32_t)gprev_a << 6 |
                                               (uint32_t)gprev_f << 7 | (uint32_t)gate << 8);
    } else if (role == 1) {
        // ---- OSC (SynthVoice.h:44-45): Port::Process, Oscillator::SetFreq / Process, WAVE_POLYBLEP_SAW,
        //      amp 0.5 ----
        const float port_c = c[VCC_PORT_COEF * n + i];
        const float inv_sr = c[VCC_INV_SR * n + i];
        float freq = s[VCS_FREQ * n + i];
        float phase = s[VCS_PHASE * n + i], port_z = s[VCS_PORT_Z * n + i];
        for (uint32_t k = 0; k < nsteps; ++k) {
            if (k == 1) {
                // the block's pitch events (NoteOn: mtof(note), SetFrequency: Hz), staged by ENV
                // before the first barrier; OSC's first chunk is step 1
                const VoiceEv ev = staged_event(a, evslot, me);
                if (ev.op & VEV_FREQ) {
                    freq = ev.freq;
                    s[VCS_FREQ * n + i] = freq;
                }
            }
            if (k >= 1 && k + 1 < nsteps) {
                float *qo = &sq[(k - 1) & 1][0][lane];
                if (len(k - 1) == (uint32_t)kVcChunk) {
                    // only Port and the phase are recurrences: run them for the chunk, then the
                    // polyBLEP saw per sample over four packed sample pairs (stage by stage, as FREQ)
                    constexpr int P = kVcChunk / 2;
                    f2 t[P], dt[P];
#pragma unroll
                    for (int q = 0; q < P; ++q) {
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            port_z = freq + port_c * (port_z - freq);     // Port::Process (Portamento.h:218-221)
                            const float inc = port_z * inv_sr;             // Oscillator::SetFreq
                            t[q][h] = phase;                               // Oscillator::Process reads, then advances
                            dt[q][h] = inc;
                            phase += inc;
                            phase = phase > 1.0f ? phase - 1.0f : phase;
                        }
                    }
                    f2 num[P], qv[P], qq[P], rlo[P], rhi[P], o[P];
                    bool lo[P][2], hi[P][2];
#pragma unroll
                    for (int q = 0; q < P; ++q) {
                        const f2 one_m = 1.0f - dt[q];
                        const f2 tm1 = t[q] - 1.0f;
#pragma unroll
                        for (int h = 0; h < 2; ++h) {
                            lo[q][h] = t[q][h] < dt[q][h];
                            hi[q][h] = t[q][h] > one_m[h];          // (lo wins the selects below)
                            num[q][h] = lo[q][h] ? t[q][h] : tm1[h];
                        }
                    }
#pragma unroll
                    for (int q = 0; q < P; ++q)
                        qv[q] = num[q] * (f2){__builtin_amdgcn_rcpf(dt[q].x), __builtin_amdgcn_rcpf(dt[q].y)};
                    // q + q - q q - 1 and q q + q + q + 1 as fma(-q, q, 2q) - 1 and fma(q, q, 2q) + 1
#pragma unroll
                    for (int q = 0; q < P; ++q) qq[q] = qv[q] + qv[q];
#pragma unroll
                    for (int q = 0; q < P; ++q) {
                        rlo[q] = __builtin_elementwise_fma(-qv[q], qv[q], qq[q]);
                        rhi[q] = __builtin_elementwise_fma(qv[q], qv[q], qq[q]);
                    }
#pragma unroll
                    for (int q = 0; q < P; ++q) { rlo[q] = rlo[q] - 1.0f; rhi[q] = rhi[q] + 1.0f; o[q] = 0.5f - t[q]; }
#pragma unroll
                    for (int q = 0; q < P; ++q) {
                        f2 blep;
#pragma unroll
                        for (int h = 0; h < 2; ++h) blep[h] = lo[q][h] ? rlo[q][h] : (hi[q][h] ? rhi[q][h] : 0.0f);
                        // -((2t - 1) - blep) / 2 as fma(1/2, blep, 1/2 - t): 2t - 1 = 2 (t - 1/2) and the
                        // halving are exact, so both round the same sum once (saw_out below)
                        const f2 y = __builtin_elementwise_fma((f2)0.5f, blep, o[q]);
                        qo[(2 * q) * 64] = y.x;
                        qo[(2 * q + 1) * 64] = y.y;
                    }
                } else {
                    for (uint32_t j = 0; j < len(k - 1); ++j) {
                        port_z = freq + port_c * (port_z - freq);
                        const float inc = port_z * inv_sr;
                        const float t = phase;
                        phase += inc;
                        phase = phase > 1.0f ? phase - 1.0f : phase;
                        qo[j * 64] = saw_out(t, polyblep(inc, t));
                    }
                }
            }
            __syncthreads();
        }
        s[VCS_PHASE * n + i] = phase;
        s[VCS_PORT_Z * n + i] = port_z;
    } else if (role == 2) {
        // ---- FREQ: Svf::SetFreq (its divisions use the hardware reciprocal, as in v4) ----
        const float damp_res = c[VCC_DAMP_RES * n + i];
        const float inv_2sr = 1.0f / (c[VCC_SR * n + i] * 2.0f);
        for (uint32_t k = 0; k < nsteps; ++k) {
            if (k >= 1 && k + 1 < nsteps) {
                const float2 *qi = &eq[(k - 1) % 3][0][lane];
                float2 *qo = &fdq[(k - 1) & 1][0][lane];
                // hands FILT (-damp, fq): its notch src - damp band is src + (-damp) band, exactly
                if (len(k - 1) == (uint32_t)kVcChunk) {
                    // no recurrence here: two samples per packed operation, the chunk's four pairs
                    // stage by stage (a packed result read by the next instruction costs a wait
                    // state; four independent pairs fill them)
                    constexpr int P = kVcChunk / 2;
                    f2 x[P], x2[P], pp[P], fq[P], sq[P];
#pragma unroll
                    for (int q = 0; q < P; ++q) {
                        const float c0 = qi[(2 * q) * 64].y;          // clamped by ENV (svf_fc)
                        const float c1 = qi[(2 * q + 1) * 64].y;
                        const f2 fcn = (f2){c0, c1} * inv_2sr;
                        const f2 arg = {__builtin_fminf(fcn.x, 0.25f), __builtin_fminf(fcn.y, 0.25f)};
                        x[q] = 3.1415927410125732f * arg;
                    }
#pragma unroll
                    for (int q = 0; q < P; ++q) x2[q] = x[q] * x[q];
#pragma unroll
                    for (int q = 0; q < P; ++q) pp[q] = __builtin_elementwise_fma((f2)2.7557319e-6f, x2[q], (f2)-1.9841270e-4f);
#pragma unroll
                    for (int q = 0; q < P; ++q) pp[q] = __builtin_elementwise_fma(pp[q], x2[q], (f2)8.3333333e-3f);
#pragma unroll
                    for (int q = 0; q < P; ++q) pp[q] = __builtin_elementwise_fma(pp[q], x2[q], (f2)-1.6666667e-1f);
#pragma unroll
                    for (int q = 0; q < P; ++q) x2[q] = x[q] * x2[q];
#pragma unroll
                    for (int q = 0; q < P; ++q) sq[q] = __builtin_elementwise_fma(x2[q], pp[q], x[q]);   // sin(x); fq = 2 sin
#pragma unroll
                    for (int q = 0; q < P; ++q) {
                        const f2 rq = {__builtin_amdgcn_rcpf(sq[q].x), __builtin_amdgcn_rcpf(sq[q].y)};
                        // 2 / fq - fq / 2 = 1 / s - s: one subtraction (and the reciprocal of s, not of 2 s)
                        const f2 lim = rq - sq[q];
                        fq[q] = sq[q] + sq[q];
                        qo[(2 * q) * 64] = make_float2(neg_damp(damp_res, lim.x), fq[q].x);
                        qo[(2 * q + 1) * 64] = make_float2(neg_damp(damp_res, lim.y), fq[q].y);
                    }
                } else {
                    for (uint32_t j = 0; j < len(k - 1); ++j) {
                        const float fc = qi[j * 64].y;
                        const float fcn = fc * inv_2sr;
                        const float arg = __builtin_fminf(fcn, 0.25f);
                        const float s1 = sin_quarter(3.1415927410125732f * arg), fq = s1 + s1;
                        const float lim = __builtin_amdgcn_rcpf(s1) - s1;
                        qo[j * 64] = make_float2(neg_damp(damp_res, lim), fq);
                    }
                }
            }
            __syncthreads();
        }
    } else {
        // ---- FILT: Svf::Process; Low() = the average of the two passes' low outputs; * amp ----
        const float drive = c[VCC_DRIVE * n + i];
        float low = s[VCS_LOW * n + i], band = s[VCS_BAND * n + i];
        for (uint32_t k = 0; k < nsteps; ++k) {
            if (k >= 2) {
                const uint32_t f0 = (k - 2) * kVcChunk;
                // the chunk's output rows through a buffer resource based at row f0: the row offset
                // j n 4 is a scalar (soffset), so a store costs no vector address arithmetic
                const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
                    a.out + (size_t)f0 * n, (short)0, (int)((uint32_t)kVcChunk * n * 4u), 0x00020000);
                const float *qs = &sq[k & 1][0][lane];         // chunk k-2: (k-2) & 1 == k & 1
                const float2 *qa = &eq[(k - 2) % 3][0][lane];
                const float2 *qf = &fdq[k & 1][0][lane];
                for_chunk(len(k - 2), [&](uint32_t j) {
                    const float2 fd = qf[j * 64];
                    const float2 sa = make_float2(qs[j * 64], qa[j * 64].x);
                    // (packing this serial recurrence's paired products cost as many register
                    // moves as it saved operations: scalar)
                    const float src = sa.x, ndamp = fd.x, fq = fd.y;     // FREQ hands over -damp
                    // contracted except the notch (see Contraction above)
                    float notch = src + ndamp * band;
                    low = __builtin_fmaf(fq, band, low);
                    float high = notch - low;
                    band = __builtin_fmaf(-((drive * band) * band), band, __builtin_fmaf(fq, high, band));
                    const float low1 = low;
                    notch = src + ndamp * band;
                    low = __builtin_fmaf(fq, band, low);
                    high = notch - low;
                    band = __builtin_fmaf(-((drive * band) * band), band, __builtin_fmaf(fq, high, band));
                    // Low() = 0.5 low1 + 0.5 low2, times amp: (low1 + low2) (amp / 2), the same rounding (halvings exact)
                    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint((low1 + low) * sa.y), ro, i * 4u, j * n * 4u, 0);
                });
            }
            __syncthreads();
        }
        s[VCS_LOW * n + i] = low;
        s[VCS_BAND * n + i] = band;
    }
}

hipError_t launch_voice(const VoiceArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    if ((uint64_t)kVcChunk * a.n * 4u > 0xFFFFFFFFull) return hipErrorInvalidValue;   // v5's chunk output resource
    const dim3 grid((a.n + 63) / 64);     // 64 voices per workgroup, one wave per role
    if (a.moog) hipLaunchKernelGGL(voice_block_v4, grid, dim3(128), 0, s, a);
    else hipLaunchKernelGGL(voice_block_v5, grid, dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
