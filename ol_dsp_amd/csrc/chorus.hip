// ol_dsp_amd/csrc/chorus.hip -- RNBO stereo chorus and gen~ pitch-shifter, one lane per instance.
//
// Spec (no executable oracle exists in the reference, parity "unpinned"):
//   mono-chorus.rnbopat: y = (1-mix) x + mix * lores~( delay~( pitchshift(x, pitch),
//                                                   D cycle~(rate_hz, phase) + D ), cutoff_hz, q )
//   pitchshift.gendsp / gencode at mono-chorus.rnbopat:962:
//       p0 = phasor(shift), p1 = (p0 + 0.5) % 1, W = mstosamps(window)
//       out = read(p1 W) cos((p1-.5)pi) + read(p0 W) cos((p0-.5)pi);  write(x) after the reads
//   stereo-chorus.rnbopat: L and R are two mono-chorus instances with shared params; L phase 1 and
//   R phase 0 are the same phase after wrap, so one LFO serves both channels.
//
// Layout: each instance owns contiguous rings [2][psize] (pitch) and [2][csize] (chorus); the
// read taps are modulated per instance, so a lane streams through its own ring and consecutive
// frames hit the same cache lines.  Stream time (write position) is shared by all instances.
#include "olfx_internal.h"

namespace olfx {

namespace {

__device__ __forceinline__ float unit24(uint32_t acc) {
    return (float)(acc >> 8) * 5.9604644775390625e-8f;   // exact: 24-bit fraction in [0,1)
}

// linear-interpolated read at fractional delay d (clamped to [dmin, dmax]) behind write pos w
__device__ __forceinline__ float read_frac(const float *ring, uint32_t mask, uint32_t w, float d,
                                           float dmin, float dmax) {
    d = fminf(fmaxf(d, dmin), dmax);
    const uint32_t di = (uint32_t)d;
    const float fr = d - (float)di;
    const float x0 = ring[(w - di) & mask];
    const float x1 = ring[(w - di - 1u) & mask];
    return x0 + fr * (x1 - x0);
}

}  // namespace

__global__ __launch_bounds__(256) void chorus_block_v1(ChorusArgs a) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= a.n) return;
    const uint32_t n = a.n;

    const uint32_t lfo_inc = a.coef[CHC_LFO_INC * n + i];
    const uint32_t lfo_off = a.coef[CHC_LFO_OFF * n + i];
    const uint32_t ps_inc = a.coef[CHC_PS_INC * n + i];
    const float D = __uint_as_float(a.coef[CHC_DEPTH * n + i]);
    const float W = __uint_as_float(a.coef[CHC_WINDOW * n + i]);
    const float b0 = __uint_as_float(a.coef[CHC_B0 * n + i]);
    const float b1 = __uint_as_float(a.coef[CHC_B1 * n + i]);
    const float b2 = __uint_as_float(a.coef[CHC_B2 * n + i]);
    const float a1 = __uint_as_float(a.coef[CHC_A1 * n + i]);
    const float a2 = __uint_as_float(a.coef[CHC_A2 * n + i]);
    const float mix = __uint_as_float(a.coef[CHC_MIX * n + i]);
    const float dry = __uint_as_float(a.coef[CHC_DRY * n + i]);

    uint32_t lfo_acc = a.state[CHS_LFO_ACC * n + i];
    uint32_t ps_acc = a.state[CHS_PS_ACC * n + i];
    float z1[2], z2[2];
    z1[0] = __uint_as_float(a.state[CHS_Z1L * n + i]);
    z2[0] = __uint_as_float(a.state[CHS_Z2L * n + i]);
    z1[1] = __uint_as_float(a.state[CHS_Z1R * n + i]);
    z2[1] = __uint_as_float(a.state[CHS_Z2R * n + i]);

    const uint32_t pmask = a.psize - 1u, cmask = a.csize - 1u;
    const float pmax = (float)(a.psize - 2u), cmax = (float)(a.csize - 2u);
    float *pring[2] = {a.pitch_ring + ((size_t)i * 2 + 0) * a.psize, a.pitch_ring + ((size_t)i * 2 + 1) * a.psize};
    float *cring[2] = {a.chorus_ring + ((size_t)i * 2 + 0) * a.csize, a.chorus_ring + ((size_t)i * 2 + 1) * a.csize};
    const size_t plane = (size_t)a.n_frames * n;
    const bool full = a.mode == 0;

    for (uint32_t f = 0; f < a.n_frames; ++f) {
        const uint32_t w = a.t0 + f;
        // cycle~ (output, then advance) and the modulated delay time D*lfo + D (mono-chorus :2920-2935)
        const float lfo = cos2pi(unit24(lfo_acc + lfo_off));
        lfo_acc += lfo_inc;
        const float dch = lfo * D + D;
        // gen~ phasor and the two crossfaded taps
        const float p0 = unit24(ps_acc);
        const float p1 = unit24(ps_acc + 0x80000000u);
        ps_acc += ps_inc;
        const float g0 = cos2pi((p0 - 0.5f) * 0.5f);
        const float g1 = cos2pi((p1 - 0.5f) * 0.5f);
        const float d0 = p0 * W, d1 = p1 * W;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const float x = a.in[(size_t)c * plane + (size_t)f * n + i];
            const float t0 = read_frac(pring[c], pmask, w, d0, 1.0f, pmax);
            const float t1 = read_frac(pring[c], pmask, w, d1, 1.0f, pmax);
            const float ps = t1 * g1 + t0 * g0;
            pring[c][w & pmask] = x;
            float y;
            if (full) {
                cring[c][w & cmask] = ps;
                const float wet = read_frac(cring[c], cmask, w, dch, 0.0f, cmax);
                const float lp = b0 * wet + z1[c];
                z1[c] = (b1 * wet - a1 * lp) + z2[c];
                z2[c] = b2 * wet - a2 * lp;
                y = x * dry + lp * mix;
            } else {
                y = ps;
            }
            a.out[(size_t)c * plane + (size_t)f * n + i] = y;
        }
    }

    a.state[CHS_LFO_ACC * n + i] = lfo_acc;
    a.state[CHS_PS_ACC * n + i] = ps_acc;
    a.state[CHS_Z1L * n + i] = __float_as_uint(z1[0]);
    a.state[CHS_Z2L * n + i] = __float_as_uint(z2[0]);
    a.state[CHS_Z1R * n + i] = __float_as_uint(z1[1]);
    a.state[CHS_Z2R * n + i] = __float_as_uint(z2[1]);
}

hipError_t launch_chorus(const ChorusArgs &a, hipStream_t s) {
    if (a.n == 0 || a.n_frames == 0) return hipSuccess;
    const uint32_t threads = 256;
    hipLaunchKernelGGL(chorus_block_v1, dim3((a.n + threads - 1) / threads), dim3(threads), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
