// ol_dsp_amd/csrc/chorus_stage.h -- device helpers shared by the chorus / pitch-shift stage and the fx rack.
//
// Spec (no executable oracle exists in the reference, parity "unpinned"):
//   mono-chorus.rnbopat: y = (1-mix) x + mix * lores~( delay~( pitchshift(x, pitch),
//                                                   D cycle~(rate_hz, phase) + D ), cutoff_hz, q )
//   pitchshift.gendsp / gencode at mono-chorus.rnbopat:962:
//       p0 = phasor(shift), p1 = (p0 + 0.5) % 1, W = mstosamps(window)
//       out = read(p1 W) cos((p1-.5)pi) + read(p0 W) cos((p0-.5)pi);  write(x) after the reads
//   stereo-chorus.rnbopat: L and R are two mono-chorus instances with shared params; L phase 1 and
//   R phase 0 are the same phase after wrap, so both channels see the same LFO.
//
// Mapping: one lane = one (instance, channel); a wave = 32 instances x 2 channels (lane 2j+ch).
// Rings are instance-private ([inst][size][2], stereo-interleaved: L and R share every tap
// position) because every tap is modulated per instance.
//
// This header holds the helpers the stages share: buffer-resource loads and stores with 32-bit
// offsets (frame offsets in SGPRs), the DPP lane-pair exchanges, the delay split / clamp and the
// reduced-range cos2pi.  The chorus / pitch-shift stage itself (line carry, software pipeline) is
// chorus_stage_l.h; the fx rack (fxrack.hip) uses the helpers only.
#pragma once
#include <type_traits>

#include "olfx_internal.h"

namespace olfx {
namespace ch {

constexpr int kThreads = 256;
constexpr int kRow = 64;                    // LDS slot stride: one wave's lanes

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __amdgpu_buffer_rsrc_t Rsrc;

__device__ __forceinline__ Rsrc rsrc(const void *p, uint64_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), (short)0,
                                             (int)(uint32_t)(bytes > 0xFFFFFFFFull ? 0xFFFFFFFFull : bytes), 0x00020000);
}
// cache policy of the streamed accesses (block input/output, ring stores): 0 = default (nt, aux
// bit 1, measured no better: DESIGN.md section 4)
constexpr int kStreamAux = 0;
// s_setprio 3 while the line-carry stage issues the next chunk's input loads and line loads (the
// other wave of the SIMD yields its issue slots for those few instructions, so they leave earlier
// and the chunk's arithmetic covers more of their latency): chorus ~1 % faster over six same-box
// pairs, pitch-shift and chain (one wave per SIMD) unchanged
constexpr int kLoadPrio = 3;

template <int AUX = 0>
__device__ __forceinline__ float ld1(Rsrc r, uint32_t voff, uint32_t soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, voff, soff, AUX));
}
template <int AUX = 0>
__device__ __forceinline__ void st1(Rsrc r, uint32_t voff, uint32_t soff, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, voff, soff, AUX);
}
__device__ __forceinline__ float4 ld4(Rsrc r, uint32_t voff) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
    return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
template <int AUX = 0>
__device__ __forceinline__ void st4(Rsrc r, uint32_t voff, float4 v) {
    u32x4 u;
    u.x = __float_as_uint(v.x); u.y = __float_as_uint(v.y); u.z = __float_as_uint(v.z); u.w = __float_as_uint(v.w);
    __builtin_amdgcn_raw_buffer_store_b128(u, r, voff, 0, AUX);
}

// exchange a value with the neighbouring lane (lanes 2j <-> 2j+1): DPP quad_perm [1,0,3,2]
__device__ __forceinline__ float swap_pair(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

__device__ __forceinline__ float unit24(uint32_t acc) {
    return (float)(acc >> 8) * 5.9604644775390625e-8f;   // exact: 24-bit fraction in [0,1)
}

// The fp32 signal path in fused multiply-adds (spec v3, round 6; the oracle's
// chorus_ref.c the same operations): interpolation, the crossfade sum, lores~ and the dry / wet mix
__device__ __forceinline__ float lerp_pair(float x0, float x1, float fr) { return __builtin_fmaf(fr, x1 - x0, x0); }
__device__ __forceinline__ float xfade(float tB, float gB, float tA, float gA) { return __builtin_fmaf(tB, gB, tA * gA); }
// lores~ (TDF-II biquad): lp = b0 w + z1; z1 = (b1 w - a1 lp) + z2; z2 = b2 w - a2 lp
__device__ __forceinline__ float lores_step(float wet, float b0, float b1, float b2, float a1, float a2, float &z1,
                                            float &z2) {
    const float lp = __builtin_fmaf(b0, wet, z1);
    z1 = __builtin_fmaf(-a1, lp, b1 * wet) + z2;
    z2 = __builtin_fmaf(-a2, lp, b2 * wet);
    return lp;
}
__device__ __forceinline__ float dry_wet(float x, float dry, float lp, float mix) { return __builtin_fmaf(lp, mix, x * dry); }

// a value of lane 2j (EVEN) or 2j+1 (odd) to both lanes of the pair: DPP quad_perm [0,0,2,2] / [1,1,3,3]
__device__ __forceinline__ float pair_even(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xA0, 0xF, 0xF, false));
}
__device__ __forceinline__ float pair_odd(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xF5, 0xF, 0xF, false));
}
__device__ __forceinline__ int pair_even_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0xA0, 0xF, 0xF, false); }
__device__ __forceinline__ int pair_odd_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0xF5, 0xF, 0xF, false); }

}  // namespace ch
}  // namespace olfx
