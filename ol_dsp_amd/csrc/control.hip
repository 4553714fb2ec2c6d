// ol_dsp_amd/csrc/control.hip -- the device side of parameter changes (olfx_set_params /
// olfx_control / olfx_update, applied at the next block boundary).
//
// The host re-derives the coefficients of the instances whose parameters changed since the last
// block -- only those, with the reference's setter arithmetic (olfx_engine.cpp derive_*) -- and
// ships them as one packet with the block (an asynchronous copy on the engine's control stream).
// This kernel scatters the packet into the field-major coefficient arrays the effect kernels read,
// on the caller's stream, ahead of the block's launch.  Work and traffic are O(changed instances).
#include "olfx_internal.h"

namespace olfx {

__global__ __launch_bounds__(256) void coef_scatter(CoefScatterArgs a) {
    const uint64_t t = (uint64_t)blockIdx.x * 256u + threadIdx.x;
    if (t >= (uint64_t)a.m * a.W) return;
    const uint32_t w = (uint32_t)(t / a.m), r = (uint32_t)(t % a.m);   // record fastest: coalesced
    const uint32_t inst = a.inst ? a.inst[r] : r;
    const uint32_t v = a.val[(size_t)w * a.m + r];
    uint32_t s = 0, w0 = w;
    while (s + 1 < a.nseg && w0 >= a.words[s]) { w0 -= a.words[s]; ++s; }
    a.dst[s][(size_t)w0 * a.stride[s] + inst] = v;
}

hipError_t launch_coef_scatter(const CoefScatterArgs &a, hipStream_t s) {
    if (a.m == 0 || a.W == 0) return hipSuccess;
    const uint64_t threads = (uint64_t)a.m * a.W;
    if (threads > (uint64_t)0xFFFFFFFFu * 256u) return hipErrorInvalidValue;
    hipLaunchKernelGGL(coef_scatter, dim3((uint32_t)((threads + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace olfx
