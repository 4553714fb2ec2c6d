// tests/gpu_probe/rcp_probe.hip -- TEST INFRASTRUCTURE: reads gfx950's v_rcp_f32 results over every
// mantissa of [1, 2) for the voice oracle's kernel-arithmetic mode (oracle/voice_ref.c, "v_rcp
// model").  Loaded only by tests/ (ctypes); the product (ol_dsp_amd/libolfx.so) does not use it.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
__global__ void rcp_mantissas(uint32_t *out) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    out[m] = __float_as_uint(__builtin_amdgcn_rcpf(__uint_as_float((127u << 23) | m)));
}
}  // namespace

// host_out: 2^23 uint32.  Returns 0 on success, else the hipError_t.
extern "C" int probe_rcp_table(uint32_t *host_out) {
    uint32_t *d = nullptr;
    hipError_t rc = hipMalloc(&d, sizeof(uint32_t) << 23);
    if (rc != hipSuccess) return (int)rc;
    hipLaunchKernelGGL(rcp_mantissas, dim3((1u << 23) / 256), dim3(256), 0, 0, d);
    rc = hipGetLastError();
    if (rc == hipSuccess) rc = hipMemcpy(host_out, d, sizeof(uint32_t) << 23, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return (int)rc;
}
