// tools/rcp_probe.hip -- what does gfx950's v_rcp_f32 return?  (diagnostic, GPU box)
//
// The voice kernels divide through __builtin_amdgcn_rcpf (v_rcp_f32, "1 ulp").  To make the
// voice's parity check bit-exact the oracle needs the instruction's exact results, so this probe
// records them: every mantissa of [1, 2) (2^23 inputs), compared with the correctly rounded 1/x of
// the host (IEEE float division), and a check that the result only depends on the mantissa
// (rcp(m 2^e) == rcp(m) 2^-e for normal results) over exponents -60..60 and both signs.
// Writes gpurun_out/rcp_exceptions.bin: uint32 pairs (mantissa bits, rcp bits) wherever v_rcp
// differs from the correctly rounded reciprocal, and prints a summary.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/rcp_probe tools/rcp_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void rcp_all(uint32_t *out, int e, uint32_t sign) {
    const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= (1u << 23)) return;
    const uint32_t bits = sign | ((uint32_t)(127 + e) << 23) | m;
    out[m] = __float_as_uint(__builtin_amdgcn_rcpf(__uint_as_float(bits)));
}

static float f(uint32_t b) { float x; std::memcpy(&x, &b, 4); return x; }
static uint32_t u(float x) { uint32_t b; std::memcpy(&b, &x, 4); return b; }

int main() {
    const uint32_t N = 1u << 23;
    uint32_t *d;
    if (hipMalloc(&d, N * 4) != hipSuccess) { printf("alloc failed\n"); return 1; }
    std::vector<uint32_t> base(N), h(N);
    hipLaunchKernelGGL(rcp_all, dim3(N / 256), dim3(256), 0, 0, d, 0, 0u);
    if (hipMemcpy(base.data(), d, N * 4, hipMemcpyDeviceToHost) != hipSuccess) { printf("copy failed\n"); return 1; }
    std::vector<uint32_t> exc;
    uint64_t up = 0, down = 0, far = 0;
    for (uint32_t m = 0; m < N; ++m) {
        const float x = f((127u << 23) | m);
        const uint32_t cr = u(1.0f / x);
        if (base[m] != cr) {
            exc.push_back(m);
            exc.push_back(base[m]);
            const int64_t dlt = (int64_t)base[m] - (int64_t)cr;
            if (dlt == 1) ++up; else if (dlt == -1) ++down; else ++far;
        }
    }
    printf("mantissas %u: v_rcp != RN(1/x) on %zu (%.4f %%): +1 ulp %llu, -1 ulp %llu, other %llu\n", N,
           exc.size() / 2, 100.0 * (exc.size() / 2) / N, (unsigned long long)up, (unsigned long long)down,
           (unsigned long long)far);
    // exponent independence: rcp(m 2^e) == rcp(m) 2^-e while the result is normal
    uint64_t bad = 0, checked = 0;
    for (int e = -60; e <= 60; e += 1) {
        for (uint32_t sign = 0; sign <= 0x80000000u; sign += 0x80000000u) {
            hipLaunchKernelGGL(rcp_all, dim3(N / 256), dim3(256), 0, 0, d, e, sign);
            hipMemcpy(h.data(), d, N * 4, hipMemcpyDeviceToHost);
            for (uint32_t m = 0; m < N; ++m) {
                const float want = std::ldexp(f(base[m]), -e) * (sign ? -1.0f : 1.0f);
                ++checked;
                if (u(want) != h[m]) {
                    if (bad < 5) printf("  e=%d sign=%u m=%06x: got %08x want %08x\n", e, sign >> 31, m, h[m], u(want));
                    ++bad;
                }
            }
            if (sign) break;
        }
    }
    printf("exponent scaling: %llu of %llu differ\n", (unsigned long long)bad, (unsigned long long)checked);
    FILE *fp = fopen("gpurun_out/rcp_exceptions.bin", "wb");
    if (!fp) { printf("cannot write\n"); return 1; }
    fwrite(exc.data(), 4, exc.size(), fp);
    fclose(fp);
    hipFree(d);
    return 0;
}
