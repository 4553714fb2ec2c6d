// tools/hwid_probe.hip -- where do the waves of a 4-wave workgroup land?  (diagnostic, GPU box)
//
// Launches the voice kernel's shape (512 workgroups x 256 threads, 24.5 KB of static LDS, two
// workgroups per CU) and records each wave's HW_ID (s_getreg HW_REG_HW_ID: wave slot [3:0],
// SIMD [5:4], CU [11:8], SH [12], SE [15:13] on gfx9) plus XCC_ID, then prints: how many workgroups
// have their 4 waves on 4 distinct SIMDs, the slot parity of wave 0, and for co-resident workgroups
// (same SE/SH/CU/XCC) whether their wave-0 slot parities differ.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/hwid_probe tools/hwid_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <map>
#include <tuple>
#include <vector>

__global__ __launch_bounds__(256) void probe(uint32_t *out, float *sink) {
    __shared__ float pad[6272];                 // ~24.5 KB, as voice_block_v5
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | (31 << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (0 << 6) | (31 << 11));   // HW_REG_XCC_ID
    pad[threadIdx.x] = (float)hw;
    __syncthreads();
    // some work so that workgroups overlap in time
    float acc = pad[(threadIdx.x + 1) & 255];
    for (int k = 0; k < 20000; ++k) acc = acc * 0.999f + 1.0f;
    if (lane == 0) {
        out[(blockIdx.x * 4 + wave) * 2] = hw;
        out[(blockIdx.x * 4 + wave) * 2 + 1] = xcc;
    }
    if (acc == 12345.0f) sink[0] = acc;
}

int main() {
    const int blocks = 512;
    uint32_t *d;
    float *s;
    hipMalloc(&d, blocks * 4 * 2 * sizeof(uint32_t));
    hipMalloc(&s, sizeof(float));
    hipLaunchKernelGGL(probe, dim3(blocks), dim3(256), 0, 0, d, s);
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    std::vector<uint32_t> h(blocks * 8);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    int distinct = 0;
    std::map<std::tuple<int, int, int, int>, std::vector<int>> cu_wgs;   // (xcc, se, sh, cu) -> wave-0 slots
    int same_par = 0, diff_par = 0, pairs = 0;
    for (int b = 0; b < blocks; ++b) {
        int m = 0;
        for (int w = 0; w < 4; ++w) m |= 1 << ((h[(b * 4 + w) * 2] >> 4) & 3);
        distinct += m == 15;
        const uint32_t hw = h[b * 8], xcc = h[b * 8 + 1];
        cu_wgs[{(int)(xcc & 0xF), (int)((hw >> 13) & 7), (int)((hw >> 12) & 1), (int)((hw >> 8) & 15)}].push_back(hw & 15);
        if (b < 8) {
            printf("wg %3d:", b);
            for (int w = 0; w < 4; ++w) {
                const uint32_t v = h[(b * 4 + w) * 2];
                printf("  w%d simd %u slot %2u cu %2u", w, (v >> 4) & 3, v & 15, (v >> 8) & 15);
            }
            printf("  xcc %u\n", h[b * 8 + 1] & 0xF);
        }
    }
    for (auto &kv : cu_wgs) {
        if (kv.second.size() == 2) {
            ++pairs;
            if ((kv.second[0] & 1) == (kv.second[1] & 1)) ++same_par; else ++diff_par;
        }
    }
    printf("workgroups with 4 distinct SIMDs: %d of %d\n", distinct, blocks);
    printf("CUs seen: %zu; CUs with 2 workgroups: %d (wave-0 slot parity same %d, different %d)\n",
           cu_wgs.size(), pairs, same_par, diff_par);
    return 0;
}
