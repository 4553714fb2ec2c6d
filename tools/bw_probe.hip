// tools/bw_probe.hip -- the achievable HBM rate on this MI355X for the read/write mixes of the
// effect kernels (the ceilings the roofline fractions are read against).
// Streams of 16-B accesses, each wave instruction 1 KB contiguous, grid-stride over 2 GiB buffers:
//   read     : R = 1, W = 0                 write : R = 0, W = 1
//   copy     : R = 1, W = 1                 r2w1  : R = 2, W = 1 (the chain's 164 : 84 B/frame)
//   r3w1     : R = 3, W = 1 (chorus 34 : 24 is ~ r3w2; reverb 117 : 58 is ~ r2w1)
//   taps     : the reverb's shape -- per 4-frame step a wave reads 12 groups of 1 KB from 12
//              streams 1 MB apart and writes 6 (R : W = 2 : 1), 1024 waves in flight
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bw_probe tools/bw_probe.hip ; run: tools/bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <int R, int W>
__global__ __launch_bounds__(256) void mix(const float4 *__restrict__ a, const float4 *__restrict__ b,
                                           const float4 *__restrict__ c, float4 *__restrict__ d,
                                           float4 *__restrict__ e, size_t n, float *sink) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = make_float4(1.f, 2.f, 3.f, 4.f);
        if (R >= 1) { const float4 x = a[i]; v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w; }
        if (R >= 2) { const float4 x = b[i]; v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w; }
        if (R >= 3) { const float4 x = c[i]; v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w; }
        if (W >= 1) d[i] = v;
        if (W >= 2) e[i] = v;
        acc.x += v.x;
    }
    if (W == 0 && acc.x == 12345.f) *sink = acc.x;
}

// the reverb's access shape: a wave owns 64 "instances" (1 KB columns); per step it reads 12 rows
// (groups) of 12 different streams and writes 6, rows advancing one group per step
__global__ __launch_bounds__(64) void taps(const float4 *__restrict__ ring, float4 *__restrict__ wring, uint32_t n,
                                           uint32_t steps, uint32_t rows, float *sink) {
    const uint32_t i = blockIdx.x * 64u + threadIdx.x;
    float acc = 0.f;
    for (uint32_t s = 0; s < steps; ++s) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            const float4 x = ring[((size_t)k * rows + (s + 37u * k) % rows) * n + i];
            v.x += x.x; v.y += x.y; v.z += x.z; v.w += x.w;
        }
#pragma unroll
        for (int k = 0; k < 6; ++k) wring[((size_t)k * rows + (s + 11u * k) % rows) * n + i] = v;
        acc += v.x;
    }
    if (acc == 12345.f) *sink = acc;
}

// the chorus's access shape (chorus_block_v11): a wave = 32 instances x 2
// channels; per 16-frame chunk and instance it reads 3 tap lines of 128 B from its own rings (two
// pitch taps in a 512-position stereo ring, one chorus tap in a 2048-position one; 8 lanes per line,
// 8 lines per instruction) and the chunk's input rows, and writes one line into each ring and the
// output rows: 32 + 24 B per frame, the chorus's algorithmic 56.  No arithmetic.
// INST instances per wave (32: the chorus's own 2 waves per SIMD at 65,536 instances; 16: the same
// bytes over twice the waves, the premise of VERDICT r5 #3's frame split)
template <uint32_t INST>
__global__ __launch_bounds__(64) void chorus_shape(const float4 *__restrict__ in, float4 *__restrict__ out,
                                                   float4 *__restrict__ pring, float4 *__restrict__ cring,
                                                   uint32_t n, uint32_t chunks, float *sink) {
    constexpr uint32_t Q = INST / 8u;                     // instructions per tap set (8 instances each)
    const uint32_t lane = threadIdx.x, inst0 = blockIdx.x * INST;
    const uint32_t piece = lane & 7u;                     // 16-B piece of a 128-B line
    float acc = 0.f;
    for (uint32_t c = 0; c < chunks; ++c) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        // tap lines: instruction q covers instances 8 q + lane / 8, 3 taps
#pragma unroll
        for (uint32_t q = 0; q < Q; ++q) {
            const uint32_t j = inst0 + 8u * q + (lane >> 3);
            const uint32_t h = j * 2654435761u;           // a per-instance tap offset
            const uint32_t pA = (c + 1u + (h & 15u)) & 31u, pB = (c + 17u + (h & 15u)) & 31u;   // 512 x 2 floats = 32 lines
            const uint32_t pC = (c + 1u + ((h >> 8) & 63u)) & 127u;                             // 2048 x 2 floats = 128 lines
            const float4 a = pring[((size_t)j * 32u + pA) * 8u + piece];
            const float4 b = pring[((size_t)j * 32u + pB) * 8u + piece];
            const float4 d = cring[((size_t)j * 128u + pC) * 8u + piece];
            v.x += a.x + b.x + d.x; v.y += a.y + b.y + d.y;
        }
        // input rows: 16 frames x 2 channels of INST instances (4 INST B each), 64 / (INST / 4) rows per
        // instruction
        constexpr uint32_t P = INST / 4u, RPI = 64u / P;    // 16-B pieces per row, rows per instruction
#pragma unroll
        for (uint32_t q = 0; q < 32u / RPI; ++q) {
            const uint32_t r = RPI * q + lane / P, f = 16u * c + (r >> 1), ch = r & 1u;
            const float4 x = in[(((size_t)ch * 16u * chunks + f) * n + inst0) / 4u + lane % P];
            v.z += x.x; v.w += x.y;
        }
        // writes: one line per instance into each ring, and the output rows
#pragma unroll
        for (uint32_t q = 0; q < Q; ++q) {
            const uint32_t j = inst0 + 8u * q + (lane >> 3);
            pring[((size_t)j * 32u + (c & 31u)) * 8u + piece] = v;
            cring[((size_t)j * 128u + (c & 127u)) * 8u + piece] = v;
        }
#pragma unroll
        for (uint32_t q = 0; q < 32u / RPI; ++q) {
            const uint32_t r = RPI * q + lane / P, f = 16u * c + (r >> 1), ch = r & 1u;
            out[(((size_t)ch * 16u * chunks + f) * n + inst0) / 4u + lane % P] = v;
        }
        acc += v.x;
    }
    if (acc == 12345.f) *sink = acc;
}

int main() {
    const size_t bytes = (size_t)2 << 30, n = bytes / 16;
    float4 *buf[5];
    for (auto &p : buf) { CHK(hipMalloc(&p, bytes)); CHK(hipMemset(p, 0, bytes)); }
    float *sink;
    CHK(hipMalloc(&sink, 4));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0)); CHK(hipEventCreate(&e1));
    int cus = 0;
    CHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const dim3 grid(cus * 8), block(256);
    auto run = [&](const char *name, auto kern, int R, int W) {
        for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, grid, block, 0, 0, buf[0], buf[1], buf[2], buf[3], buf[4], n, sink);
        CHK(hipEventRecord(e0));
        const int it = 10;
        for (int w = 0; w < it; ++w) hipLaunchKernelGGL(kern, grid, block, 0, 0, buf[0], buf[1], buf[2], buf[3], buf[4], n, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double gbs = (double)bytes * (R + W) * it / (ms * 1e-3) / 1e9;
        std::printf("%-6s R%d W%d  %8.1f GB/s  %.3f of 8000\n", name, R, W, gbs, gbs / 8000.0);
    };
    run("read", mix<1, 0>, 1, 0);
    run("write", mix<0, 1>, 0, 1);
    run("copy", mix<1, 1>, 1, 1);
    run("r2w1", mix<2, 1>, 2, 1);
    run("r3w1", mix<3, 1>, 3, 1);
    run("r3w2", mix<3, 2>, 3, 2);
    {   // the tap shape: 65,536 columns, 12 read streams and 6 write streams of 2,048 rows
        const uint32_t cols = 65536, rows = 2048, steps = 64;
        float4 *ring, *wring;
        CHK(hipMalloc(&ring, (size_t)12 * rows * cols * 16));
        CHK(hipMalloc(&wring, (size_t)6 * rows * cols * 16));
        for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(taps, dim3(cols / 64), dim3(64), 0, 0, ring, wring, cols, steps, rows, sink);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(taps, dim3(cols / 64), dim3(64), 0, 0, ring, wring, cols, steps, rows, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHK(hipEventElapsedTime(&ms, e0, e1));
        const double gbs = (double)cols * steps * 18 * 16 / (ms * 1e-3) / 1e9;
        std::printf("taps   R12 W6 (1 wave/64 cols, 1024 waves)  %8.1f GB/s  %.3f of 8000\n", gbs, gbs / 8000.0);
    }
    {   // the chorus's shape: 65,536 instances, 256-frame blocks (16 chunks)
        const uint32_t n = 65536, chunks = 16, F = 16 * chunks;
        float4 *in, *out, *pr, *cr;
        CHK(hipMalloc(&in, (size_t)2 * F * n * 4)); CHK(hipMalloc(&out, (size_t)2 * F * n * 4));
        CHK(hipMalloc(&pr, (size_t)n * 512 * 2 * 4)); CHK(hipMalloc(&cr, (size_t)n * 2048 * 2 * 4));
        auto shape = [&](auto kern, uint32_t inst, const char *what) {
            for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(kern, dim3(n / inst), dim3(64), 0, 0, in, out, pr, cr, n, chunks, sink);
            CHK(hipEventRecord(e0));
            const int it = 20;
            for (int w = 0; w < it; ++w) hipLaunchKernelGGL(kern, dim3(n / inst), dim3(64), 0, 0, in, out, pr, cr, n, chunks, sink);
            CHK(hipEventRecord(e1));
            CHK(hipEventSynchronize(e1));
            float ms = 0.f;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            const double gbs = (double)n * F * 56.0 * it / (ms * 1e-3) / 1e9;
            std::printf("chorus R32 W24 B/frame (%s, 65,536 instances)  %8.1f GB/s  %.3f of 8000  %.4f ms per block\n",
                        what, gbs, gbs / 8000.0, ms / it);
        };
        shape(chorus_shape<32>, 32, "32 instances per wave: 2 waves/SIMD");
        shape(chorus_shape<16>, 16, "16 instances per wave: 4 waves/SIMD");
        shape(chorus_shape<32>, 32, "32 instances per wave: 2 waves/SIMD, again");
    }
    return 0;
}
