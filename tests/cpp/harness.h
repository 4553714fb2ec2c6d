/*
 * tests/cpp/harness.h -- the small TEST/EXPECT harness of the C++ tests (gtest is not in the image)
 * and their shared input helpers (TEST INFRASTRUCTURE).
 */
#ifndef OLFX_TEST_HARNESS_H
#define OLFX_TEST_HARNESS_H
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../oracle/oracle.h"

namespace {
struct Case { const char *suite, *name; std::function<void()> fn; };
std::vector<Case> &cases() { static std::vector<Case> c; return c; }
int g_failures = 0;
struct Reg { Reg(const char *s, const char *n, std::function<void()> f) { cases().push_back({s, n, std::move(f)}); } };
#define TEST(S, N) static void S##_##N(); static Reg reg_##S##_##N(#S, #N, S##_##N); static void S##_##N()
#define EXPECT_TRUE(c) do { if (!(c)) { ++g_failures; std::printf("  FAILED %s:%d: %s\n", __FILE__, __LINE__, #c); } } while (0)
#define EXPECT_EQ(a, b) EXPECT_TRUE((a) == (b))

/* xorshift32 white noise in [-1,1): the SURVEY section 8c KAT generator, one seed per instance */
std::vector<float> noise(uint32_t ch, uint32_t frames, uint32_t n, uint32_t seed) {
    std::vector<float> x((size_t)ch * frames * n);
    for (uint32_t c = 0; c < ch; ++c)
        for (uint32_t i = 0; i < n; ++i)
            oracle_xorshift_noise(seed + 7919u * i + 104729u * c, x.data() + (size_t)c * frames * n + i,
                                  frames, n);
    return x;
}

struct Lcg {   /* deterministic parameter draws */
    uint64_t s;
    explicit Lcg(uint64_t seed) : s(seed) {}
    float uni(float lo, float hi) {
        s = s * 6364136223846793005ull + 1442695040888963407ull;
        return lo + (hi - lo) * (float)((s >> 40) * (1.0 / 16777216.0));
    }
};

[[maybe_unused]] size_t first_bit_mismatch(const std::vector<float> &a, const std::vector<float> &b) {
    for (size_t k = 0; k < a.size(); ++k)
        if (std::memcmp(&a[k], &b[k], 4) != 0) return k;
    return (size_t)-1;
}

/* Process `frames` frames through `op` in blocks of `block` frames; layout [ch][frames][n]. */
template <class F>
std::vector<float> run_blocks(F &&proc, const std::vector<float> &x, uint32_t ich, uint32_t och,
                              uint32_t frames, uint32_t n, uint32_t block) {
    std::vector<float> y((size_t)och * frames * n), xin((size_t)ich * block * n), yb((size_t)och * block * n);
    for (uint32_t f0 = 0; f0 < frames; f0 += block) {
        uint32_t b = std::min(block, frames - f0);
        for (uint32_t c = 0; c < ich; ++c)
            std::memcpy(&xin[(size_t)c * b * n], &x[((size_t)c * frames + f0) * n], (size_t)b * n * 4);
        proc(xin.data(), yb.data(), b);
        for (uint32_t c = 0; c < och; ++c)
            std::memcpy(&y[((size_t)c * frames + f0) * n], &yb[(size_t)c * b * n], (size_t)b * n * 4);
    }
    return y;
}
}  // namespace

inline int run_all_tests() {
    for (auto &c : cases()) {
        int before = g_failures;
        std::printf("[ RUN      ] %s.%s\n", c.suite, c.name);
        try { c.fn(); } catch (const std::exception &e) { ++g_failures; std::printf("  exception: %s\n", e.what()); }
        std::printf("[ %s ] %s.%s\n", g_failures == before ? "      OK" : " FAILED ", c.suite, c.name);
    }
    std::printf("%zu tests, %d failures\n", cases().size(), g_failures);
    return g_failures ? 1 : 0;
}

#endif
