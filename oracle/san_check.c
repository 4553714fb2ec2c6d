/*
 * oracle/san_check.c -- every CPU restatement under AddressSanitizer and UndefinedBehaviorSanitizer
 * (sanitizers on the CPU side).  TEST INFRASTRUCTURE ONLY.
 *
 * Built by `make -C oracle san` together with the oracle sources, all with
 * -fsanitize=address,undefined -fno-sanitize-recover=all, and run by tests/test_sanitizers.py: any
 * out-of-bounds access, leak, signed overflow, misaligned or invalid shift aborts the run.  The
 * drive covers the paths the GPU parity tests use: the Dattorro plate past its uint16 t wrap with
 * pre-delays 0 .. 4800 (verb.cpp:137-139, 298); chorus and pitch-shift (fp32 and double) through
 * phasor wraps and RNBO clamps; both voice models through every note / gate / frequency event; the
 * rack in all five topologies with delays 0 .. 47,999 (Fx.h:23).
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int check_finite(const float *x, long n, const char *what)
{
    for (long k = 0; k < n; ++k)
        if (!isfinite(x[k])) {
            printf("%s: non-finite output at %ld\n", what, k);
            return 1;
        }
    return 0;
}

int main(void)
{
    int bad = 0;
    const int n = 5;
    const long F = 70000;                                   /* past t = 65536 (uint16 wrap) */
    float *x = malloc(sizeof(float) * 2 * F * n), *y = malloc(sizeof(float) * 2 * F * n);
    double *yd = malloc(sizeof(double) * 2 * F * n);
    for (int c = 0; c < 2; ++c)
        for (int i = 0; i < n; ++i) oracle_xorshift_noise(12345u + 7u * (uint32_t)i + 101u * (uint32_t)c, x + (long)c * F * n + i, F, n);

    /* Dattorro: pre-delays 0, 1, 480, 4799, 4800 samples */
    oracle_dattorro *d = oracle_dattorro_create(n);
    const float pd[5] = {0.f, 1.f / 4800.f, 0.1f, 4799.f / 4800.f, 1.f};
    for (int i = 0; i < n; ++i) {
        oracle_dattorro_set(d, i, 0, pd[i]);
        oracle_dattorro_set(d, i, 5, 0.25f + 0.15f * (float)i);
    }
    oracle_dattorro_process(d, x, 2, y, F, 1);
    bad |= check_finite(y, 2 * F * n, "dattorro");
    oracle_dattorro_destroy(d);

    /* chorus / pitch-shift, fp32 and double: fastest phasor, clamped params */
    for (int mode = 0; mode < 2; ++mode) {
        oracle_chorus *c = oracle_chorus_create(n, 48000.f, mode);
        oracle_chorus64 *c64 = oracle_chorus64_create(n, 48000.0, mode);
        for (int i = 0; i < n; ++i)
            for (int f = 0; f < 8; ++f) {
                const float v = f == 0 ? 3.0f * (float)i / (n - 1) : (f == 7 ? 4.0f + 1.5f * (float)i : -1.0f + 0.6f * (float)i);
                oracle_chorus_set(c, i, f, v);
                oracle_chorus64_set(c64, i, f, v);
            }
        oracle_chorus_process(c, x, y, 20000, 1);
        bad |= check_finite(y, 2 * 20000L * n, mode ? "pitch-shift" : "chorus");
        oracle_chorus64_process(c64, x, yd, 20000);
        oracle_chorus_destroy(c);
        oracle_chorus64_destroy(c64);
    }
    double sum = 0;
    const float cp[8] = {1.5f, 0.5f, 0.5f, 0.3f, 1.f, 0.5f, 0.2f, 10.f};
    oracle_chorus_c1(48000.f, cp, 48000, 256, &sum);

    /* voices: both models, every event type, configured and members-before-Init */
    for (int model = 0; model < 2; ++model) {
        oracle_voice *v = oracle_voice_create_model(n, 48000.f, model);
        float cfg[16] = {2000.f, 0.4f, 0.5f, 0.6f, 0.01f, 0.5f, 0.1f, 0.5f, 0.05f, 0.9f, 0.005f, 0.f, 0.1f, 0.7f, 0.05f, 0.002f};
        for (int i = 0; i < n; ++i) {
            if (i == 0) oracle_voice_init_members(v, i, cfg);
            else oracle_voice_config(v, i, cfg);
            oracle_voice_note(v, i, 1, 40 + 10 * i);
        }
        for (int b = 0; b < 20; ++b) {
            for (int i = 0; i < n; ++i) oracle_voice_event(v, i, (b + i) % 5, 30 + b, 110.f + (float)b);
            oracle_voice_process(v, y, 256, 1);
        }
        oracle_voice_destroy(v);
    }

    /* the rack, topologies 0..4, delays 0 .. 47,999 */
    oracle_fxrack *r = oracle_fxrack_create(n, 48000.f);
    const float dt[5] = {0.f, 1.f / 48000.f, 0.5f, 0.999f, 1.f};
    for (int i = 0; i < n; ++i) {
        oracle_fxrack_set(r, i, OFR_DELAY_TIME, dt[i]);
        oracle_fxrack_set(r, i, OFR_FILTER_TYPE, (float)i);
        oracle_fxrack_set(r, i, OFR_TOPOLOGY, (float)i);
    }
    oracle_fxrack_process(r, x, y, 50000, 1);
    bad |= check_finite(y, 2 * 50000L * n, "fxrack");
    oracle_fxrack_destroy(r);

    free(x); free(y); free(yd);
    printf("san_check: %s\n", bad ? "FAILED" : "ok");
    return bad;
}
