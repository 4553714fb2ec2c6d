/*
 * oracle/ref_verb_wrap.cpp -- C wrapper around the REAL reference Dattorro reverb.
 *
 * TEST INFRASTRUCTURE ONLY.  oracle/Makefile compiles this file together with
 * /root/reference/libs/dattorro-verb/verb.cpp (from where it lies; nothing is copied) into
 * oracle/_ref/libverb_ref.so.  The reference's own functions are C++-mangled
 * (verb.h has no extern "C"), so this wrapper re-exports a small extern "C" batch API that
 * tests/ and bench.py's cpu_baseline leg call through ctypes:
 *   - per-instance per-sample loop exactly like the reference call pattern
 *     (DattorroVerb_process + getLeft/getRight per frame; ReverbFx.cpp:11-27 for stereo in)
 *   - instances split statically over OpenMP threads.
 */
#include <cstdint>
#include <cstdlib>
#include "verb.h"

extern "C" {

struct ref_bank {
    int n;
    sDattorroVerb **v;
};

void *ref_verb_create(int n)
{
    if (n <= 0) return nullptr;
    ref_bank *b = static_cast<ref_bank *>(std::calloc(1, sizeof(ref_bank)));
    b->n = n;
    b->v = static_cast<sDattorroVerb **>(std::calloc((size_t)n, sizeof(sDattorroVerb *)));
    for (int i = 0; i < n; i++) b->v[i] = DattorroVerb_create();
    return b;
}

void ref_verb_destroy(void *p)
{
    ref_bank *b = static_cast<ref_bank *>(p);
    if (!b) return;
    for (int i = 0; i < b->n; i++)
        if (b->v[i]) DattorroVerb_delete(b->v[i]);
    std::free(b->v);
    std::free(b);
}

/* field order = oracle.h ODT_* */
int ref_verb_set(void *p, int inst, int field, float value)
{
    ref_bank *b = static_cast<ref_bank *>(p);
    if (!b || inst < 0 || inst >= b->n) return -1;
    sDattorroVerb *v = b->v[inst];
    switch (field) {
    case 0: DattorroVerb_setPreDelay(v, value); break;
    case 1: DattorroVerb_setPreFilter(v, value); break;
    case 2: DattorroVerb_setInputDiffusion1(v, value); break;
    case 3: DattorroVerb_setInputDiffusion2(v, value); break;
    case 4: DattorroVerb_setDecayDiffusion(v, value); break;
    case 5: DattorroVerb_setDecay(v, value); break;
    case 6: DattorroVerb_setDamping(v, value); break;
    default: return -1;
    }
    return 0;
}

/* in [in_ch][n_frames][n], out [2][n_frames][n] */
int ref_verb_process(void *p, const float *in, int in_ch, float *out, int n_frames, int n_threads)
{
    ref_bank *b = static_cast<ref_bank *>(p);
    if (!b || (in_ch != 1 && in_ch != 2)) return -1;
    const long n = b->n;
    const long plane = n * (long)n_frames;
    (void)n_threads;
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
#endif
    for (long i = 0; i < n; i++) {
        sDattorroVerb *v = b->v[i];
        for (int f = 0; f < n_frames; f++) {
            float x = in[(long)f * n + i];
            if (in_ch == 2) x = (x + in[plane + (long)f * n + i]) / 2;
            DattorroVerb_process(v, x);
            out[(long)f * n + i] = DattorroVerb_getLeft(v);
            out[plane + (long)f * n + i] = DattorroVerb_getRight(v);
        }
    }
    return 0;
}

}  // extern "C"
