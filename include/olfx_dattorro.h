/*
 * include/olfx_dattorro.h -- the reference's dattorro-verb C API, by name, over the GPU engine
 * (libolfx.so).  SURVEY section 8b: "also extern "C" DattorroVerb_* with the same names and
 * signatures".
 *
 * Replaces, function for function, libs/dattorro-verb/verb.h:5-26 (bodies verb.cpp:137-325):
 *   DattorroVerb_create / _delete          verb.h:5,8    (verb.cpp:225-251)
 *   DattorroVerb_setPreDelay ... setDamping verb.h:10-16  (verb.cpp:137-170)
 *   DattorroVerb_process                   verb.h:19     (verb.cpp:258-299)
 *   DattorroVerb_getLeft / getRight        verb.h:22,25  (verb.cpp:302-325)
 *
 * libolfx.so exports each name twice: with C linkage (this header) and with the C++ linkage the
 * reference's own callers bind to -- verb.h has no extern "C", so modules/fxlib/ReverbFx.cpp:16-36
 * compiled against verb.h links to the mangled names (_Z20DattorroVerb_processP13sDattorroVerbf
 * ...).  Either way a caller swaps verb.cpp for libolfx.so without a source change.
 *
 * How per-sample calls reach a batch GPU kernel: every instance created here is an olfx_sample
 * of kind OLFX_KIND_DATTORRO at 48 kHz (include/olfx_sample.h) and joins that process-wide pool.
 * Instances created before the pool first runs form one engine (a "generation") of N instances on
 * the GPU; instances created later start the next generation.  DattorroVerb_process
 * buffers the sample; when every live instance of a generation has been given `block` samples,
 * the generation runs one olfx_process over the whole block for all of them.  Consequences,
 * stated as the interface contract:
 *   - Latency: getLeft/getRight after the k-th process call return the reference's output for
 *     sample k - D * block (0 before; D = the pool depth, 1 by default).  Bit-exact otherwise (the
 *     engine is, verb.cpp order).
 *   - Call order: any interleaving in which no instance runs more than the pool depth D (default
 *     1) blocks ahead of the slowest live one: the per-frame callback shape of every reference
 *     caller (ReverbFx_process per frame; workout_buddy / Daisy callbacks), and hosts that run
 *     each reverb over its whole buffer in turn with D = buffer / block, or ceil(buffer / block) + 1
 *     for a buffer that is not a multiple of the block (olfx_dattorro_pool_config_depth; the latency
 *     is then D blocks).  An instance that runs D
 *     blocks ahead of the others is an error.
 *   - Setters take effect at the next block boundary (olfx_set_params), not the next sample.
 * Errors: the reference functions return void (create returns NULL on allocation failure,
 * verb.cpp:227).  Any other failure -- no GPU, a HIP error, a lockstep violation -- prints the
 * reason to stderr and aborts: there is no CPU fallback behind these names.
 */
#ifndef OLFX_DATTORRO_H
#define OLFX_DATTORRO_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef float t_sample;            /* verb.h:1 */
struct sDattorroVerb;              /* opaque, as in verb.h:2 */

struct sDattorroVerb *DattorroVerb_create(void);
void DattorroVerb_delete(struct sDattorroVerb *v);

void DattorroVerb_setPreDelay(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setPreFilter(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setInputDiffusion1(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setInputDiffusion2(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setDecayDiffusion(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setDecay(struct sDattorroVerb *v, t_sample value);
void DattorroVerb_setDamping(struct sDattorroVerb *v, t_sample value);

void DattorroVerb_process(struct sDattorroVerb *v, t_sample in);
t_sample DattorroVerb_getLeft(struct sDattorroVerb *v);
t_sample DattorroVerb_getRight(struct sDattorroVerb *v);

/* ---- pool control (new; not in verb.h) ---- */
/* Device and block (frames per GPU call = the latency, a positive multiple of 4) used by
   generations created after this call -- the setting of olfx_sample_pool_config, shared with the
   other per-sample operators.  Defaults: device 0, block 256.  Returns OLFX_OK (0) or OLFX_E_ARG. */
int olfx_dattorro_pool_config(int device, uint32_t block);
/* The same with the pool depth D (1..8; olfx_sample_pool_config_depth): instances may run up to D
   blocks ahead of each other (e.g. each reverb over a whole host buffer of D blocks in turn); the
   latency is D * block. */
int olfx_dattorro_pool_config_depth(int device, uint32_t block, uint32_t depth);
/* The latency in samples of instance v (its generation's depth x block). */
uint32_t olfx_dattorro_latency(const struct sDattorroVerb *v);
/* Generation facts: instances in v's generation and v's index in it (the engine instance). */
uint32_t olfx_dattorro_generation_size(const struct sDattorroVerb *v);
uint32_t olfx_dattorro_index(const struct sDattorroVerb *v);

#ifdef __cplusplus
}
#endif
#endif /* OLFX_DATTORRO_H */
