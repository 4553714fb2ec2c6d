/*
 * include/olfx_sample.h -- per-instance, per-sample operators over the batch GPU engine.
 *
 * The reference's operators are objects processed one sample (one frame) at a time:
 *   ChorusEffect::init / setDepth / setRate / process(float)          README.md:114-128
 *   SynthVoice::Init / UpdateConfig / NoteOn / NoteOff / Process(out) modules/synthlib/SynthVoice.h:31-98,245-256
 *   ol::fx::FxRack<2>::Init / UpdateMidiControl / Process(in, out)   modules/fxlib/Fx.h:398-492
 *   DattorroVerb_create / _process / getLeft / getRight               libs/dattorro-verb/verb.h:5-26
 * An olfx_sample is one such object.  Every olfx_sample of one kind and sample rate created
 * before the pool first runs them joins one engine of that many instances (a "generation");
 * later ones start the next generation.  olfx_sample_process buffers one frame; block b of the
 * generation runs (one olfx_process over the whole block) once every live instance has been given
 * its frames of block b.  The contract, for a pool depth D (olfx_sample_pool_config_depth; 1 by
 * default):
 *   - Latency: the output frame returned by the k-th olfx_sample_process is the engine's output
 *     frame k - D * block (zeros for k < D * block); bit-identical to olfx_process otherwise.
 *   - Call order: any interleaving of the instances in which no instance runs more than D blocks
 *     ahead of the slowest live one.  D = 1 takes the per-frame callback shape of the reference's
 *     callers (every instance once per frame, frame-major) and instance-major hosts whose buffer is
 *     one block; D = buffer / block takes a host that runs each object over its whole buffer in
 *     turn (per-plugin processBlock, modules/juce/host/host.cpp:682), ceil(buffer / block) + 1 when
 *     the buffer is not a multiple of the block.  An instance D blocks ahead gets OLFX_E_STATE and
 *     its frame is not taken.
 *   - Parameters, note events and control changes take effect at the instance's first block
 *     boundary at or after the call (never on frames it gave before it), in call order (the JUCE
 *     host's queue, modules/juce/host/host.cpp:646-653).
 * include/olfx_dattorro.h puts the verb.h names on this pool; include/olfx_fx.hpp has the C++
 * classes with the reference's method names (olfx::ChorusEffect, olfx::SynthVoice, olfx::FxRack).
 */
#ifndef OLFX_SAMPLE_H
#define OLFX_SAMPLE_H
#include <stdint.h>

#include "olfx.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct olfx_sample olfx_sample;

/* Device and block (frames per GPU call = the latency; a positive multiple of 4) of generations
   created after this call, with depth 1.  Defaults: device 0, block 256. */
int olfx_sample_pool_config(int device, uint32_t block);
/* The same with the depth D (1..8): how many blocks an instance may run ahead of the others
   (host ring of D input blocks and D + 1 output blocks per generation); latency D * block. */
int olfx_sample_pool_config_depth(int device, uint32_t block, uint32_t depth);

/* A new instance of `kind` at `sample_rate`, in the reference's freshly initialised state.
   Host-only until its generation first runs (no device call here). */
int olfx_sample_create(int kind, float sample_rate, olfx_sample **out);
int olfx_sample_destroy(olfx_sample *s);

/* Per-instance parameter (OLFX_DT_* / OLFX_CH_* / OLFX_VC_* / OLFX_FR_* field and value, as
   olfx_set_param), note event (voices) and control change (as olfx_control). */
int olfx_sample_set_param(olfx_sample *s, uint32_t field, float value);
/* A member value without Update() (olfx_set_member: setters called before the reference's Init). */
int olfx_sample_set_member(olfx_sample *s, uint32_t field, float value);
int olfx_sample_note(olfx_sample *s, uint8_t type, uint8_t note, uint8_t velocity);
/* Any voice event (olfx_voice_event: GateOn / GateOff / SetFrequency as well) and Update(). */
int olfx_sample_voice_event(olfx_sample *s, uint8_t type, uint8_t note, uint8_t velocity, float value);
int olfx_sample_update(olfx_sample *s);
int olfx_sample_control(olfx_sample *s, uint8_t control, int source, float value);

/* One frame: in[in_channels] (NULL for voices) -> out[out_channels] (olfx_kind_info_get). */
int olfx_sample_process(olfx_sample *s, const float *in, float *out);

uint32_t olfx_sample_latency(const olfx_sample *s);          /* = depth x the generation's block */
uint32_t olfx_sample_generation_size(const olfx_sample *s);  /* instances in its engine */
uint32_t olfx_sample_index(const olfx_sample *s);            /* its instance in that engine */

#ifdef __cplusplus
}
#endif
#endif /* OLFX_SAMPLE_H */
