// ol_dsp_amd/csrc/olfx_dattorro_pool.cpp -- the reference's per-sample dattorro-verb API
// (libs/dattorro-verb/verb.h:5-26) on the per-sample pool (olfx_sample_pool.cpp).  Contract in
// include/olfx_dattorro.h.
//
// verb.h's process takes a mono sample; the engine's reverb takes stereo and feeds (l+r)/2
// (modules/fxlib/ReverbFx.cpp:13-16).  The sample goes into both channels: (x+x)/2 of a float is
// the float itself, so the kernel sees exactly verb.cpp's mono input.  getLeft/getRight return the
// outputs of the last process call.  The reference functions return void: any failure prints the
// reason and aborts (there is no CPU fallback behind these names).
#include <cstdio>
#include <cstdlib>
#include <new>

#include "../../include/olfx.h"
#include "../../include/olfx_dattorro.h"
#include "../../include/olfx_sample.h"

struct sDattorroVerb {
    olfx_sample *s;
    float out[2];
};

namespace {

[[noreturn]] void fatal(const char *call) {
    std::fprintf(stderr, "olfx DattorroVerb: %s: %s\n", call, olfx_last_error(nullptr));
    std::abort();
}

void set_field(sDattorroVerb *v, uint32_t field, float value) {
    if (v && olfx_sample_set_param(v->s, field, value)) fatal("set");
}

}  // namespace

namespace olfx_dv {

sDattorroVerb *create() {
    sDattorroVerb *v = new (std::nothrow) sDattorroVerb{};
    if (!v) return nullptr;                          // verb.cpp:227: NULL on allocation failure
    if (olfx_sample_create(OLFX_KIND_DATTORRO, 48000.f, &v->s)) {
        delete v;
        return nullptr;
    }
    return v;
}

void destroy(sDattorroVerb *v) {
    if (!v) return;
    if (olfx_sample_destroy(v->s)) fatal("delete");
    delete v;
}

void process(sDattorroVerb *v, float x) {
    if (!v) return;
    const float in[2] = {x, x};
    if (olfx_sample_process(v->s, in, v->out)) fatal("process");
}

void set_field_cxx(sDattorroVerb *v, unsigned field, float value) { set_field(v, field, value); }

float get(const sDattorroVerb *v, int ch) { return v ? v->out[ch] : 0.f; }

}  // namespace olfx_dv

extern "C" {

struct sDattorroVerb *DattorroVerb_create(void) { return olfx_dv::create(); }
void DattorroVerb_delete(struct sDattorroVerb *v) { olfx_dv::destroy(v); }
void DattorroVerb_setPreDelay(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_PREDELAY, value); }
void DattorroVerb_setPreFilter(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_PREFILTER, value); }
void DattorroVerb_setInputDiffusion1(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_INPUT_DIFFUSION1, value); }
void DattorroVerb_setInputDiffusion2(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_INPUT_DIFFUSION2, value); }
void DattorroVerb_setDecayDiffusion(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_DECAY_DIFFUSION, value); }
void DattorroVerb_setDecay(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_DECAY, value); }
void DattorroVerb_setDamping(struct sDattorroVerb *v, t_sample value) { set_field(v, OLFX_DT_DAMPING, value); }
void DattorroVerb_process(struct sDattorroVerb *v, t_sample in) { olfx_dv::process(v, in); }
t_sample DattorroVerb_getLeft(struct sDattorroVerb *v) { return olfx_dv::get(v, 0); }
t_sample DattorroVerb_getRight(struct sDattorroVerb *v) { return olfx_dv::get(v, 1); }

int olfx_dattorro_pool_config(int device, uint32_t block) { return olfx_sample_pool_config(device, block); }
int olfx_dattorro_pool_config_depth(int device, uint32_t block, uint32_t depth) {
    return olfx_sample_pool_config_depth(device, block, depth);
}
uint32_t olfx_dattorro_latency(const struct sDattorroVerb *v) { return v ? olfx_sample_latency(v->s) : 0; }
uint32_t olfx_dattorro_generation_size(const struct sDattorroVerb *v) { return v ? olfx_sample_generation_size(v->s) : 0; }
uint32_t olfx_dattorro_index(const struct sDattorroVerb *v) { return v ? olfx_sample_index(v->s) : 0; }

}  // extern "C"
