// ol_dsp_amd/csrc/olfx_dattorro_cxx.cpp -- the dattorro-verb API with the C++ linkage the
// reference's callers bind to.  libs/dattorro-verb/verb.h:5-26 declares its functions without
// extern "C", so C++ code compiled against it (modules/fxlib/ReverbFx.cpp:16-36) references the
// mangled names.  This translation unit declares the same signatures with C++ linkage (it must not
// see include/olfx_dattorro.h, whose extern "C" declarations would clash) and forwards to the pool
// in olfx_dattorro_pool.cpp.
typedef float t_sample;
struct sDattorroVerb;

namespace olfx_dv {
sDattorroVerb *create();
void destroy(sDattorroVerb *v);
void process(sDattorroVerb *v, float x);
float get(const sDattorroVerb *v, int ch);
void set_field_cxx(sDattorroVerb *v, unsigned field, float value);
}  // namespace olfx_dv

__attribute__((visibility("default"))) sDattorroVerb *DattorroVerb_create(void) { return olfx_dv::create(); }
__attribute__((visibility("default"))) void DattorroVerb_delete(sDattorroVerb *v) { olfx_dv::destroy(v); }
// field numbers: OLFX_DT_* (include/olfx.h), the order of verb.h:10-16's setters
__attribute__((visibility("default"))) void DattorroVerb_setPreDelay(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 0, x); }
__attribute__((visibility("default"))) void DattorroVerb_setPreFilter(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 1, x); }
__attribute__((visibility("default"))) void DattorroVerb_setInputDiffusion1(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 2, x); }
__attribute__((visibility("default"))) void DattorroVerb_setInputDiffusion2(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 3, x); }
__attribute__((visibility("default"))) void DattorroVerb_setDecayDiffusion(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 4, x); }
__attribute__((visibility("default"))) void DattorroVerb_setDecay(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 5, x); }
__attribute__((visibility("default"))) void DattorroVerb_setDamping(sDattorroVerb *v, t_sample x) { olfx_dv::set_field_cxx(v, 6, x); }
__attribute__((visibility("default"))) void DattorroVerb_process(sDattorroVerb *v, t_sample in) { olfx_dv::process(v, in); }
__attribute__((visibility("default"))) t_sample DattorroVerb_getLeft(sDattorroVerb *v) { return olfx_dv::get(v, 0); }
__attribute__((visibility("default"))) t_sample DattorroVerb_getRight(sDattorroVerb *v) { return olfx_dv::get(v, 1); }
