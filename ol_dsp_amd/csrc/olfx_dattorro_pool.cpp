// ol_dsp_amd/csrc/olfx_dattorro_pool.cpp -- the reference's per-sample dattorro-verb API
// (libs/dattorro-verb/verb.h:5-26) over the batch GPU engine.  Contract in include/olfx_dattorro.h.
//
// A generation = the instances created before the pool first ran them = one OLFX_KIND_DATTORRO
// engine of that many instances.  Per-sample calls fill a host block [2][block][n] (the mono input
// duplicated into both planes: the engine's (l+r)/2 of two equal floats is the float itself, so
// the kernel sees exactly verb.cpp's mono input); the last instance to complete a block runs the
// whole generation once.  Outputs are double-buffered by block parity: while an instance feeds
// block b it reads block b-1's outputs, so the flush that writes block b's never races a reader.
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/olfx.h"
#include "../../include/olfx_dattorro.h"

namespace {

struct Generation;

}  // namespace

struct sDattorroVerb {
    Generation *g;
    uint32_t idx;       // engine instance
    uint32_t pos;       // samples of the current block given so far
    int rd;             // output buffer (block parity) getLeft/getRight read; -1 = before block 1
    uint32_t rd_pos;    // frame within that block
};

namespace {

struct Generation {
    int device;
    uint32_t block;
    olfx_engine *e = nullptr;            // created when the generation first runs (freeze)
    std::vector<sDattorroVerb *> members;
    std::vector<float> params;           // [field][n] host shadow until the engine exists
    std::vector<float> in;               // [2][block][n]
    std::vector<float> out[2];           // [2][block][n], by block parity
    uint32_t live = 0, complete = 0;
    uint64_t blocks = 0;                 // blocks run so far
};

std::mutex g_mu;
int g_device = 0;
uint32_t g_block = 256;
Generation *g_open = nullptr;            // accepting new members (not yet run)

[[noreturn]] void fatal(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    std::fputs("olfx DattorroVerb: ", stderr);
    std::vfprintf(stderr, fmt, ap);
    std::fputc('\n', stderr);
    va_end(ap);
    std::abort();
}

// the reference defaults set by DattorroVerb_create (verb.cpp:215-221), in OLFX_DT_* order
const float kDefaults[OLFX_DT_NPARAMS] = {0.1f, 0.85f, 0.75f, 0.625f, 0.7f, 0.75f, 0.95f};

void freeze(Generation *g) {
    if (g == g_open) g_open = nullptr;
    const uint32_t n = (uint32_t)g->members.size();
    int rc = olfx_create(OLFX_KIND_DATTORRO, g->device, n, 48000.f, g->block, &g->e);
    if (rc) fatal("olfx_create(%u instances, device %d) failed: %s (code %d)", n, g->device, olfx_last_error(nullptr), rc);
    rc = olfx_set_params(g->e, 0, n, 0, OLFX_DT_NPARAMS, g->params.data());
    if (rc) fatal("olfx_set_params failed: %s (code %d)", olfx_last_error(g->e), rc);
    g->params.clear();
    g->in.assign((size_t)2 * g->block * n, 0.f);
    g->out[0].assign((size_t)2 * g->block * n, 0.f);
    g->out[1].assign((size_t)2 * g->block * n, 0.f);
}

void run_block(Generation *g) {
    std::vector<float> &o = g->out[g->blocks & 1];
    const int rc = olfx_process(g->e, g->in.data(), o.data(), g->block, OLFX_IO_HOST, nullptr);
    if (rc) fatal("olfx_process failed: %s (code %d)", olfx_last_error(g->e), rc);
    ++g->blocks;
    g->complete = 0;
    for (sDattorroVerb *m : g->members)
        if (m) m->pos = 0;
}

void set_field(sDattorroVerb *v, uint32_t field, float value) {
    if (!v) return;
    std::lock_guard<std::mutex> lk(g_mu);
    Generation *g = v->g;
    if (!g->e) {
        g->params[(size_t)field * g->members.size() + v->idx] = value;
        return;
    }
    const int rc = olfx_set_param(g->e, v->idx, field, value);
    if (rc) fatal("olfx_set_param failed: %s (code %d)", olfx_last_error(g->e), rc);
}

}  // namespace

namespace olfx_dv {

sDattorroVerb *create() {
    std::lock_guard<std::mutex> lk(g_mu);
    sDattorroVerb *v = new (std::nothrow) sDattorroVerb{};
    if (!v) return nullptr;                          // verb.cpp:227: NULL on allocation failure
    try {
        if (!g_open) {
            g_open = new Generation;
            g_open->device = g_device;
            g_open->block = g_block;
        }
        Generation *g = g_open;
        const uint32_t n_old = (uint32_t)g->members.size(), n = n_old + 1;
        std::vector<float> p((size_t)OLFX_DT_NPARAMS * n);
        for (uint32_t f = 0; f < OLFX_DT_NPARAMS; ++f) {
            for (uint32_t i = 0; i < n_old; ++i) p[(size_t)f * n + i] = g->params[(size_t)f * n_old + i];
            p[(size_t)f * n + n_old] = kDefaults[f];
        }
        g->params.swap(p);
        g->members.push_back(v);
        ++g->live;
        *v = sDattorroVerb{g, n_old, 0, -1, 0};
    } catch (const std::bad_alloc &) {
        delete v;
        return nullptr;
    }
    return v;
}

void destroy(sDattorroVerb *v) {
    if (!v) return;
    std::lock_guard<std::mutex> lk(g_mu);
    Generation *g = v->g;
    g->members[v->idx] = nullptr;
    if (v->pos == g->block) --g->complete;
    --g->live;
    if (g->e) {   // the slot keeps running on silence, unobserved
        for (int c = 0; c < 2; ++c)
            for (uint32_t f = 0; f < g->block; ++f) g->in[((size_t)c * g->block + f) * g->members.size() + v->idx] = 0.f;
    }
    delete v;
    if (g->live == 0) {
        if (g == g_open) g_open = nullptr;
        if (g->e) olfx_destroy(g->e);
        delete g;
    } else if (g->e && g->complete == g->live) {
        run_block(g);   // the remaining instances were only waiting for this one
    }
}

void process(sDattorroVerb *v, float x) {
    if (!v) return;
    std::lock_guard<std::mutex> lk(g_mu);
    Generation *g = v->g;
    if (!g->e) freeze(g);
    if (v->pos == g->block)
        fatal("instance %u started block %llu before the other %u live instances of its generation finished "
              "block %llu (per-sample calls must be frame-major, see olfx_dattorro.h)",
              v->idx, (unsigned long long)(g->blocks + 1), g->live - 1, (unsigned long long)g->blocks);
    const size_t n = g->members.size();
    g->in[(size_t)v->pos * n + v->idx] = x;
    g->in[((size_t)g->block + v->pos) * n + v->idx] = x;
    v->rd = g->blocks == 0 ? -1 : (int)((g->blocks - 1) & 1);
    v->rd_pos = v->pos;
    if (++v->pos == g->block && ++g->complete == g->live) run_block(g);
}

void set_field_cxx(sDattorroVerb *v, unsigned field, float value) { set_field(v, field, value); }

float get(const sDattorroVerb *v, int ch) {
    if (!v || v->rd < 0) return 0.f;
    const Generation *g = v->g;
    return g->out[v->rd][((size_t)ch * g->block + v->rd_pos) * g->members.size() + v->idx];
}

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

int olfx_dattorro_pool_config(int device, uint32_t block) {
    if (device < 0 || block == 0 || (block & 3u)) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    g_device = device;
    g_block = block;
    return OLFX_OK;
}
uint32_t olfx_dattorro_latency(const struct sDattorroVerb *v) { return v ? v->g->block : 0; }
uint32_t olfx_dattorro_generation_size(const struct sDattorroVerb *v) { return v ? (uint32_t)v->g->members.size() : 0; }
uint32_t olfx_dattorro_index(const struct sDattorroVerb *v) { return v ? v->idx : 0; }

}  // extern "C"
