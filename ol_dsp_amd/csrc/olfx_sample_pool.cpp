// ol_dsp_amd/csrc/olfx_sample_pool.cpp -- per-instance, per-sample operators over the batch
// engine (include/olfx_sample.h: contract; include/olfx_dattorro.h and include/olfx_fx.hpp: the
// reference's names on top).
//
// A generation = the instances of one (kind, sample rate) created before the pool first ran them
// = one engine of that many instances.  Per-frame calls fill a host block [in_ch][block][n]; the
// last instance to complete a block runs the whole generation once.  Outputs are double-buffered
// by block parity: while an instance feeds block b it reads block b-1's outputs, so the run that
// writes block b's never races a reader.  Parameter / note / control calls made before the
// engine exists or while a block is being filled are queued and applied, in order, when it is
// created or right after that block's run: a call never reaches frames given before it.
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/olfx.h"
#include "../../include/olfx_sample.h"
#include "olfx_internal.h"

namespace {

struct Generation;

}  // namespace

struct olfx_sample {
    Generation *g;
    uint32_t idx;       // engine instance
    uint32_t pos;       // frames of the current block given so far
};

namespace {

struct PendingOp {      // a call waiting for the next block boundary
    enum { PARAM, NOTE, CONTROL } type;
    uint32_t inst, field;
    float value;
    uint8_t a, b, c;
};

struct Generation {
    int kind, device;
    float sr;
    uint32_t block, ich, och;
    olfx_engine *e = nullptr;             // created when the generation first runs
    std::vector<olfx_sample *> members;
    std::vector<PendingOp> pending;
    std::vector<float> in;                // [ich][block][n]
    std::vector<float> out[2];            // [och][block][n], by block parity
    uint32_t live = 0, complete = 0;
    uint64_t given = 0;                   // frames given for the block being filled (all instances)
    uint64_t blocks = 0;                  // blocks run so far
};

std::mutex g_mu;
int g_device = 0;
uint32_t g_block = 256;
std::vector<Generation *> g_open;         // generations accepting members, one per (kind, sr)

int fail(int code, const char *what) {
    olfx::internal_set_error(what);
    return code;
}

int engine_fail(Generation *g, int code, const char *call) {
    char buf[512];
    std::snprintf(buf, sizeof buf, "%s: %s", call, olfx_last_error(g->e));
    return fail(code, buf);
}

int apply(Generation *g, const PendingOp &op) {
    switch (op.type) {
    case PendingOp::PARAM: return olfx_set_param(g->e, op.inst, op.field, op.value);
    case PendingOp::NOTE: {
        olfx_event ev{};
        ev.inst = op.inst; ev.type = op.a; ev.note = op.b; ev.velocity = op.c;
        return olfx_note_events(g->e, &ev, 1);
    }
    case PendingOp::CONTROL: {
        olfx_control_event ev{};
        ev.inst = op.inst; ev.control = op.a; ev.source = op.b; ev.value = op.value;
        return olfx_control(g->e, &ev, 1);
    }
    }
    return OLFX_E_ARG;
}

// calls made while a block was being filled take effect at the next block boundary: after the
// run of that block (rounding the boundary up, so no call reaches frames given before it)
int apply_pending(Generation *g) {
    for (const PendingOp &op : g->pending) {
        const int rc = apply(g, op);
        if (rc) return engine_fail(g, rc, "applying a queued call");
    }
    g->pending.clear();
    return OLFX_OK;
}

int freeze(Generation *g) {
    for (auto it = g_open.begin(); it != g_open.end(); ++it)
        if (*it == g) { g_open.erase(it); break; }
    const uint32_t n = (uint32_t)g->members.size();
    int rc = olfx_create(g->kind, g->device, n, g->sr, g->block, &g->e);
    if (rc) {
        g->e = nullptr;
        char buf[512];
        std::snprintf(buf, sizeof buf, "olfx_create(kind %d, %u instances, device %d): %s", g->kind, n, g->device,
                      olfx_last_error(nullptr));
        return fail(rc, buf);
    }
    if ((rc = apply_pending(g))) return rc;
    g->in.assign((size_t)(g->ich ? g->ich : 1) * g->block * n, 0.f);
    g->out[0].assign((size_t)g->och * g->block * n, 0.f);
    g->out[1].assign((size_t)g->och * g->block * n, 0.f);
    return OLFX_OK;
}

int run_block(Generation *g) {
    std::vector<float> &o = g->out[g->blocks & 1];
    const int rc = olfx_process(g->e, g->ich ? g->in.data() : nullptr, o.data(), g->block, OLFX_IO_HOST, nullptr);
    if (rc) return engine_fail(g, rc, "olfx_process");
    ++g->blocks;
    g->complete = 0;
    g->given = 0;
    for (olfx_sample *m : g->members)
        if (m) m->pos = 0;
    return apply_pending(g);
}

int queue_or_apply(olfx_sample *s, const PendingOp &op) {
    Generation *g = s->g;
    if (!g->e || g->given) {   // before the engine exists, or mid-block: at the next boundary
        g->pending.push_back(op);
        return OLFX_OK;
    }
    const int rc = apply(g, op);
    return rc ? engine_fail(g, rc, "olfx_sample call") : OLFX_OK;
}

}  // namespace

extern "C" {

int olfx_sample_pool_config(int device, uint32_t block) {
    if (device < 0 || block == 0 || (block & 3u)) return fail(OLFX_E_ARG, "olfx_sample_pool_config: bad argument");
    std::lock_guard<std::mutex> lk(g_mu);
    g_device = device;
    g_block = block;
    return OLFX_OK;
}

int olfx_sample_create(int kind, float sample_rate, olfx_sample **out) {
    if (!out) return fail(OLFX_E_ARG, "olfx_sample_create: null out");
    *out = nullptr;
    olfx_kind_info info;
    int rc = olfx_kind_info_get(kind, sample_rate, &info);
    if (rc) return rc;
    if (!(sample_rate > 1000.f && sample_rate <= 384000.f)) return fail(OLFX_E_ARG, "olfx_sample_create: bad sample rate");
    std::lock_guard<std::mutex> lk(g_mu);
    olfx_sample *s = new (std::nothrow) olfx_sample{};
    if (!s) return fail(OLFX_E_NOMEM, "olfx_sample_create: out of host memory");
    try {
        Generation *g = nullptr;
        for (Generation *c : g_open)
            if (c->kind == kind && c->sr == sample_rate && c->device == g_device && c->block == g_block) g = c;
        if (!g) {
            g = new Generation;
            g->kind = kind; g->device = g_device; g->sr = sample_rate; g->block = g_block;
            g->ich = info.in_channels; g->och = info.out_channels;
            g_open.push_back(g);
        }
        *s = olfx_sample{g, (uint32_t)g->members.size(), 0};
        g->members.push_back(s);
        ++g->live;
    } catch (const std::bad_alloc &) {
        delete s;
        return fail(OLFX_E_NOMEM, "olfx_sample_create: out of host memory");
    }
    *out = s;
    return OLFX_OK;
}

int olfx_sample_destroy(olfx_sample *s) {
    if (!s) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    Generation *g = s->g;
    g->members[s->idx] = nullptr;
    if (s->pos == g->block) --g->complete;
    --g->live;
    if (g->e && g->ich) {   // the slot keeps running on silence, unobserved
        const size_t n = g->members.size();
        for (uint32_t c = 0; c < g->ich; ++c)
            for (uint32_t f = 0; f < g->block; ++f) g->in[((size_t)c * g->block + f) * n + s->idx] = 0.f;
    }
    delete s;
    int rc = OLFX_OK;
    if (g->live == 0) {
        for (auto it = g_open.begin(); it != g_open.end(); ++it)
            if (*it == g) { g_open.erase(it); break; }
        if (g->e) olfx_destroy(g->e);
        delete g;
    } else if (g->e && g->complete == g->live) {
        rc = run_block(g);   // the remaining instances were only waiting for this one
    }
    return rc;
}

int olfx_sample_set_param(olfx_sample *s, uint32_t field, float value) {
    if (!s) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    PendingOp op{PendingOp::PARAM, s->idx, field, value, 0, 0, 0};
    return queue_or_apply(s, op);
}

int olfx_sample_note(olfx_sample *s, uint8_t type, uint8_t note, uint8_t velocity) {
    if (!s) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    if (s->g->ich != 0) return fail(OLFX_E_STATE, "olfx_sample_note: not a voice");
    PendingOp op{PendingOp::NOTE, s->idx, 0, 0.f, type, note, velocity};
    return queue_or_apply(s, op);
}

int olfx_sample_control(olfx_sample *s, uint8_t control, int source, float value) {
    if (!s || (source != OLFX_CTL_MIDI && source != OLFX_CTL_HARDWARE)) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    PendingOp op{PendingOp::CONTROL, s->idx, 0, value, control, (uint8_t)source, 0};
    return queue_or_apply(s, op);
}

int olfx_sample_process(olfx_sample *s, const float *in, float *out) {
    if (!s || !out || (s->g->ich && !in)) return OLFX_E_ARG;
    std::lock_guard<std::mutex> lk(g_mu);
    Generation *g = s->g;
    int rc;
    if (!g->e && (rc = freeze(g))) return rc;
    if (s->pos == g->block) {
        char buf[256];
        std::snprintf(buf, sizeof buf,
                      "olfx_sample_process: instance %u started block %llu before the other %u live instances of "
                      "its generation finished block %llu (calls must be frame-major, olfx_sample.h)",
                      s->idx, (unsigned long long)(g->blocks + 1), g->live - 1, (unsigned long long)g->blocks);
        return fail(OLFX_E_STATE, buf);
    }
    const size_t n = g->members.size();
    for (uint32_t c = 0; c < g->ich; ++c) g->in[((size_t)c * g->block + s->pos) * n + s->idx] = in[c];
    // this frame's output: frame s->pos of the previous block (zeros before the first block ran)
    for (uint32_t c = 0; c < g->och; ++c)
        out[c] = g->blocks == 0 ? 0.f : g->out[(g->blocks - 1) & 1][((size_t)c * g->block + s->pos) * n + s->idx];
    ++g->given;
    if (++s->pos == g->block && ++g->complete == g->live) return run_block(g);
    return OLFX_OK;
}

uint32_t olfx_sample_latency(const olfx_sample *s) { return s ? s->g->block : 0; }
uint32_t olfx_sample_generation_size(const olfx_sample *s) { return s ? (uint32_t)s->g->members.size() : 0; }
uint32_t olfx_sample_index(const olfx_sample *s) { return s ? s->idx : 0; }

}  // extern "C"
