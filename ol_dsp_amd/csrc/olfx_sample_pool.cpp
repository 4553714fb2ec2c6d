// ol_dsp_amd/csrc/olfx_sample_pool.cpp -- per-instance, per-sample operators over the batch
// engine (include/olfx_sample.h: contract; include/olfx_dattorro.h, include/olfx_fx.hpp and
// include/olfx_ref.hpp: the reference's names on top).
//
// A generation = the instances of one (kind, sample rate) created before the pool first ran them
// = one engine of that many instances.  Per-frame calls fill a host ring of `depth` input blocks
// [depth][in_ch][block][n]: an instance may run up to `depth` blocks ahead of the engine, in any
// order relative to the other instances (frame-major callbacks, or instance-major hosts that run
// each object over its whole buffer in turn, modules/juce/host/host.cpp:682).  Block b runs once
// every live instance has given all its frames, blocks in order; the instance whose frame
// completes the last missing block runs it (and any later blocks that are complete too).  An
// instance's frame p returns the engine's output frame p - depth * block, from a ring of depth + 1
// output blocks: an instance giving input block b reads output block b - depth, whose slot only the
// run of block b + 1 rewrites, and that run waits for this instance's input block b + 1.  Calls
// take effect at the instance's next block boundary at or after its position (never on frames it
// gave before the call): applied at once when that boundary is the engine's next block, else
// queued with that block as target and applied, in call order, right before it runs.
//
// Locking.  The per-frame call (olfx_sample_process) takes no lock except once per block (its
// frame that completes a block takes the generation's mutex to count it and run what is
// complete): it touches only its own instance's column of the rings and atomics.  Parameter /
// note / control calls take the generation's mutex.  Only create / destroy / the first run
// (freeze) take the pool's mutex (the list of open generations).  Different generations never
// share a lock.
#include <atomic>
#include <cmath>
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
    uint32_t idx;                   // engine instance
    std::atomic<uint64_t> given;    // frames given so far (its position in the generation's stream)
};

namespace {

struct PendingOp {      // a call waiting for a block boundary
    enum { PARAM, MEMBER, EVENT, CONTROL, UPDATE } type;
    uint32_t inst, field;
    float value;
    uint8_t a, b, c;
    uint64_t target;    // applied right before block `target` runs
};

constexpr uint32_t kMaxDepth = 8;

struct Generation {
    int kind, device;
    float sr;
    uint32_t block, depth, ich, och;
    std::mutex mu;                        // pending, engine calls, run_complete, members' slots, complete[]
    std::atomic<olfx_engine *> e{nullptr};  // created when the generation first runs
    std::vector<olfx_sample *> members;   // fixed once frozen (destroyed slots become null)
    std::vector<PendingOp> pending;
    std::vector<float> in;                // [depth][ich][block][n]: input block b in slot b % depth
    std::vector<float> out;               // [depth + 1][och][block][n]: output block b in slot b % (depth + 1)
    std::atomic<uint32_t> live{0};
    uint32_t complete[kMaxDepth] = {};    // live instances that gave all of block b (slot b % depth)
    std::atomic<uint64_t> blocks{0};      // blocks run so far

    size_t n() const { return members.size(); }
    float *in_block(uint64_t b) { return in.data() + (size_t)(b % depth) * (ich ? ich : 1) * block * n(); }
    float *out_block(uint64_t b) { return out.data() + (size_t)(b % (depth + 1)) * och * block * n(); }
};

std::mutex g_mu;                          // g_open, the pool config, generation membership
int g_device = 0;
uint32_t g_block = 256, g_depth = 1;
std::vector<Generation *> g_open;         // generations accepting members, one per (kind, sr)

int fail(int code, const char *what) {
    olfx::internal_set_error(what);
    return code;
}

int engine_fail(Generation *g, int code, const char *call) {
    char buf[512];
    std::snprintf(buf, sizeof buf, "%s: %s", call, olfx_last_error(g->e.load()));
    return fail(code, buf);
}

int apply(Generation *g, const PendingOp &op) {
    olfx_engine *e = g->e.load();
    switch (op.type) {
    case PendingOp::PARAM: return olfx_set_param(e, op.inst, op.field, op.value);
    case PendingOp::MEMBER: return olfx_set_member(e, op.inst, op.field, op.value);
    case PendingOp::EVENT: {
        olfx_voice_event ev{};
        ev.inst = op.inst; ev.type = op.a; ev.note = op.b; ev.velocity = op.c; ev.value = op.value;
        return olfx_voice_events(e, &ev, 1);
    }
    case PendingOp::CONTROL: {
        olfx_control_event ev{};
        ev.inst = op.inst; ev.control = op.a; ev.source = op.b; ev.value = op.value;
        return olfx_control(e, &ev, 1);
    }
    case PendingOp::UPDATE: return olfx_update(e, op.inst, 1);
    }
    return OLFX_E_ARG;
}

// the queued calls whose boundary is block `upto` or earlier, in call order (an instance's
// targets never decrease, and calls of different instances commute).  Caller holds g->mu.
int apply_pending(Generation *g, uint64_t upto) {
    size_t keep = 0;
    for (size_t k = 0; k < g->pending.size(); ++k) {
        const PendingOp &op = g->pending[k];
        if (op.target > upto) {
            g->pending[keep++] = op;
            continue;
        }
        const int rc = apply(g, op);
        if (rc) {
            g->pending.erase(g->pending.begin() + (ptrdiff_t)keep, g->pending.begin() + (ptrdiff_t)k + 1);
            return engine_fail(g, rc, "applying a queued call");
        }
    }
    g->pending.resize(keep);
    return OLFX_OK;
}

// Caller holds g_mu and g->mu.
int freeze(Generation *g) {
    for (auto it = g_open.begin(); it != g_open.end(); ++it)
        if (*it == g) { g_open.erase(it); break; }
    const uint32_t n = (uint32_t)g->members.size();
    olfx_engine *e = nullptr;
    int rc = olfx_create(g->kind, g->device, n, g->sr, g->block, &e);
    if (rc) {
        char buf[512];
        std::snprintf(buf, sizeof buf, "olfx_create(kind %d, %u instances, device %d): %s", g->kind, n, g->device,
                      olfx_last_error(nullptr));
        return fail(rc, buf);
    }
    try {
        g->in.assign((size_t)g->depth * (g->ich ? g->ich : 1) * g->block * n, 0.f);
        g->out.assign((size_t)(g->depth + 1) * g->och * g->block * n, 0.f);
    } catch (const std::bad_alloc &) {
        olfx_destroy(e);
        return fail(OLFX_E_NOMEM, "olfx_sample: out of host memory for the generation's blocks");
    }
    g->e.store(e, std::memory_order_release);
    return apply_pending(g, ~0ull);
}

// Run every block that is complete, in order: block R = blocks needs each live instance's whole
// input block R (complete[R % depth] == live).  Caller holds g->mu.
int run_complete(Generation *g) {
    for (;;) {
        const uint64_t b = g->blocks.load(std::memory_order_relaxed);
        const uint32_t live = g->live.load();
        if (live == 0 || g->complete[b % g->depth] != live) return OLFX_OK;
        int rc = apply_pending(g, b);
        if (rc) return rc;
        rc = olfx_process(g->e.load(), g->ich ? g->in_block(b) : nullptr, g->out_block(b), g->block, OLFX_IO_HOST,
                          nullptr);
        if (rc) return engine_fail(g, rc, "olfx_process");
        g->complete[b % g->depth] = 0;          // the slot now counts block b + depth
        // release: an instance that reads the new count (acquire) sees this run's outputs, and may
        // refill input slot b % depth
        g->blocks.store(b + 1, std::memory_order_release);
        // the calls queued for block b + 1 land now: queue_or_apply applies a later call with that
        // target at once, so none may stay queued behind it (an instance's calls keep call order)
        rc = apply_pending(g, b + 1);
        if (rc) return rc;
    }
}

// a call lands at the instance's next block boundary at or after its position.  Invariant (held
// under g->mu): every queued call targets a block past the engine's next one, so a call applied at
// once never overtakes a queued call of the same instance
int queue_or_apply(olfx_sample *s, PendingOp op) {
    Generation *g = s->g;
    std::lock_guard<std::mutex> lk(g->mu);
    const uint64_t at = s->given.load(std::memory_order_relaxed);
    op.target = (at + g->block - 1) / g->block;
    // before the engine exists, or a boundary past the engine's next block: queued
    if (!g->e.load() || op.target > g->blocks.load(std::memory_order_relaxed)) {
        g->pending.push_back(op);
        return OLFX_OK;
    }
    const int rc = apply(g, op);
    return rc ? engine_fail(g, rc, "olfx_sample call") : OLFX_OK;
}

}  // namespace

extern "C" {

int olfx_sample_pool_config_depth(int device, uint32_t block, uint32_t depth) {
    if (device < 0 || block == 0 || (block & 3u) || depth == 0 || depth > kMaxDepth)
        return fail(OLFX_E_ARG, "olfx_sample_pool_config: bad argument");
    std::lock_guard<std::mutex> lk(g_mu);
    g_device = device;
    g_block = block;
    g_depth = depth;
    return OLFX_OK;
}

int olfx_sample_pool_config(int device, uint32_t block) { return olfx_sample_pool_config_depth(device, block, 1); }

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
            if (c->kind == kind && c->sr == sample_rate && c->device == g_device && c->block == g_block &&
                c->depth == g_depth)
                g = c;
        if (!g) {
            g = new Generation;
            g->kind = kind; g->device = g_device; g->sr = sample_rate; g->block = g_block; g->depth = g_depth;
            g->ich = info.in_channels; g->och = info.out_channels;
            g_open.push_back(g);
        }
        std::lock_guard<std::mutex> gl(g->mu);
        s->g = g;
        s->idx = (uint32_t)g->members.size();
        s->given.store(0);
        g->members.push_back(s);
        g->live.fetch_add(1);
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
    int rc = OLFX_OK;
    bool last = false;
    {
        std::lock_guard<std::mutex> gl(g->mu);
        g->members[s->idx] = nullptr;
        // un-count the blocks it completed that have not run
        const uint64_t R = g->blocks.load(), given = s->given.load();
        for (uint64_t b = R; b < R + g->depth && (b + 1) * g->block <= given; ++b) --g->complete[b % g->depth];
        const uint32_t live = g->live.fetch_sub(1) - 1;
        if (g->e.load() && g->ich) {   // the slot keeps running on silence, unobserved
            const size_t n = g->members.size();
            for (uint32_t q = 0; q < g->depth; ++q)
                for (uint32_t c = 0; c < g->ich; ++c)
                    for (uint32_t f = 0; f < g->block; ++f)
                        g->in[(((size_t)q * g->ich + c) * g->block + f) * n + s->idx] = 0.f;
        }
        if (live == 0) last = true;
        else if (g->e.load()) rc = run_complete(g);   // the rest may have waited only for this one
    }
    delete s;
    if (last) {
        for (auto it = g_open.begin(); it != g_open.end(); ++it)
            if (*it == g) { g_open.erase(it); break; }
        if (olfx_engine *e = g->e.load()) olfx_destroy(e);
        delete g;
    }
    return rc;
}

int olfx_sample_set_param(olfx_sample *s, uint32_t field, float value) {
    if (!s) return OLFX_E_ARG;
    return queue_or_apply(s, PendingOp{PendingOp::PARAM, s->idx, field, value, 0, 0, 0});
}

int olfx_sample_set_member(olfx_sample *s, uint32_t field, float value) {
    if (!s) return OLFX_E_ARG;
    return queue_or_apply(s, PendingOp{PendingOp::MEMBER, s->idx, field, value, 0, 0, 0});
}

int olfx_sample_note(olfx_sample *s, uint8_t type, uint8_t note, uint8_t velocity) {
    if (!s) return OLFX_E_ARG;
    if (s->g->ich != 0) return fail(OLFX_E_STATE, "olfx_sample_note: not a voice");
    if (type > OLFX_EV_GATE_OFF || note > 127) return fail(OLFX_E_ARG, "olfx_sample_note: bad event");
    return queue_or_apply(s, PendingOp{PendingOp::EVENT, s->idx, 0, 0.f, type, note, velocity});
}

int olfx_sample_voice_event(olfx_sample *s, uint8_t type, uint8_t note, uint8_t velocity, float value) {
    if (!s) return OLFX_E_ARG;
    if (s->g->ich != 0) return fail(OLFX_E_STATE, "olfx_sample_voice_event: not a voice");
    // validated here too, so a queued event cannot fail later at the block boundary
    if (type > OLFX_EV_SET_FREQUENCY || note > 127 || (type == OLFX_EV_SET_FREQUENCY && !std::isfinite(value)))
        return fail(OLFX_E_ARG, "olfx_sample_voice_event: bad event");
    return queue_or_apply(s, PendingOp{PendingOp::EVENT, s->idx, 0, value, type, note, velocity});
}

int olfx_sample_update(olfx_sample *s) {
    if (!s) return OLFX_E_ARG;
    return queue_or_apply(s, PendingOp{PendingOp::UPDATE, s->idx, 0, 0.f, 0, 0, 0});
}

int olfx_sample_control(olfx_sample *s, uint8_t control, int source, float value) {
    if (!s || (source != OLFX_CTL_MIDI && source != OLFX_CTL_HARDWARE)) return OLFX_E_ARG;
    return queue_or_apply(s, PendingOp{PendingOp::CONTROL, s->idx, 0, value, control, (uint8_t)source, 0});
}

int olfx_sample_process(olfx_sample *s, const float *in, float *out) {
    if (!s || !out || (s->g->ich && !in)) return OLFX_E_ARG;
    Generation *g = s->g;
    if (!g->e.load(std::memory_order_acquire)) {
        std::lock_guard<std::mutex> lk(g_mu);
        std::lock_guard<std::mutex> gl(g->mu);
        if (!g->e.load()) {
            const int rc = freeze(g);
            if (rc) return rc;
        }
    }
    const uint64_t p = s->given.load(std::memory_order_relaxed);     // written by this instance only
    const uint64_t R = g->blocks.load(std::memory_order_acquire);    // pairs with run_complete's release
    const uint64_t B = g->block, b = p / B;
    if (b >= R + g->depth) {
        char buf[320];
        std::snprintf(buf, sizeof buf,
                      "olfx_sample_process: instance %u started block %llu before the other %u live instances of "
                      "its generation finished block %llu (an instance may run at most %u block(s) ahead: "
                      "olfx_sample_pool_config_depth, olfx_sample.h)",
                      s->idx, (unsigned long long)b, g->live.load() - 1, (unsigned long long)R, g->depth);
        return fail(OLFX_E_STATE, buf);
    }
    const size_t n = g->members.size();
    const size_t at = (size_t)(p % B) * n + s->idx;
    const size_t plane = (size_t)B * n;
    float *ib = g->in_block(b);
    for (uint32_t c = 0; c < g->ich; ++c) ib[c * plane + at] = in[c];
    // this frame's output: the engine's frame p - depth * block (zeros before it exists); that
    // block has run (b - depth < R) and its slot is not rewritten before this instance gives block b + 1
    if (b < g->depth) {
        for (uint32_t c = 0; c < g->och; ++c) out[c] = 0.f;
    } else {
        const float *o = g->out_block(b - g->depth);
        for (uint32_t c = 0; c < g->och; ++c) out[c] = o[c * plane + at];
    }
    s->given.store(p + 1, std::memory_order_relaxed);
    if (p % B == B - 1) {            // its last frame of block b: count it, run what is complete
        std::lock_guard<std::mutex> gl(g->mu);
        ++g->complete[b % g->depth];
        return run_complete(g);
    }
    return OLFX_OK;
}

uint32_t olfx_sample_latency(const olfx_sample *s) { return s ? s->g->block * s->g->depth : 0; }
uint32_t olfx_sample_generation_size(const olfx_sample *s) { return s ? (uint32_t)s->g->members.size() : 0; }
uint32_t olfx_sample_index(const olfx_sample *s) { return s ? s->idx : 0; }

}  // extern "C"
