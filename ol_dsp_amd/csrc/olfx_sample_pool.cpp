// ol_dsp_amd/csrc/olfx_sample_pool.cpp -- per-instance, per-sample operators over the batch
// engine (include/olfx_sample.h: contract; include/olfx_dattorro.h, include/olfx_fx.hpp and
// include/olfx_ref.hpp: the reference's names on top).
//
// A generation = the instances of one (kind, sample rate) created before the pool first ran them
// = one engine of that many instances.  Per-frame calls fill a host block [in_ch][block][n]; the
// last instance to complete a block runs the whole generation once.  Outputs are double-buffered
// by block parity: while an instance feeds block b it reads block b-1's outputs, so the run that
// writes block b's never races a reader.  Parameter / note / control calls made before the
// engine exists or while a block is being filled are queued and applied, in order, when it is
// created or right after that block's run: a call never reaches frames given before it.
//
// Locking.  The per-frame call (olfx_sample_process) takes no lock: it touches only its own
// instance's column of the block and the generation's atomic counters; the instance that
// completes a block takes the generation's mutex to run it.  Parameter / note / control calls
// take the generation's mutex.  Only create / destroy / the first run (freeze) take the pool's
// mutex (the list of open generations).  Different generations never share a lock.
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
    std::atomic<uint32_t> pos;      // frames of the current block given so far
};

namespace {

struct PendingOp {      // a call waiting for the next block boundary
    enum { PARAM, MEMBER, EVENT, CONTROL, UPDATE } type;
    uint32_t inst, field;
    float value;
    uint8_t a, b, c;
};

struct Generation {
    int kind, device;
    float sr;
    uint32_t block, ich, och;
    std::mutex mu;                        // pending, engine calls, run_block, members' slots
    std::atomic<olfx_engine *> e{nullptr};  // created when the generation first runs
    std::vector<olfx_sample *> members;   // fixed once frozen (destroyed slots become null)
    std::vector<PendingOp> pending;
    std::vector<float> in;                // [ich][block][n]
    std::vector<float> out[2];            // [och][block][n], by block parity
    std::atomic<uint32_t> live{0}, complete{0};
    std::atomic<bool> filling{false};     // some instance has given a frame of the block being filled
    std::atomic<uint64_t> blocks{0};      // blocks run so far
};

std::mutex g_mu;                          // g_open, the pool config, generation membership
int g_device = 0;
uint32_t g_block = 256;
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

// calls made while a block was being filled take effect at the next block boundary: after the
// run of that block (rounding the boundary up, so no call reaches frames given before it).
// Caller holds g->mu.
int apply_pending(Generation *g) {
    for (const PendingOp &op : g->pending) {
        const int rc = apply(g, op);
        if (rc) return engine_fail(g, rc, "applying a queued call");
    }
    g->pending.clear();
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
        g->in.assign((size_t)(g->ich ? g->ich : 1) * g->block * n, 0.f);
        g->out[0].assign((size_t)g->och * g->block * n, 0.f);
        g->out[1].assign((size_t)g->och * g->block * n, 0.f);
    } catch (const std::bad_alloc &) {
        olfx_destroy(e);
        return fail(OLFX_E_NOMEM, "olfx_sample: out of host memory for the generation's block");
    }
    g->e.store(e, std::memory_order_release);
    return apply_pending(g);
}

// Caller holds g->mu; every live instance has given the whole block.
int run_block(Generation *g) {
    const uint64_t b = g->blocks.load(std::memory_order_relaxed);
    std::vector<float> &o = g->out[b & 1];
    const int rc = olfx_process(g->e.load(), g->ich ? g->in.data() : nullptr, o.data(), g->block, OLFX_IO_HOST, nullptr);
    if (rc) return engine_fail(g, rc, "olfx_process");
    g->complete.store(0, std::memory_order_relaxed);
    g->filling.store(false, std::memory_order_relaxed);
    // publish the new block count first, then each member's pos = 0 with release: a member that
    // reads its pos 0 (acquire) also sees the new count and this run's outputs
    g->blocks.store(b + 1, std::memory_order_release);
    for (olfx_sample *m : g->members)
        if (m) m->pos.store(0, std::memory_order_release);
    return apply_pending(g);
}

int queue_or_apply(olfx_sample *s, const PendingOp &op) {
    Generation *g = s->g;
    std::lock_guard<std::mutex> lk(g->mu);
    if (!g->e.load() || g->filling.load()) {   // before the engine exists, or mid-block: at the next boundary
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
        std::lock_guard<std::mutex> gl(g->mu);
        s->g = g;
        s->idx = (uint32_t)g->members.size();
        s->pos.store(0);
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
        if (s->pos.load() == g->block) g->complete.fetch_sub(1);
        const uint32_t live = g->live.fetch_sub(1) - 1;
        if (g->e.load() && g->ich) {   // the slot keeps running on silence, unobserved
            const size_t n = g->members.size();
            for (uint32_t c = 0; c < g->ich; ++c)
                for (uint32_t f = 0; f < g->block; ++f) g->in[((size_t)c * g->block + f) * n + s->idx] = 0.f;
        }
        if (live == 0) last = true;
        else if (g->e.load() && g->complete.load() == live) rc = run_block(g);   // the rest only waited for this one
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
    // pos first (acquire, pairs with run_block's release of pos = 0), then the block count: a reset
    // pos is never seen with the previous count (the output buffer of the wrong parity)
    const uint32_t pos = s->pos.load(std::memory_order_acquire);
    const uint64_t blocks = g->blocks.load(std::memory_order_acquire);
    if (pos == g->block) {
        char buf[256];
        std::snprintf(buf, sizeof buf,
                      "olfx_sample_process: instance %u started block %llu before the other %u live instances of "
                      "its generation finished block %llu (calls must be frame-major, olfx_sample.h)",
                      s->idx, (unsigned long long)(blocks + 1), g->live.load() - 1, (unsigned long long)blocks);
        return fail(OLFX_E_STATE, buf);
    }
    const size_t n = g->members.size();
    const size_t at = (size_t)pos * n + s->idx;
    const size_t plane = (size_t)g->block * n;
    for (uint32_t c = 0; c < g->ich; ++c) g->in[c * plane + at] = in[c];
    // this frame's output: frame pos of the previous block (zeros before the first block ran)
    if (blocks == 0) {
        for (uint32_t c = 0; c < g->och; ++c) out[c] = 0.f;
    } else {
        const float *o = g->out[(blocks - 1) & 1].data();
        for (uint32_t c = 0; c < g->och; ++c) out[c] = o[c * plane + at];
    }
    if (pos == 0) g->filling.store(true, std::memory_order_relaxed);   // once per instance per block
    s->pos.store(pos + 1, std::memory_order_relaxed);
    if (pos + 1 == g->block && g->complete.fetch_add(1, std::memory_order_acq_rel) + 1 == g->live.load()) {
        std::lock_guard<std::mutex> gl(g->mu);
        // re-checked under the lock: a concurrent destroy may have run the block already
        if (g->complete.load() == g->live.load() && g->blocks.load() == blocks) return run_block(g);
    }
    return OLFX_OK;
}

uint32_t olfx_sample_latency(const olfx_sample *s) { return s ? s->g->block : 0; }
uint32_t olfx_sample_generation_size(const olfx_sample *s) { return s ? (uint32_t)s->g->members.size() : 0; }
uint32_t olfx_sample_index(const olfx_sample *s) { return s ? s->idx : 0; }

}  // extern "C"
