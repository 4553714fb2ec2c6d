"""GPU parity at the BASELINE configs' full per-GPU sizes, on the bench's own synthetic workload
(ol_dsp_amd.workload: parameters hashed from the global instance index, SURVEY 8d xorshift input
streams), through the C-ABI.

At these sizes the oracle cannot run every instance, so each test checks size-independent
properties:
  * clones: odd instances copy instance 0's parameters and input stream, and must produce
    bit-identical output to it (every wave / workgroup / XCD position computes the same thing);
  * samples: instances spread over the grid (first, last, wave and workgroup edges) are checked
    against the oracle -- bit-exact for the reverb, chorus, pitch-shift, chain and rack; within
    the written voice tolerance for the voice;
  * shards: the job split into ranks' shards (dist.shard), each run by its own engine with
    parameters and inputs from the global index, reproduces the one-engine job bit for bit.
"""
import numpy as np
import pytest

import oracle as O
from helpers import bits_equal, first_mismatch, rel_err

pytestmark = pytest.mark.gpu

VOICE_TOL = 1e-5   # max |gpu - ref| / max(|ref|, rms(ref)) per voice (tests/test_gpu_parity.py)


def _engine(kind, n):
    import ol_dsp_amd as ofx
    return ofx.Engine(kind, n)


def _inputs(first, n, blocks, cuda, clone):
    import torch

    from ol_dsp_amd.workload import noise_torch
    xs = noise_torch(first, n, 256, 2, cuda, blocks=blocks)
    if clone:
        for x in xs:
            x[:, :, 1::2] = x[:, :, 0:1]
    torch.cuda.synchronize()
    return xs


def _params(kind, first, n, clone):
    from ol_dsp_amd.workload import instance_params
    p = instance_params(kind, first, n)
    if clone:
        p[:, 1::2] = p[:, 0:1]
    return p


def _run(e, xs):
    import torch
    y = torch.cat([e.process(x) for x in xs], 1)
    torch.cuda.synchronize()
    return y


def _sample_idx(n):
    idx = {0, 2, 62, 64, 126, 1024, n // 2, n // 2 + 64, n - 2, n - 64 if n > 128 else 4}
    return np.array(sorted(i for i in idx if i < n and i % 2 == 0), np.int64)


def _oracle(kind, p, idx, x):
    """The oracle of `kind` for the instances idx (params p[:, idx]) on input x [2][F][len(idx)]."""
    m = len(idx)
    if kind == "dattorro":
        d = O.Dattorro(m)
        for k, i in enumerate(idx):
            for f in range(7):
                d.set(k, f, float(p[f, i]))
        return d.process(x)
    if kind in ("chorus", "pitchshift"):
        c = O.Chorus(m, mode=0 if kind == "chorus" else 1)
        for k, i in enumerate(idx):
            for f in range(p.shape[0]):
                c.set(k, f if kind == "chorus" else (0, 7)[f], float(p[f, i]))
        return c.process(x)
    if kind == "fxrack":
        r = O.FxRack(m)
        for k, i in enumerate(idx):
            for f in range(p.shape[0]):
                r.set(k, f, float(p[f, i]))
        return r.process(x)
    assert kind == "chain"
    c1, c2, d = O.Chorus(m), O.Chorus(m, mode=1), O.Dattorro(m)
    for k, i in enumerate(idx):
        for f in range(8):
            c1.set(k, f, float(p[f, i]))
        c2.set(k, "pitch", float(p[8, i]))
        c2.set(k, "window", float(p[9, i]))
        for f in range(7):
            d.set(k, f, float(p[10 + f, i]))
    return d.process(c2.process(c1.process(x)))


def _check_clones(y, n):
    import torch
    assert torch.equal(y[:, :, 1::2], y[:, :, 0:1].expand(-1, -1, n // 2)), "cloned instances differ"


@pytest.mark.parametrize("kind,n", [("chain", 65536), ("chain", 16384), ("dattorro", 65536), ("chorus", 65536),
                                    ("pitchshift", 65536), ("fxrack", 65536)])
def test_full_size_stream_kinds(cuda, kind, n):
    """configs[1] chorus, configs[2] reverb, the north star's 65,536 chains, configs[4]'s 16,384-chain
    shard, the pitch-shifter and the fxlib rack at 65,536: clones bit-identical, samples bit-exact."""
    import torch
    p = _params(kind, 0, n, clone=True)
    xs = _inputs(0, n, 2, cuda, clone=True)
    e = _engine(kind, n)
    e.set_params(0, p)
    y = _run(e, xs)
    assert torch.isfinite(y).all()
    _check_clones(y, n)
    idx = _sample_idx(n)
    x = torch.cat(xs, 1)[:, :, idx].cpu().numpy()
    yr = _oracle(kind, p, idx, np.ascontiguousarray(x))
    yg = y[:, :, idx].cpu().numpy()
    assert bits_equal(yg, yr), first_mismatch(yg, yr)
    e.close()


@pytest.mark.parametrize("pset,kind", [("dattorro_rpd", "dattorro"), ("chain_rpd", "chain")])
def test_full_size_random_predelay(cuda, pset, kind):
    """The bench's dattorro_rpd / chain_rpd legs at 65,536: a random pre-delay per instance
    (verb.cpp:137-139), so the standalone reverb runs the split network over its pre-delay ring in
    rows (dattorro_block_v5) and the chain its pre-delay rows (dt::PreRow).  Two blocks; clones bit-identical,
    sampled instances (workgroup edges included) bit-exact against the oracle."""
    import torch
    n = 65536
    p = _params(pset, 0, n, clone=True)
    xs = _inputs(0, n, 2, cuda, clone=True)
    e = _engine(kind, n)
    e.set_params(0, p)
    y = _run(e, xs)
    if kind == "dattorro":
        assert e.kernel_name == "dattorro_block_v5"
    assert torch.isfinite(y).all()
    _check_clones(y, n)
    idx = np.union1d(_sample_idx(n), np.array([30, 32, 34, 96, 65502, 65534], np.int64))
    x = torch.cat(xs, 1)[:, :, idx].cpu().numpy()
    yr = _oracle(kind, p, idx, np.ascontiguousarray(x))
    yg = y[:, :, idx].cpu().numpy()
    assert bits_equal(yg, yr), first_mismatch(yg, yr)
    e.close()


def test_v5_large_ragged_long_run(cuda):
    """dattorro_block_v5 for per-instance pre-delays at the sizes where uniform ones run v4, with a
    partial last 64-instance group: n = CUs x 128 + 37 instances, pre-delays on row and window edges
    (0, 1, 15..17, 31..33, 4800, 8191) among random ones, 18 calls of 256 frames and, between them, of
    4 and 1,020 frames moving t0 off the 16-position rows.  Sampled instances, the partial group's
    included, bit-exact against the oracle."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 128 + 37
    rng = np.random.default_rng(606)
    from helpers import dt_params
    p = dt_params(rng, n, 0.0)
    edge = np.array([0, 1, 15, 16, 17, 31, 32, 33, 4800, 8191], np.float64) / 4800
    p[0, :] = rng.uniform(0, 1, n).astype(np.float32)
    p[0, -len(edge):] = edge.astype(np.float32)
    p[0, :len(edge)] = edge.astype(np.float32)
    e = _engine("dattorro", n)
    e.set_params(0, p)
    idx = np.unique(np.concatenate([np.arange(12), np.array([63, 64, 127, n // 2]), np.arange(n - 40, n)]))
    d = O.Dattorro(len(idx))
    for k, i in enumerate(idx):
        for f in range(7):
            d.set(k, f, float(p[f, i]))
    from ol_dsp_amd.workload import noise_torch
    ys, yrs = [], []
    for F in [256] * 10 + [4, 1020] + [256] * 6:
        x = torch.cat(noise_torch(len(ys) * 7, n, F, 2, cuda, blocks=1), 1)
        y = e.process(x)
        torch.cuda.synchronize()
        ys.append(y[:, :, idx].cpu().numpy())
        yrs.append(d.process(np.ascontiguousarray(x[:, :, idx].cpu().numpy())))
    assert e.kernel_name == "dattorro_block_v5"
    yg, yr = np.concatenate(ys, 1), np.concatenate(yrs, 1)
    assert bits_equal(yg, yr), first_mismatch(yg, yr)
    e.close()


def test_reverb_network_switches_at_full_size(cuda):
    """configs[2]'s 65,536 reverbs: uniform pre-delays run dattorro_block_v4 (pre-delay ring
    position-major), per-instance pre-delays dattorro_block_v5 (ring in rows); each switch converts
    the ring's content (dattorro_pre_layout).  Uniform -> per instance -> uniform, two blocks each,
    then one 2,048-frame call: sampled instances bit-exact against the oracle over the whole run."""
    import torch
    from ol_dsp_amd.workload import instance_params
    n = 65536
    p = instance_params("dattorro", 0, n)
    rpd = instance_params("dattorro_rpd", 0, n)[0]
    e = _engine("dattorro", n)
    e.set_params(0, p)
    idx = np.union1d(_sample_idx(n), np.array([1, 63, 65, 32767, 65535], np.int64))
    d = O.Dattorro(len(idx))
    for k, i in enumerate(idx):
        for f in range(7):
            d.set(k, f, float(p[f, i]))
    ys, yrs, kernels = [], [], []
    for phase, pd in enumerate([None, rpd, p[0], None]):
        if pd is not None:
            e.set_params("pre_delay", np.ascontiguousarray(pd[None, :]))
            for k, i in enumerate(idx):
                d.set(k, 0, float(pd[i]))
        xs = _inputs(1000 * phase, n, 2, cuda, clone=False) if phase < 3 else \
            [torch.cat(_inputs(3000, n, 8, cuda, clone=False), 1)]
        y = _run(e, xs)
        kernels.append(e.kernel_name)
        ys.append(y[:, :, idx].cpu().numpy())
        yrs.append(d.process(np.ascontiguousarray(torch.cat(xs, 1)[:, :, idx].cpu().numpy())))
    assert kernels == ["dattorro_block_v4", "dattorro_block_v5", "dattorro_block_v4", "dattorro_block_v4"]
    yg, yr = np.concatenate(ys, 1), np.concatenate(yrs, 1)
    assert bits_equal(yg, yr), first_mismatch(yg, yr)
    e.close()


def test_chain_persistent_groups_ragged(cuda):
    """chain_block_v5 runs one workgroup per CU over 64-instance groups back to back, its queues and
    counters running on across groups.  n = CUs x 64 x 2 + 37 instances: every workgroup runs two
    or three groups, the last one ragged (37 of 64); sampled instances in first, middle and last
    groups of several workgroups, over two blocks, bit-exact against the composed oracle."""
    import torch
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    n = cus * 64 * 2 + 37
    p = _params("chain", 0, n, clone=False)
    xs = _inputs(0, n, 2, cuda, clone=False)
    e = _engine("chain", n)
    e.set_params(0, p)
    y = _run(e, xs)
    assert torch.isfinite(y).all()
    idx = np.array(sorted({0, 63, 64, cus * 64 - 1, cus * 64, cus * 64 + 65, 2 * cus * 64 - 1,
                           2 * cus * 64, 2 * cus * 64 + 17, n - 1}), np.int64)
    x = torch.cat(xs, 1)[:, :, idx].cpu().numpy()
    yr = _oracle("chain", p, idx, np.ascontiguousarray(x))
    yg = y[:, :, idx].cpu().numpy()
    assert bits_equal(yg, yr), first_mismatch(yg, yr)
    e.close()


@pytest.mark.parametrize("kind", ["voice", "voice_moog"])
def test_full_size_voices(cuda, rcp_table, kind):
    """configs[3]'s per-GPU shard: 32,768 voices, NoteOn at block 0 and NoteOff at block 2 of 4 (SURVEY
    8d): clones bit-identical; sampled voices within the voice tolerance of the oracle, and
    bit-exact against its kernel-arithmetic mode (oracle/voice_ref.c)."""
    import torch

    from ol_dsp_amd.workload import voice_notes
    n = 32768
    p = _params(kind, 0, n, clone=True)
    notes = voice_notes(0, n)
    notes[1::2] = notes[0]
    e = _engine(kind, n)
    e.set_params(0, p)
    e.note_events(e.make_events(np.arange(n), 1, notes))
    out = torch.empty((1, 1024, n), device=cuda)
    for b in range(4):
        if b == 2:
            e.note_events(e.make_events(np.arange(n), 0, notes))
        ob = torch.empty((1, 256, n), device=cuda)
        e.process(None, out=ob)
        out[:, 256 * b:256 * (b + 1)] = ob
    torch.cuda.synchronize()
    _check_clones(out, n)
    idx = np.union1d(_sample_idx(n), np.array([64 * 97, 64 * 97 + 62, 64 * 311 + 30, 20000], np.int64))
    yg = out[:, :, idx].cpu().numpy()

    def oracle_run(kernel_arith):
        ref = O.Voice(len(idx), moog=kind == "voice_moog", kernel_arith=kernel_arith)
        for k, i in enumerate(idx):
            ref.config(k, p[:, i])
            ref.note(k, True, int(notes[i]))
        yr = ref.process(512)
        for k, i in enumerate(idx):
            ref.note(k, False, int(notes[i]))
        return np.concatenate([yr, ref.process(512)], 1)

    yk = oracle_run(True)
    fin = np.isfinite(yk)
    assert np.array_equal(fin, np.isfinite(yg)) and np.array_equal(yg[fin].view(np.uint32), yk[fin].view(np.uint32))
    yr = oracle_run(False)
    fin = np.isfinite(yr)
    assert np.array_equal(fin, np.isfinite(yg)), "non-finite pattern differs from the oracle"
    keep = fin.all(axis=(0, 1))
    assert keep.sum() >= len(idx) // 2
    assert rel_err(yg[0][:, keep].T, yr[0][:, keep].T) <= VOICE_TOL
    e.close()


@pytest.mark.parametrize("kind,n,world", [("chain", 4096, 3), ("dattorro", 4096, 2), ("chorus", 2048, 4),
                                          ("fxrack", 2048, 3)])
def test_shards_reproduce_the_single_engine_job(cuda, kind, n, world):
    """The multi-GPU layout on one GPU: the job of n global instances run as `world` shards (one
    engine per rank, params and input streams from the global index) equals the one-engine job."""
    import torch

    from ol_dsp_amd.dist import shard
    e = _engine(kind, n)
    e.set_params(0, _params(kind, 0, n, clone=False))
    y_all = _run(e, _inputs(0, n, 2, cuda, clone=False))
    e.close()
    parts = []
    for r in range(world):
        first, count = shard(n, world, r)
        es = _engine(kind, count)
        es.set_params(0, _params(kind, first, count, clone=False))
        parts.append(_run(es, _inputs(first, count, 2, cuda, clone=False)))
        es.close()
    y_sh = torch.cat(parts, 2)
    assert torch.equal(y_all.view(torch.int32), y_sh.view(torch.int32))


def test_voice_shards_reproduce_the_single_engine_job(cuda):
    import torch

    from ol_dsp_amd.dist import shard
    from ol_dsp_amd.workload import voice_notes
    n, world = 3000, 4

    def run(first, count):
        e = _engine("voice", count)
        e.set_params(0, _params("voice", first, count, clone=False))
        e.note_events(e.make_events(np.arange(count), 1, voice_notes(first, count)))
        y = torch.empty((1, 512, count), device=cuda)
        e.process(None, out=y)
        torch.cuda.synchronize()
        e.close()
        return y

    y_all = run(0, n)
    y_sh = torch.cat([run(*shard(n, world, r)) for r in range(world)], 2)
    assert torch.equal(y_all.view(torch.int32), y_sh.view(torch.int32))


def test_device_noise_pool_equals_the_seeded_streams(cuda):
    """bench.py's device-generated input pool is the SURVEY 8d xorshift stream of each (global
    instance, channel), bit for bit (the CPU form is checked against the oracle in test_workload)."""
    from ol_dsp_amd.workload import noise_np, noise_torch
    import torch
    xs = noise_torch(70000, 300, 256, 2, cuda, blocks=3)
    got = torch.cat(xs, 1).cpu().numpy()
    assert bits_equal(got, noise_np(70000, 300, 768, 2))
