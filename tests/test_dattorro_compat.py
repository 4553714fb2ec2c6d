"""The reference's dattorro-verb API by name (include/olfx_dattorro.h): the verb.h:5-26
functions over the GPU engine, with one block of latency.

CPU: both linkages are exported (C, and the C++-mangled names the reference's own callers bind
to, checked against the symbols of the real reference built in oracle/_ref when it is present);
pool-config argument checks; without a GPU the first process call aborts loudly.
GPU: per-sample calls, frame-major over N instances, equal the oracle (bit-exact, pinned to the
reference) delayed by exactly one block; setters land at the next block boundary; deleting an
instance mid-block; instances created after the pool ran form a second generation; an instance
running a block ahead aborts.
"""
import ctypes
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle as O
import ol_dsp_amd as ofx
from ol_dsp_amd import _lib
from helpers import bits_equal, first_mismatch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SETTERS = ["setPreDelay", "setPreFilter", "setInputDiffusion1", "setInputDiffusion2", "setDecayDiffusion",
           "setDecay", "setDamping"]          # verb.h:10-16 order == OLFX_DT_* field order


def _mangled(name, args):
    return f"_Z{len(name)}{name}{args}"


MANGLED = {n: _mangled(n, a) for n, a in [
    ("DattorroVerb_create", "v"), ("DattorroVerb_delete", "P13sDattorroVerb"),
    ("DattorroVerb_process", "P13sDattorroVerbf"), ("DattorroVerb_getLeft", "P13sDattorroVerb"),
    ("DattorroVerb_getRight", "P13sDattorroVerb")] + [("DattorroVerb_" + s, "P13sDattorroVerbf") for s in SETTERS]}


def _exports(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return set(re.findall(r"\bT\s+(\S+)", out))


def test_both_linkages_exported():
    ex = _exports(_lib.LIB_PATH)
    for n in _lib.DATTORRO_SIGNATURES:
        assert n in ex, n
    for n, m in MANGLED.items():
        assert m in ex, (n, m)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (reference absent)")
def test_mangled_names_equal_the_reference_build():
    """Every DattorroVerb_* symbol the real verb.cpp exports (C++ linkage, as compiled against
    verb.h) is exported by libolfx.so under the identical mangled name: a link-level drop-in."""
    ref = {s for s in _exports(os.path.join(ROOT, "oracle", "_ref", "libverb_ref.so")) if "DattorroVerb_" in s}
    assert len(ref) == 12
    assert ref == set(MANGLED.values())
    assert ref <= _exports(_lib.LIB_PATH)


def test_pool_config_arguments():
    lib = ofx.load()
    assert lib.olfx_dattorro_pool_config(0, 250) == _lib.OLFX_E_ARG
    assert lib.olfx_dattorro_pool_config(0, 0) == _lib.OLFX_E_ARG
    assert lib.olfx_dattorro_pool_config(-1, 256) == _lib.OLFX_E_ARG
    assert lib.olfx_dattorro_pool_config(0, 256) == _lib.OLFX_OK
    assert lib.olfx_dattorro_latency(None) == 0


def _run_child(code):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    return subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True,
                          timeout=300, env=env, cwd=ROOT)


def _gpu_visible():
    return os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK)


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU path")
def test_without_gpu_process_aborts_loudly():
    r = _run_child("""
        import ol_dsp_amd as ofx
        lib = ofx.load()
        v = lib.DattorroVerb_create()
        assert v and lib.olfx_dattorro_generation_size(v) == 1
        lib.DattorroVerb_setDecay(v, 0.5)          # before the engine exists: host shadow only
        lib.DattorroVerb_process(v, 0.25)
        print("unreachable")
    """)
    assert r.returncode != 0 and "unreachable" not in r.stdout
    assert "olfx DattorroVerb: process: olfx_create" in r.stderr and "no HIP device" in r.stderr


# ---------------------------------------------------------------------------------------- GPU

def _fns(lib, mangled):
    """The 12 verb.h functions, by C name or by the reference's C++-mangled name."""
    out = {}
    for n, (res, args) in _lib.DATTORRO_SIGNATURES.items():
        f = getattr(lib, MANGLED[n] if mangled else n)
        f.restype, f.argtypes = res, args
        out[n[len("DattorroVerb_"):]] = f
    return out


def _oracle(n, params, x, changes=()):
    """Oracle output for mono input x [frames][n]; changes = [(frame, inst, field, value)] applied
    before that frame (frame multiple of the oracle's process split)."""
    ref = O.Dattorro(n)
    for i in range(n):
        for f in range(7):
            ref.set(i, f, float(params[f, i]))
    frames = x.shape[0]
    cuts = sorted({0, frames} | {c[0] for c in changes})
    ys = []
    for a, b in zip(cuts[:-1], cuts[1:]):
        for (fr, i, f, v) in changes:
            if fr == a:
                ref.set(i, f, v)
        seg = np.ascontiguousarray(np.stack([x[a:b], x[a:b]]))
        ys.append(ref.process(seg))
    ref.close()
    return np.concatenate(ys, axis=1)


def _draw_params(n, rng):
    p = np.empty((7, n), np.float32)
    p[0] = rng.uniform(0.0, 0.02, n)          # pre-delay up to 96 samples
    for f in range(1, 7):
        p[f] = rng.uniform(0.1, 0.9, n)
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("mangled", [False, True])
def test_per_sample_calls_equal_oracle_delayed_one_block(cuda, mangled):
    lib = ofx.load()
    F = _fns(lib, mangled)
    B, n, blocks = 256, 5, 6
    assert lib.olfx_dattorro_pool_config(0, B) == 0
    rng = np.random.default_rng(11 + mangled)
    p = _draw_params(n, rng)
    vs = [F["create"]() for _ in range(n)]
    assert all(vs) and lib.olfx_dattorro_generation_size(vs[0]) == n
    assert [lib.olfx_dattorro_index(v) for v in vs] == list(range(n))
    assert lib.olfx_dattorro_latency(vs[0]) == B
    for i, v in enumerate(vs):
        for f, s in enumerate(SETTERS):
            F[s](v, float(p[f, i]))
    x = (rng.random((B * blocks, n), dtype=np.float32) - 0.5).astype(np.float32)
    y = np.zeros((2, B * blocks, n), np.float32)
    for t in range(B * blocks):                # frame-major: the per-frame callback shape
        for i, v in enumerate(vs):
            F["process"](v, float(x[t, i]))
            y[0, t, i] = F["getLeft"](v)
            y[1, t, i] = F["getRight"](v)
    for v in vs:
        F["delete"](v)
    ref = _oracle(n, p, x)
    assert not np.any(y[:, :B])                # the first block: latency
    got, want = y[:, B:], ref[:, :B * (blocks - 1)]
    assert bits_equal(got, want), first_mismatch(got, want)
    assert np.any(want != 0)


@pytest.mark.gpu
def test_setter_lands_at_next_block_and_delete_mid_block(cuda):
    lib = ofx.load()
    F = _fns(lib, False)
    B, n, blocks = 256, 3, 6
    assert lib.olfx_dattorro_pool_config(0, B) == 0
    rng = np.random.default_rng(5)
    p = _draw_params(n, rng)
    vs = [F["create"]() for _ in range(n)]
    for i, v in enumerate(vs):
        for f, s in enumerate(SETTERS):
            F[s](v, float(p[f, i]))
    x = (rng.random((B * blocks, n), dtype=np.float32) - 0.5).astype(np.float32)
    y = np.zeros((2, B * blocks, n), np.float32)
    t_set, t_del = B + 7, 4 * B + 10          # a setter mid-block 1; delete instance 2 mid-block 4
    for t in range(B * blocks):
        if t == t_set:
            F["setDecay"](vs[1], 0.3)
            F["setDamping"](vs[0], 0.2)
        if t == t_del:
            F["delete"](vs[2])
            vs[2] = None
        for i, v in enumerate(vs):
            if v is None:
                continue
            F["process"](v, float(x[t, i]))
            y[0, t, i] = F["getLeft"](v)
            y[1, t, i] = F["getRight"](v)
    for v in vs:
        if v is not None:
            F["delete"](v)
    # the setters take effect at the start of block 2 (input frame 2B)
    ref = _oracle(n, p, x, changes=[(2 * B, 1, 5, 0.3), (2 * B, 0, 6, 0.2)])
    got, want = y[:, B:, :2], ref[:, :B * (blocks - 1), :2]
    assert bits_equal(got, want), first_mismatch(got, want)
    got2, want2 = y[:, B:t_del, 2], ref[:, :t_del - B, 2]   # instance 2 until its deletion
    assert bits_equal(got2, want2)
    assert np.any(ref[:, 2 * B:3 * B, :2] != 0)


@pytest.mark.gpu
def test_late_instances_form_a_second_generation(cuda):
    lib = ofx.load()
    F = _fns(lib, False)
    B = 256
    assert lib.olfx_dattorro_pool_config(0, B) == 0
    a = F["create"]()
    F["setPreDelay"](a, 0.0)
    F["process"](a, 1.0)                       # generation 1 runs with one instance
    b = F["create"]()
    F["setPreDelay"](b, 0.0)
    assert lib.olfx_dattorro_generation_size(a) == 1 and lib.olfx_dattorro_generation_size(b) == 1
    x = np.zeros((4 * B, 2), np.float32)
    x[0, :] = 1.0                              # impulses: a at its frame 0, b at its frame 0
    ya, yb = [], []
    for t in range(1, 4 * B):
        F["process"](a, float(x[t, 0]))
        ya.append(F["getLeft"](a))
    for t in range(4 * B):
        F["process"](b, float(x[t, 1]))
        yb.append(F["getLeft"](b))
    F["delete"](a)
    F["delete"](b)
    ref = _oracle(1, np.array([[0.0], [0.85], [0.75], [0.625], [0.7], [0.75], [0.95]], np.float32), x[:, :1])
    # independent generations: each instance alone equals the oracle (delayed one block)
    assert bits_equal(np.array(ya[B - 1:], np.float32), ref[0, :3 * B, 0])
    assert bits_equal(np.array(yb[B:], np.float32), ref[0, :3 * B, 0])
    assert np.any(ref[0, :3 * B, 0] != 0)


@pytest.mark.gpu
@pytest.mark.parametrize("depth,buf", [(2, 512), (1, 256), (4, 600)])
def test_instance_major_host_buffers(cuda, depth, buf):
    """a host that runs each reverb over its whole buffer in turn (instance-major,
    the per-plugin processBlock shape, modules/juce/host/host.cpp:682) -- 3 instances, `buf` frames
    each per cycle, 5 cycles -- with the pool depth D = ceil(buf / block): equals the oracle delayed
    by the documented latency D * block, bit for bit, with a setter landing at the instance's next
    block boundary.  (buf = 600 is not a multiple of the block: the lead reaches ceil(600 / 256) + 1 = 4.)"""
    lib = ofx.load()
    F = _fns(lib, False)
    B, n, cycles = 256, 3, 5
    assert lib.olfx_dattorro_pool_config_depth(0, B, depth) == 0
    rng = np.random.default_rng(40 + depth)
    p = _draw_params(n, rng)
    vs = [F["create"]() for _ in range(n)]
    assert lib.olfx_dattorro_latency(vs[0]) == depth * B
    for i, v in enumerate(vs):
        for f, s in enumerate(SETTERS):
            F[s](v, float(p[f, i]))
    T = buf * cycles
    x = (rng.random((T, n), dtype=np.float32) - 0.5).astype(np.float32)
    y = np.zeros((2, T, n), np.float32)
    t_set = 2 * buf                              # instance 1's setter before its third buffer
    for c in range(cycles):
        for i, v in enumerate(vs):
            if i == 1 and c * buf == t_set:
                F["setDecay"](v, 0.35)
            for t in range(c * buf, (c + 1) * buf):
                F["process"](v, float(x[t, i]))
                y[0, t, i] = F["getLeft"](v)
                y[1, t, i] = F["getRight"](v)
    for v in vs:
        F["delete"](v)
    assert lib.olfx_dattorro_pool_config(0, B) == 0
    L = depth * B
    land = -(-t_set // B) * B                    # the instance's next block boundary at or after it
    ref = _oracle(n, p, x, changes=[(land, 1, 5, 0.35)])
    assert not np.any(y[:, :L])
    got, want = y[:, L:], ref[:, :T - L]
    assert bits_equal(got, want), first_mismatch(got, want)
    assert np.any(want != 0)


@pytest.mark.gpu
def test_instance_running_a_block_ahead_aborts(cuda):
    r = _run_child("""
        import ol_dsp_amd as ofx
        lib = ofx.load()
        assert lib.olfx_dattorro_pool_config(0, 8) == 0
        a, b = lib.DattorroVerb_create(), lib.DattorroVerb_create()
        for t in range(9):                     # a runs ahead of b (instance-major order)
            lib.DattorroVerb_process(a, 0.5)
        print("unreachable")
    """)
    assert r.returncode != 0 and "unreachable" not in r.stdout
    assert "started block 1 before the other 1 live instances" in r.stderr
    # depth 2: two blocks of run-ahead are taken, the third aborts
    r = _run_child("""
        import ol_dsp_amd as ofx
        lib = ofx.load()
        assert lib.olfx_dattorro_pool_config_depth(0, 8, 2) == 0
        a, b = lib.DattorroVerb_create(), lib.DattorroVerb_create()
        for t in range(16):
            lib.DattorroVerb_process(a, 0.5)
        print("sixteen taken", flush=True)
        lib.DattorroVerb_process(a, 0.5)
        print("unreachable")
    """)
    assert r.returncode != 0 and "sixteen taken" in r.stdout and "unreachable" not in r.stdout
    assert "started block 2 before the other 1 live instances" in r.stderr
