#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run in the dev container only).

Dattorro fixtures are produced by the REAL reference reverb (libs/dattorro-verb/verb.cpp compiled
from /root/reference by oracle/Makefile into oracle/_ref/libverb_ref.so, -O2 -ffp-contract=off),
and cross-checked against the -O0 build (the reference's own CMake default: no build type).
Chorus / pitch-shift / voice fixtures freeze the build's own spec oracle (parity unpinned: no
reference implementation exists for them), so they pin the oracle against regressions only.

Inputs are never stored: they are regenerated from xorshift32 seeds.
Usage:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

IMPULSE_KAT_FRAMES = [0, 1, 479, 480, 481, 1000, 2000, 4800, 12800, 20800, 28800, 36800, 44800, 47999]

# Dattorro sweep groups: each group shares one pre-delay (the engine also takes per-instance ones).
DT_GROUPS = [
    {"pre_delay": 0.1, "n": 8, "frames": 4100, "seed": 1},
    {"pre_delay": 0.0, "n": 8, "frames": 2600, "seed": 2},
    {"pre_delay": 0.37, "n": 5, "frames": 3000, "seed": 3},
    {"pre_delay": 1.0, "n": 3, "frames": 9000, "seed": 4},
]


def noise_block(n: int, frames: int, base: int, ch: int = 2) -> np.ndarray:
    x = np.empty((ch, frames, n), dtype=np.float32)
    for i in range(n):
        for c in range(ch):
            x[c, :, i] = O.xorshift_noise(O.instance_seed(base + i, c), frames)
    return x


def dt_params(rng: np.random.Generator, n: int, pre_delay: float) -> np.ndarray:
    p = np.empty((7, n), dtype=np.float32)
    p[0] = pre_delay
    p[1] = rng.uniform(0.5, 0.95, n)      # pre_filter
    p[2] = rng.uniform(0.4, 0.8, n)       # input_diffusion1
    p[3] = rng.uniform(0.4, 0.8, n)       # input_diffusion2
    p[4] = rng.uniform(0.3, 0.8, n)       # decay_diffusion
    p[5] = rng.uniform(0.25, 0.95, n)     # decay
    p[6] = rng.uniform(0.05, 0.95, n)     # damping
    return p


def run_dt(bank, params: np.ndarray, x: np.ndarray) -> np.ndarray:
    for i in range(params.shape[1]):
        for f in range(7):
            bank.set(i, f, float(params[f, i]))
    return bank.process(x)


def chorus_params(rng: np.random.Generator, n: int) -> np.ndarray:
    p = np.empty((8, n), dtype=np.float32)
    p[0] = rng.uniform(0, 3, n)          # pitch Hz
    p[1] = rng.uniform(0, 1, n)          # mix
    p[2] = rng.uniform(0, 0.95, n)       # q
    p[3] = rng.uniform(0, 1, n)          # cutoff
    p[4] = rng.uniform(0, 1, n)          # phase
    p[5] = rng.uniform(0.08, 1, n)       # depth
    p[6] = rng.uniform(0.01, 1, n)       # rate
    p[7] = rng.uniform(4, 10, n)         # window ms
    return p


def voice_configs(rng: np.random.Generator, n: int) -> np.ndarray:
    p = np.empty((16, n), dtype=np.float32)
    p[0] = rng.uniform(100, 8000, n)     # filter_cutoff Hz
    p[1] = rng.uniform(0, 0.9, n)        # resonance
    p[2] = rng.uniform(0, 1, n)          # drive
    p[3] = rng.uniform(0, 1, n)          # filter env amount
    p[4] = rng.uniform(0.001, 0.5, n)    # filter attack
    p[5] = rng.uniform(0, 1, n)          # attack shape
    p[6] = rng.uniform(0.001, 0.5, n)    # decay
    p[7] = rng.uniform(0, 1, n)          # sustain
    p[8] = rng.uniform(0.001, 0.5, n)    # release
    p[9] = rng.uniform(0.2, 1, n)        # amp env amount
    p[10] = rng.uniform(0.001, 0.5, n)
    p[11] = rng.uniform(0, 1, n)
    p[12] = rng.uniform(0.001, 0.5, n)
    p[13] = rng.uniform(0, 1, n)
    p[14] = rng.uniform(0.001, 0.5, n)
    p[15] = rng.uniform(0, 0.05, n)      # portamento htime
    return p


def fxrack_params(rng: np.random.Generator, n: int) -> np.ndarray:
    """Same draw as tests/helpers.py: fxrack_params."""
    p = np.empty((11, n), dtype=np.float32)
    p[0] = rng.uniform(0, 1, n)
    p[0, ::4] = rng.uniform(0, 17, len(p[0, ::4])) / 48000
    p[1] = rng.uniform(0, 0.9, n)
    p[2] = rng.uniform(0, 1, n)
    p[3] = rng.uniform(100, 12000, n)
    p[4] = rng.uniform(0, 0.8, n)
    p[5] = rng.uniform(0, 1, n)
    p[6] = rng.uniform(100, 12000, n)
    p[7] = rng.uniform(0, 0.8, n)
    p[8] = rng.uniform(0, 1, n)
    p[9] = rng.integers(0, 5, n).astype(np.float32)
    p[10] = rng.uniform(0, 1, n)
    return p


def main() -> None:
    if not O.ref_available() or not O.ref_available(o0=True):
        O.build()
    gold: dict = {"generator": "tests/golden/gen_golden.py",
                  "dattorro_reference": "libs/dattorro-verb/verb.cpp via oracle/_ref (g++ -O2 -ffp-contract=off; -O0 cross-check)"}

    # ---- dattorro: impulse KAT (reference C API: mono in) ----
    imp = np.zeros((1, 48000, 1), np.float32)
    imp[0, 0, 0] = 1.0
    y = O.Dattorro(1, ref=True).process(imp)
    y0 = O.Dattorro(1, ref=True, o0=True).process(imp)
    assert np.array_equal(y.view(np.uint32), y0.view(np.uint32)), "-O0 and -O2 reference builds differ"
    gold["dattorro_impulse"] = {
        "frames": 48000,
        "kat": {str(n): [float(y[0, n, 0]), float(y[1, n, 0])] for n in IMPULSE_KAT_FRAMES},
        "fnv1a64": f"{O.fnv1a64_lr(y[0, :, 0], y[1, :, 0]):016x}",
    }
    np.save(os.path.join(HERE, "dattorro_impulse_4096.npy"), np.ascontiguousarray(y[:, :4096, 0]))

    # ---- dattorro: 10 s xorshift noise KAT ----
    x = O.xorshift_noise(12345, 480000)
    y = O.Dattorro(1, ref=True).process(x[None, :, None])
    gold["dattorro_noise_10s"] = {
        "seed": 12345, "frames": 480000,
        "fnv1a64": f"{O.fnv1a64_lr(y[0, :, 0], y[1, :, 0]):016x}",
        "sum_l2": float(np.sum(y[0, :, 0].astype(np.float64) ** 2)),
        "survey_sum_l2": 221499.833,
    }

    # ---- dattorro: parameter sweeps, stereo in (fxlib glue), several pre-delays ----
    groups = []
    base = 0
    for g in DT_GROUPS:
        rng = np.random.default_rng(1000 + g["seed"])
        p = dt_params(rng, g["n"], g["pre_delay"])
        xg = noise_block(g["n"], g["frames"], base)
        yr = run_dt(O.Dattorro(g["n"], ref=True), p, xg)
        yr0 = run_dt(O.Dattorro(g["n"], ref=True, o0=True), p, xg)
        assert np.array_equal(yr.view(np.uint32), yr0.view(np.uint32))
        groups.append({**g, "input_base": base, "params": p.tolist(),
                       "fnv1a64": [f"{O.fnv1a64_lr(yr[0, :, i], yr[1, :, i]):016x}" for i in range(g["n"])]})
        base += g["n"]
    gold["dattorro_sweep"] = groups

    # ---- chorus / pitch-shift / voice: frozen spec-oracle vectors (parity unpinned) ----
    rng = np.random.default_rng(77)
    n, frames = 6, 6000
    pc = chorus_params(rng, n)
    xc = noise_block(n, frames, 500)
    for mode, key in ((0, "chorus"), (1, "pitchshift")):
        ch = O.Chorus(n, 48000.0, mode)
        for i in range(n):
            for f in range(8):
                ch.set(i, f, float(pc[f, i]))
        yc = ch.process(xc)
        gold[key] = {"n": n, "frames": frames, "input_base": 500, "params": pc.tolist(),
                     "fnv1a64": [f"{O.fnv1a64_lr(yc[0, :, i], yc[1, :, i]):016x}" for i in range(n)]}

    nv, fv = 5, 9600
    pv = voice_configs(rng, nv)
    notes = [int(v) for v in rng.integers(36, 97, nv)]
    vo = O.Voice(nv)
    for i in range(nv):
        vo.config(i, pv[:, i])
        vo.note(i, True, notes[i])
    ya = vo.process(fv // 2)
    for i in range(nv):
        vo.note(i, False, notes[i])
    yb = vo.process(fv // 2)
    yv = np.concatenate([ya, yb], axis=1)
    gold["voice"] = {"n": nv, "frames": fv, "note_off_at": fv // 2, "notes": notes, "params": pv.tolist(),
                     "fnv1a64": [f"{O.fnv1a64_lr(yv[0, :, i], yv[0, :, i]):016x}" for i in range(nv)]}

    # ---- MoogFilter voice (daisysp::LadderFilter restated): frozen spec-oracle vectors ----
    rm = np.random.default_rng(97)
    nm, fm = 5, 4800
    pm = voice_configs(rm, nm)
    notes_m = [int(v) for v in rm.integers(36, 97, nm)]
    vm = O.Voice(nm, moog=True)
    for i in range(nm):
        vm.config(i, pm[:, i])
        vm.note(i, True, notes_m[i])
    ya = vm.process(fm // 2)
    for i in range(nm):
        vm.note(i, False, notes_m[i])
    ym = np.concatenate([ya, vm.process(fm // 2)], axis=1)
    gold["voice_moog"] = {"n": nm, "frames": fm, "note_off_at": fm // 2, "notes": notes_m, "params": pm.tolist(),
                          "fnv1a64": [f"{O.fnv1a64_lr(ym[0, :, i], ym[0, :, i]):016x}" for i in range(nm)]}

    # ---- fx rack (FxRack<2>): frozen spec-oracle vectors, past the echo and the 48000 wrap ----
    nr, fr = 6, 60000
    pr = fxrack_params(np.random.default_rng(91), nr)
    xr = noise_block(nr, fr, 900)
    rk = O.FxRack(nr)
    for i in range(nr):
        for f in range(pr.shape[0]):
            rk.set(i, f, float(pr[f, i]))
    yr = rk.process(xr)
    gold["fxrack"] = {"n": nr, "frames": fr, "input_base": 900, "params": pr.tolist(),
                      "fnv1a64": [f"{O.fnv1a64_lr(yr[0, :, i], yr[1, :, i]):016x}" for i in range(nr)]}

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(gold, f, indent=1)
    print("wrote", os.path.join(HERE, "golden.json"))


if __name__ == "__main__":
    main()
