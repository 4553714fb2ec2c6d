"""Synthetic workloads of SURVEY.md section 8d, as pure functions of the GLOBAL instance index.

bench.py and the tests draw every instance's parameters and input stream from its global index
(and a seed), never from the rank that happens to run it: an N-GPU run of `total` instances,
sharded by `dist.shard`, processes exactly the instances a one-GPU run of `total` would, with the
same parameters and the same inputs.

  instance_params(kind, first, count)  per-instance parameters, uniform within the section 8d
                                        ranges, from a counter-based hash of (seed, field, index)
  noise_np / noise_torch               input of instance i, channel c: xorshift32 seeded
                                        s0 = (0x9E3779B9 ^ ((2i+c+1) 0x85EBCA6B)) | 1, one step per
                                        frame, x = (float)(int32)s / 2^31 * 0.5 (the section 8c KAT
                                        step; oracle/dattorro_ref.c oracle_xorshift_noise)
"""
from __future__ import annotations

from typing import List

import numpy as np

M32 = 0xFFFFFFFF

# (lo, hi) per parameter field in C-ABI order (include/olfx.h); a float is a
# constant; "int5" draws an integer 0..4 (the rack's filter type)
RANGES = {
    "chorus": [(0, 3), (0, 1), (0, .95), (0, 1), (0, 1), (.08, 1), (.01, 1), 10.0],
    "pitchshift": [(0, 3), 10.0],
    # dattorro: pre-delay fixed 0.1 (uniform taps), diffusions at their defaults
    "dattorro": [0.1, (.5, .95), .75, .625, .70, (.25, .95), (.05, .95)],
    "voice": [(100, 8000), (0, .9), (0, 1), (0, 1), (.001, .5), (0, 1), (.001, .5), (0, 1), (.001, .5),
              (.2, 1), (.001, .5), (0, 1), (.001, .5), (0, 1), (.001, .5), (0, .05)],
    "fxrack": [(0.05, 1), (0, .9), (0, 1), (100, 12000), (0, .8), (0, 1), (100, 12000), (0, .8),
               (0, 1), "int5", (0, 1), 0.0],
}
RANGES["voice_moog"] = RANGES["voice"]
RANGES["chain"] = RANGES["chorus"] + RANGES["pitchshift"] + RANGES["dattorro"]
# random per-instance pre-delay in [0, 1] x 4800 samples (section 8d's gather-path variant)
RANGES["dattorro_rpd"] = [(0, 1)] + RANGES["dattorro"][1:]
RANGES["chain_rpd"] = RANGES["chorus"] + RANGES["pitchshift"] + RANGES["dattorro_rpd"]


def _splitmix64(z: np.ndarray) -> np.ndarray:
    z = (z + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(0xFFFFFFFFFFFFFFFF)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniform01(seed: int, field: int, first: int, count: int) -> np.ndarray:
    """[count] float64 in [0, 1): hash of (seed, field, global index first..first+count)."""
    idx = np.arange(first, first + count, dtype=np.uint64)
    key = idx ^ np.uint64(((seed & 0xFF) << 56) | ((field & 0xFF) << 48))
    with np.errstate(over="ignore"):
        z = _splitmix64(key)
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / (1 << 53))


def instance_params(kind: str, first: int, count: int, seed: int = 0) -> np.ndarray:
    """[n_fields][count] float32 parameters of global instances first..first+count."""
    rows = []
    for f, r in enumerate(RANGES[kind]):
        if isinstance(r, float):
            rows.append(np.full(count, r, np.float32))
        elif r == "int5":
            rows.append(np.floor(uniform01(seed, f, first, count) * 5).astype(np.float32))
        else:
            lo, hi = r
            rows.append((lo + (hi - lo) * uniform01(seed, f, first, count)).astype(np.float32))
    return np.stack(rows)


def voice_notes(first: int, count: int) -> np.ndarray:
    """MIDI note of each global voice, in [36, 96] (section 8d)."""
    return 36 + (np.arange(first, first + count, dtype=np.int64) * 7) % 61


def seeds(first: int, count: int, ch: int) -> np.ndarray:
    """[ch][count] uint32 xorshift seeds of (global instance, channel) (section 8d)."""
    i = np.arange(first, first + count, dtype=np.uint64)[None, :]
    c = np.arange(ch, dtype=np.uint64)[:, None]
    mul = ((np.uint64(2) * i + c + np.uint64(1)) * np.uint64(0x85EBCA6B)) & np.uint64(M32)
    return ((np.uint64(0x9E3779B9) ^ mul) | np.uint64(1)).astype(np.uint32)


def noise_np(first: int, count: int, frames: int, ch: int = 2, skip: int = 0) -> np.ndarray:
    """[ch][frames][count] float32: frames skip..skip+frames of each (instance, channel) stream."""
    s = seeds(first, count, ch).astype(np.uint32)
    out = np.empty((ch, frames, count), np.float32)
    for f in range(skip + frames):
        s ^= s << np.uint32(13)
        s ^= s >> np.uint32(17)
        s ^= s << np.uint32(5)
        if f >= skip:
            out[:, f - skip, :] = s.view(np.int32).astype(np.float32) * np.float32(2.0 ** -32)
    return out


def noise_torch(first: int, count: int, frames: int, ch: int, device, blocks: int = 1) -> List:
    """The same streams generated on the device, cut into `blocks` consecutive [ch][frames][count]
    tensors (block b holds frames b*frames .. (b+1)*frames of every stream).  The streams are
    stepped on the host (vectorised over instances) and each block is copied to the device once,
    untimed: a handful of copies instead of thousands of tiny device launches, so profiler runs
    see only the engine's kernels and a copy per block."""
    import torch
    s = seeds(first, count, ch).astype(np.uint32)
    out = []
    host = np.empty((ch, frames, count), np.float32)
    for _ in range(blocks):
        for f in range(frames):
            s ^= s << np.uint32(13)
            s ^= s >> np.uint32(17)
            s ^= s << np.uint32(5)
            host[:, f, :] = s.view(np.int32).astype(np.float32) * np.float32(2.0 ** -32)
        out.append(torch.from_numpy(host).to(device, copy=True))
    return out
