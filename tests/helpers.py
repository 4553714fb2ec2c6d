"""Shared test helpers: seeded inputs, parameter draws, bit comparisons."""
from __future__ import annotations

import numpy as np

import oracle as O


def noise_block(n: int, frames: int, base: int = 0, ch: int = 2) -> np.ndarray:
    """[ch][frames][n] xorshift32 white noise, seeded per (instance, channel)."""
    x = np.empty((ch, frames, n), dtype=np.float32)
    for i in range(n):
        for c in range(ch):
            x[c, :, i] = O.xorshift_noise(O.instance_seed(base + i, c), frames)
    return x


def fast_noise(n: int, frames: int, seed: int = 0, ch: int = 2) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return (rng.random((ch, frames, n), dtype=np.float32) - 0.5).astype(np.float32)


def bits_equal(a: np.ndarray, b: np.ndarray) -> bool:
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def first_mismatch(a: np.ndarray, b: np.ndarray):
    d = np.argwhere(a.view(np.uint32) != b.view(np.uint32))
    return None if len(d) == 0 else (tuple(d[0]), float(a[tuple(d[0])]), float(b[tuple(d[0])]), len(d))


def rel_err(a: np.ndarray, ref: np.ndarray) -> float:
    """max |a - ref| / max(|ref|, rms(ref)) per instance (SURVEY 8c acceptance floor)."""
    a = a.astype(np.float64)
    ref = ref.astype(np.float64)
    rms = np.sqrt(np.mean(ref ** 2, axis=1, keepdims=True)) + 1e-30
    return float(np.max(np.abs(a - ref) / np.maximum(np.abs(ref), rms)))


def dt_params(rng: np.random.Generator, n: int, pre_delay: float) -> np.ndarray:
    p = np.empty((7, n), dtype=np.float32)
    p[0] = pre_delay
    p[1] = rng.uniform(0.5, 0.95, n)
    p[2] = rng.uniform(0.4, 0.8, n)
    p[3] = rng.uniform(0.4, 0.8, n)
    p[4] = rng.uniform(0.3, 0.8, n)
    p[5] = rng.uniform(0.25, 0.95, n)
    p[6] = rng.uniform(0.05, 0.95, n)
    return p


def chorus_params(rng: np.random.Generator, n: int) -> np.ndarray:
    p = np.empty((8, n), dtype=np.float32)
    p[0] = rng.uniform(0, 3, n)
    p[1] = rng.uniform(0, 1, n)
    p[2] = rng.uniform(0, 0.95, n)
    p[3] = rng.uniform(0, 1, n)
    p[4] = rng.uniform(0, 1, n)
    p[5] = rng.uniform(0.08, 1, n)
    p[6] = rng.uniform(0.01, 1, n)
    p[7] = rng.uniform(4, 10, n)
    return p


def voice_configs(rng: np.random.Generator, n: int) -> np.ndarray:
    p = np.empty((16, n), dtype=np.float32)
    p[0] = rng.uniform(100, 8000, n)
    p[1] = rng.uniform(0, 0.9, n)
    p[2] = rng.uniform(0, 1, n)
    p[3] = rng.uniform(0, 1, n)
    p[4] = rng.uniform(0.001, 0.5, n)
    p[5] = rng.uniform(0, 1, n)
    p[6] = rng.uniform(0.001, 0.5, n)
    p[7] = rng.uniform(0, 1, n)
    p[8] = rng.uniform(0.001, 0.5, n)
    p[9] = rng.uniform(0.2, 1, n)
    p[10] = rng.uniform(0.001, 0.5, n)
    p[11] = rng.uniform(0, 1, n)
    p[12] = rng.uniform(0.001, 0.5, n)
    p[13] = rng.uniform(0, 1, n)
    p[14] = rng.uniform(0.001, 0.5, n)
    p[15] = rng.uniform(0, 0.05, n)
    return p

def fxrack_params(rng: np.random.Generator, n: int) -> np.ndarray:
    """FxRack<2> member values (FR_FIELDS order), seeded; every 4th instance gets a delay shorter
    than a 16-frame chunk (time * 48000 in [0, 17)), the path that reads its own chunk's writes."""
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
