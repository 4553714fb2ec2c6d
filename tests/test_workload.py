"""The synthetic workload of bench.py and the full-size GPU tests (ol_dsp_amd.workload): input
streams are the SURVEY 8d xorshift streams (checked against the oracle's KAT generator), and
parameters are pure functions of the global instance index, so shards compose to the whole job."""
import numpy as np
import torch

import oracle as O
from helpers import bits_equal
from ol_dsp_amd.dist import shard
from ol_dsp_amd.workload import RANGES, instance_params, noise_np, noise_torch, seeds, voice_notes


def test_noise_streams_match_the_oracle_generator():
    x = noise_np(1000, 6, 700)
    for i in range(6):
        for c in range(2):
            assert bits_equal(x[c, :, i], O.xorshift_noise(O.instance_seed(1000 + i, c), 700))
    assert seeds(5, 1, 2)[1, 0] == O.instance_seed(5, 1)


def test_noise_skip_and_torch_form():
    a = noise_np(7, 9, 600)
    assert bits_equal(noise_np(7, 9, 344, skip=256), a[:, 256:])
    t = torch.cat(noise_torch(7, 9, 200, 2, "cpu", blocks=3), 1).numpy()
    assert bits_equal(t, a[:, :600])


def test_params_are_functions_of_the_global_index():
    for kind in RANGES:
        whole = instance_params(kind, 0, 1000)
        for world in (2, 3, 8):
            parts = [instance_params(kind, *shard(1000, world, r)) for r in range(world)]
            assert bits_equal(np.concatenate(parts, 1), whole), kind
        assert whole.shape[0] == len(RANGES[kind])
    p = instance_params("chorus", 0, 20000)
    assert p[5].min() >= 0.08 and p[5].max() <= 1 and p[6].min() >= 0.01
    assert set(np.unique(instance_params("fxrack", 0, 5000)[9])) == {0, 1, 2, 3, 4}
    n = voice_notes(0, 1000)
    assert n.min() >= 36 and n.max() <= 96
