import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def _ensure_built():
    lib = os.path.join(ROOT, "ol_dsp_amd", "libolfx.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "ol_dsp_amd", "csrc")], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test requested but no GPU is visible")
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def rcp_table(cuda):
    """The voice oracle's v_rcp_f32 model (oracle/voice_ref.c "kernels' arithmetic"): the COMMITTED
    table tests/golden/rcp_f32_gfx950.npz (oracle/rcp_model.py: within one ulp of the correctly
    rounded 1/x, checked against its own committed sha256), installed for the bit-exact voice
    tests.  The device under test is only compared with it: its v_rcp_f32 over every mantissa of
    [1, 2), read by the test helper tests/gpu_probe/librcp_probe.so, must equal the committed model
    bit for bit, so a regression in the probe or the table handling cannot move oracle and kernel
    together.  Yields the table; the model is removed after."""
    import ctypes

    import numpy as np

    import oracle as O
    import rcp_model
    tab = rcp_model.load()
    path = os.path.join(ROOT, "tests", "gpu_probe", "librcp_probe.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} not built (make -C tests/gpu_probe)")
    L = ctypes.CDLL(path)
    L.probe_rcp_table.argtypes = [ctypes.c_void_p]
    dev = np.empty(1 << 23, np.uint32)
    assert L.probe_rcp_table(dev.ctypes.data) == 0
    bad = int(np.count_nonzero(dev != tab))
    assert bad == 0, f"v_rcp_f32 on this device differs from the committed model on {bad} mantissas"
    O.set_rcp_table(tab)
    yield tab
    O.set_rcp_table(None)
