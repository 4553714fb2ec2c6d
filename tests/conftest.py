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
    """gfx950's v_rcp_f32 over every mantissa of [1, 2), read from the device by the test helper
    tests/gpu_probe/librcp_probe.so, checked against the documented error model (within one ulp of
    the correctly rounded 1/x, never further) and installed as the voice oracle's v_rcp model
    (oracle/voice_ref.c "kernels' arithmetic").  Yields the table; the model is removed after."""
    import ctypes

    import numpy as np

    import oracle as O
    path = os.path.join(ROOT, "tests", "gpu_probe", "librcp_probe.so")
    if not os.path.exists(path):
        pytest.fail(f"{path} not built (make -C tests/gpu_probe)")
    L = ctypes.CDLL(path)
    L.probe_rcp_table.argtypes = [ctypes.c_void_p]
    tab = np.empty(1 << 23, np.uint32)
    assert L.probe_rcp_table(tab.ctypes.data) == 0
    x = ((np.uint32(127) << np.uint32(23)) | np.arange(1 << 23, dtype=np.uint32)).view(np.float32)
    cr = (np.float32(1.0) / x).view(np.uint32)            # numpy float32 division: correctly rounded
    d = tab.astype(np.int64) - cr.astype(np.int64)
    assert np.abs(d).max() <= 1, "v_rcp_f32 outside one ulp of 1/x"
    O.set_rcp_table(tab)
    yield tab
    O.set_rcp_table(None)
