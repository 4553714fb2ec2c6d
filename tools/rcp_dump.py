#!/usr/bin/env python3
"""tools/rcp_dump.py -- GPU box: read gfx950's v_rcp_f32 over every mantissa of [1, 2) (the voice
oracle's kernel-arithmetic model, oracle/voice_ref.c) through tests/gpu_probe/librcp_probe.so and
write it as the committed fixture tests/golden/rcp_f32_gfx950.npz: the instruction's result minus
the correctly rounded 1/x, in ulps (-1, 0 or +1), two bits per mantissa, plus the sha256 of the
full uint32 table.  The fixture is then the model the bit-exact voice tests use
(tests/conftest.py rcp_table; oracle/rcp_model.py), and the device under test is only checked against it.

Usage (repo root, on the GPU box):  python tools/rcp_dump.py gpurun_out/rcp_f32_gfx950.npz
"""
import ctypes
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main(dst: str) -> None:
    from rcp_model import encode, decode
    L = ctypes.CDLL(os.path.join(ROOT, "tests", "gpu_probe", "librcp_probe.so"))
    L.probe_rcp_table.argtypes = [ctypes.c_void_p]
    tab = np.empty(1 << 23, np.uint32)
    assert L.probe_rcp_table(tab.ctypes.data) == 0
    packed = encode(tab)
    assert np.array_equal(decode(packed), tab)
    sha = hashlib.sha256(tab.tobytes()).hexdigest()
    np.savez_compressed(dst, packed=packed, sha256=np.array(sha))
    nz = int(np.count_nonzero(np.unpackbits(packed).reshape(-1, 2).any(1)))
    print(f"{dst}: sha256 {sha}, {nz} of {1 << 23} mantissas off the correctly rounded 1/x "
          f"({100.0 * nz / (1 << 23):.2f} %), {os.path.getsize(dst)} bytes")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "rcp_f32_gfx950.npz"))
