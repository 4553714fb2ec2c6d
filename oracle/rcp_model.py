"""oracle/rcp_model.py -- the committed v_rcp_f32 model of gfx950 (TEST INFRASTRUCTURE: the
checker's data, never loaded by the product).

The voice oracle's kernel-arithmetic mode (oracle/voice_ref.c) needs what gfx950's v_rcp_f32
returns for every mantissa of [1, 2).  The instruction is within one ulp of the correctly rounded
1/x, so the table is stored as that difference, two bits per mantissa (0: exact, 1: +1 ulp, 2: -1
ulp), in tests/golden/rcp_f32_gfx950.npz with the sha256 of the full uint32 table (written once by
tools/rcp_dump.py on an MI355X).  The bit-exact voice tests install THIS table; the device under
test is only compared with it (tests/conftest.py rcp_table)."""
import hashlib
import os

import numpy as np

PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                    "rcp_f32_gfx950.npz")


def correctly_rounded() -> np.ndarray:
    """1/x correctly rounded (numpy float32 division) for x = 1 + m 2^-23, m = 0 .. 2^23 - 1."""
    x = ((np.uint32(127) << np.uint32(23)) | np.arange(1 << 23, dtype=np.uint32)).view(np.float32)
    return (np.float32(1.0) / x).view(np.uint32)


def encode(tab: np.ndarray) -> np.ndarray:
    d = tab.astype(np.int64) - correctly_rounded().astype(np.int64)
    if np.abs(d).max() > 1:
        raise ValueError("v_rcp_f32 outside one ulp of 1/x")
    code = np.where(d == 1, 1, np.where(d == -1, 2, 0)).astype(np.uint8)
    bits = np.stack([(code >> 1) & 1, code & 1], axis=1).reshape(-1)
    return np.packbits(bits)


def decode(packed: np.ndarray) -> np.ndarray:
    bits = np.unpackbits(packed)[: 2 << 23].reshape(-1, 2)
    code = (bits[:, 0] << 1) | bits[:, 1]
    d = np.where(code == 1, 1, np.where(code == 2, -1, 0)).astype(np.int64)
    return (correctly_rounded().astype(np.int64) + d).astype(np.uint32)


def load() -> np.ndarray:
    """The committed table, checked against its own committed sha256."""
    with np.load(PATH, allow_pickle=False) as z:
        tab = decode(z["packed"])
        sha = str(z["sha256"])
    if hashlib.sha256(tab.tobytes()).hexdigest() != sha:
        raise ValueError(f"{PATH}: table does not match its sha256")
    return tab
