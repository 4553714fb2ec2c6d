"""CPU tests of the C-ABI boundary: the library loads, exports exactly what include/olfx.h
declares, and host-side logic that needs no GPU behaves (kind info, error paths)."""
import ctypes
import os
import re
import subprocess

import pytest

import ol_dsp_amd as ofx
from ol_dsp_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "olfx.h")
C_HEADERS = [os.path.join(ROOT, "include", h) for h in ("olfx.h", "olfx_sample.h", "olfx_dattorro.h")]


def declared_functions(prefix="olfx_"):
    names = []
    for h in C_HEADERS:
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        names += re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(" + prefix + r"\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_the_abi():
    names = declared_functions()
    for must in ("olfx_create", "olfx_destroy", "olfx_set_params", "olfx_process", "olfx_note_events",
                 "olfx_last_error", "olfx_kind_info_get"):
        assert must in names
    assert len(names) >= 15


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = set(re.findall(r"\bT\s+(olfx_\w+)", out))
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    # every exported olfx_ symbol is declared (no undocumented ABI)
    assert exported == set(declared_functions())


def test_python_mirror_binds_every_symbol():
    assert set(_lib.SIGNATURES) == set(declared_functions())
    assert set(_lib.DATTORRO_SIGNATURES) == set(declared_functions("DattorroVerb_"))
    lib = ofx.load()
    for n in list(_lib.SIGNATURES) + list(_lib.DATTORRO_SIGNATURES):
        assert getattr(lib, n) is not None


def test_library_has_gfx950_code_object():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob
    for k in (b"dattorro_block", b"chorus_block", b"voice_block"):
        assert k in blob


def test_abi_version_and_kind_info():
    lib = ofx.load()
    assert lib.olfx_abi_version() == 2
    info = ofx.kind_info(ofx.KIND_DATTORRO)
    assert (info.n_params, info.in_channels, info.out_channels) == (7, 2, 2)
    # 42,368 ring floats + 3 recursive scalars + 7 coefficients per instance
    assert info.state_bytes_per_instance == (42368 + 3 + 8) * 4
    ch = ofx.kind_info(ofx.KIND_CHORUS, 48000.0)
    assert (ch.n_params, ch.in_channels, ch.out_channels) == (8, 2, 2)
    # rings + 8 state words (two 64-bit phasors, 4 biquad floats) + 17 coefficient words (spec v2:
    # D as a double, W in 32.32 fixed point)
    assert ch.state_bytes_per_instance == (2 * (512 + 2048) + 8 + 17) * 4
    vc = ofx.kind_info(ofx.KIND_VOICE)
    assert (vc.n_params, vc.in_channels, vc.out_channels) == (16, 0, 1)
    assert vc.state_bytes_per_instance == (8 + 19) * 4
    vm = ofx.kind_info(ofx.KIND_VOICE_MOOG)
    assert (vm.n_params, vm.in_channels, vm.out_channels) == (16, 0, 1)
    assert vm.state_bytes_per_instance == (8 + 9 + 19) * 4      # + LadderFilter z0_[4], z1_[4], oldinput_
    assert ofx.kind_info(ofx.KIND_CHAIN).n_params == 8 + 2 + 7
    fr = ofx.kind_info(ofx.KIND_FXRACK)
    assert fr.n_params == 12 and fr.in_channels == 2 and fr.out_channels == 2
    assert fr.state_bytes_per_instance == (48000 * 2 + 4 + 14) * 4   # rings, Svf states, coefficients
    with pytest.raises(ofx.OlfxError):
        ofx.kind_info(99)


def test_param_names_match_header():
    from ol_dsp_amd.engine import PARAMS
    src = open(HEADER).read()
    assert len(PARAMS[ofx.KIND_DATTORRO]) == 7 and "OLFX_DT_NPARAMS" in src
    assert len(PARAMS[ofx.KIND_VOICE]) == 16
    assert len(PARAMS[ofx.KIND_CHAIN]) == 17


def _torch_has_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_torch_has_gpu(), reason="checks the no-GPU error path")
def test_create_without_gpu_fails_loudly():
    lib = ofx.load()
    h = ctypes.c_void_p()
    rc = lib.olfx_create(ofx.KIND_DATTORRO, 0, 64, 48000.0, 256, ctypes.byref(h))
    assert rc == _lib.OLFX_E_NODEVICE
    assert not h.value
    assert b"no HIP device" in lib.olfx_last_error(None)
    with pytest.raises(ofx.OlfxError):
        ofx.Engine("dattorro", 64)


def test_bad_arguments_rejected_before_device_probe():
    lib = ofx.load()
    h = ctypes.c_void_p()
    assert lib.olfx_create(ofx.KIND_DATTORRO, 0, 0, 48000.0, 256, ctypes.byref(h)) == _lib.OLFX_E_ARG
    assert lib.olfx_create(ofx.KIND_DATTORRO, 0, 64, 48000.0, 250, ctypes.byref(h)) == _lib.OLFX_E_ARG
    assert lib.olfx_create(77, 0, 64, 48000.0, 256, ctypes.byref(h)) == _lib.OLFX_E_KIND
    assert lib.olfx_destroy(None) == _lib.OLFX_E_ARG
    assert lib.olfx_process(None, None, None, 256, 0, None) == _lib.OLFX_E_ARG


def test_product_does_not_link_the_oracle():
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out and "verb_ref" not in out
    syms = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in syms and "ref_verb" not in syms
    # libolfx.so exports the verb.h names (include/olfx_dattorro.h) but none of verb.cpp's
    # internals: the reference implementation is not inside the product
    for internal in ("DelayBuffer_", "AllPassFilter_", "LowPassFilter_", "_Z10initialize", "_Z5clampfff"):
        assert internal not in syms, internal
