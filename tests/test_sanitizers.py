"""Sanitizer runs of the CPU-side code, on the CPU box:

  oracle/_san/san_check           every CPU restatement (oracle/) under ASan + UBSan: the Dattorro
                                  plate past its uint16 t wrap, chorus / pitch-shift in fp32 and
                                  double, both voice models through every event, the rack in all
                                  five topologies (oracle/san_check.c)
  tests/cpp/test_adapter_asan     the per-frame -> block adapter's host logic (include/olfx_adapter.hpp)
                                  under ASan + UBSan
  tests/cpp/test_adapter_tsan     the same under TSan, including Queue() from a second thread

Any sanitizer report aborts the binary (-fno-sanitize-recover=all) or is matched below.
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REPORTS = ("runtime error", "ERROR: AddressSanitizer", "ERROR: LeakSanitizer", "WARNING: ThreadSanitizer")


def _make(d, target):
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, d), target], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        pytest.fail(r.stdout + r.stderr)


def _run(path, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    r = subprocess.run([path], capture_output=True, text=True, timeout=600, env=env)
    out = r.stdout + r.stderr
    print(out[-2000:])
    assert r.returncode == 0, out[-4000:]
    for rep in REPORTS:
        assert rep not in out, out[-4000:]
    return out


def test_oracle_under_asan_ubsan():
    _make("oracle", "san")
    out = _run(os.path.join(ROOT, "oracle", "_san", "san_check"), {"ASAN_OPTIONS": "detect_leaks=1"})
    assert "san_check: ok" in out


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_adapter_under_sanitizers(kind):
    _make("tests/cpp", f"test_adapter_{kind}")
    out = _run(os.path.join(ROOT, "tests", "cpp", f"test_adapter_{kind}"),
               {"UBSAN_OPTIONS": "print_stacktrace=1", "TSAN_OPTIONS": "halt_on_error=1"})
    assert "4 tests, 0 failures" in out
