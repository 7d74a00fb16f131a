"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer, driven by
many threads (tools/sanitize/host_stress.cpp): every host entry point on one
coder with batching on and off, then the device API from threads on their own
streams, each result checked by an independent route.  Needs the sanitizer
build (tools/sanitize/run.sh build, made in the build container; the binaries
travel with the tree); skipped when it is missing or older than the sources."""
import glob
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

BIN = os.path.join(ROOT, "tools", "sanitize", "out", "host_stress")
SOURCES = glob.glob(os.path.join(ROOT, "elect_amd", "csrc", "*.*")) + \
    [os.path.join(ROOT, "include", "elect_ec.h"), os.path.join(ROOT, "tools", "sanitize", "host_stress.cpp")]


def _fresh() -> bool:
    return os.path.exists(BIN) and os.path.getmtime(BIN) >= max(os.path.getmtime(s) for s in SOURCES)


@pytest.mark.skipif(not _fresh(), reason="sanitizer build missing or stale: tools/sanitize/run.sh build")
def test_host_code_under_asan_ubsan_with_many_threads():
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize", "run.sh"), "run", "16", "6", "1"],
                       capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "device API: 16 threads x 6 iterations, failures so far 0" in out, out[-3000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-3000:]
