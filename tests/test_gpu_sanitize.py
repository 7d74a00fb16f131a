"""The host code under AddressSanitizer + UndefinedBehaviorSanitizer, driven by
many threads (tools/sanitize/host_stress.cpp): every host entry point on one
coder with batching on and off, then the device API from threads on their own
streams, each result checked by an independent route.  The sanitizer build is
made by __graft_entry__.build() (elect_amd.build.build_sanitize, content-stamped)
and travels with the tree; if it is missing or was built from other sources,
this test builds it first (hipcc, host code instrumented only) instead of
skipping."""
import os
import subprocess

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def test_host_code_under_asan_ubsan_with_many_threads():
    from elect_amd import build
    if not build.sanitize_current():
        build.build_sanitize()
    assert build.sanitize_current()
    r = subprocess.run([os.path.join(ROOT, "tools", "sanitize", "run.sh"), "run", "16", "6", "1"],
                       capture_output=True, text=True, timeout=300)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-3000:]
    assert "device API: 16 threads x 6 iterations, failures so far 0" in out, out[-3000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-3000:]
