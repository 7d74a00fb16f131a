"""The host path from a process without torch (tests/cpp/host_notorch.cpp): the
library on /opt/rocm's HIP / HSA runtime, as a JVM loads it (the
Python suite imports torch first, which binds the library to torch's bundled
runtime).  Every JNI method ELECT calls, at ELECT's codeLength, units at odd
offsets back to back (the locked + pipelined direct path with arena edges), a
lone caller then 4 concurrent ones; every output against the CPU oracle."""
import os
import subprocess

import numpy as np
import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

SRC = os.path.join(ROOT, "tests", "cpp", "host_notorch.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "host_notorch")


def build() -> str:
    lib_dir = os.path.join(ROOT, "elect_amd")
    deps = [SRC, os.path.join(ROOT, "include", "elect_ec.h"), os.path.join(lib_dir, "libelect_ec.so")]
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(os.path.getmtime(p) for p in deps):
        subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), SRC, "-L", lib_dir,
                        "-lelect_ec", f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/opt/rocm/lib", "-pthread", "-o", BIN],
                       check=True)
    return BIN


def test_host_path_without_torch_matches_oracle(tmp_path, oracle):
    T, L, k, m = 4, 4404020, 4, 2
    env = dict(os.environ, ELECT_EC_ZEROCOPY="0")
    env.pop("LD_LIBRARY_PATH", None)  # /opt/rocm's runtime, through the library's own links
    r = subprocess.run([build(), str(tmp_path), str(T), str(L)], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    stats = [int(x) for x in (tmp_path / "stats.txt").read_text().split()]
    assert stats[3] == 0 and stats[7] == 0, stats  # no per-thread engine fallback, no failed unlock
    assert stats[5] >= 4 * (T + 1), stats            # the locked direct (pipelined) path served the calls
    enc = oracle.Encoder(k, m)
    rd = lambda t, n: np.fromfile(tmp_path / f"t{t}_{n}", dtype=np.uint8)  # noqa: E731
    for t in range(T + 1):
        data = [rd(t, f"data{j}") for j in range(k)]
        want = enc.encode(data)
        assert all(np.array_equal(rd(t, f"parity{r}"), want[r]) for r in range(m)), t
        assert np.array_equal(rd(t, "rebuilt2"), data[2]), t
        lens = [L // 3, L, L - 4097, L - 9]
        want_ex = enc.encode([oracle.zero_fill(x[:n], L) for x, n in zip(data, lens)])
        assert all(np.array_equal(rd(t, f"parity_ex{r}"), want_ex[r]) for r in range(m)), t
        hashes = np.fromfile(tmp_path / f"t{t}_hashes_ex", dtype=np.int32).tolist()
        assert hashes == [oracle.java_hashcode(x) for x in want_ex], t
        want_upd = enc.encode([data[0], rd(t, "new"), data[2], data[3]])
        assert all(np.array_equal(rd(t, f"parity_upd{r}"), want_upd[r]) for r in range(m)), t
