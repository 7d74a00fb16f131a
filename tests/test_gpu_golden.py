"""GPU against the committed golden fixtures (tests/golden/*.json) directly —
not through the oracle — so a GPU/oracle drift and an oracle change both show.
PARITY UNPINNED vs ISA-L itself: see tests/golden/make_golden.py."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

from tests.golden.make_golden import seed_of

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def digest(a):
    b = np.ascontiguousarray(a, np.uint8).tobytes()
    return b.hex() if len(b) <= 64 else "sha256:" + hashlib.sha256(b).hexdigest()


def _splitmix(seed, n):
    from oracle import ec_oracle  # input generator only (splitmix64 bytes)
    return ec_oracle.splitmix_bytes(seed, n)


def test_golden_encode_on_gpu(dev):
    from elect_amd.batch import encode_batch
    from elect_amd.coder import RSCoder
    g = load("encode.json")
    for c in g["cases"]:
        k, m, L = c["k"], c["m"], c["L"]
        coder = RSCoder(k, m)
        assert coder.encode_matrix().tobytes().hex() == g["matrices"][f"{k},{m}"]
        data = np.stack([_splitmix(s, L) for s in c["seeds"]])[None]
        par = torch.zeros((1, m, L), dtype=torch.uint8, device=dev)
        encode_batch(coder, torch.from_numpy(data).to(dev), par)
        got = par.cpu().numpy()[0]
        assert [digest(p) for p in got] == c["parity"], (k, m, L)


def test_golden_decode_on_gpu(dev):
    """Every decode fixture with bytes, incl. singular survivor sets: compat mode
    codes them with the partially reduced inverse exactly as libec.so does
    (EC/erasure_coder.c:257-258 ignores gf_invert_matrix's -1) and reports
    ELECT_EC_WARN_SINGULAR; strict mode refuses them with ESINGULAR."""
    from elect_amd import _lib
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    g = load("decode.json")
    ran_singular = 0
    for c in g["cases"]:
        k, m, L = c["k"], c["m"], c["L"]
        if L == 0:
            continue
        coder = RSCoder(k, m)
        tag = c.get("input_tag", "elect" if "input_seeds" in c else "dec")
        st = torch.zeros((1, k + m, L), dtype=torch.uint8, device=dev)
        st[0, :k] = torch.from_numpy(np.stack([_splitmix(seed_of(tag, k, L, j), L) for j in range(k)])).to(dev)
        encode_batch(coder, st[:, :k], st[:, k:])
        out = torch.full((1, len(c["erased"]), L), 0x5A, dtype=torch.uint8, device=dev)
        mode = 1 if c["mode"] == "strict" else 0
        if c.get("singular") and mode == 1:
            with pytest.raises(_lib.ECSingularError):
                decode_batch(coder, st, c["decode_indexes"], c["erased"], out, mode=mode, inputs_by_unit=True)
            continue
        st_code = decode_batch(coder, st, c["decode_indexes"], c["erased"], out, mode=mode, inputs_by_unit=True)
        assert st_code == (_lib.WARN_SINGULAR if c["status"] == -1 else c["status"])
        assert [digest(x) for x in out.cpu().numpy()[0]] == c["outputs"], c
        ran_singular += bool(c.get("singular"))
    assert ran_singular >= 12


def test_golden_singular_decode_host_path(dev):
    """The same singular compat fixtures through the host-memory path (the JNI
    decodeImpl convention), where libec.so's callers meet them."""
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    g = load("decode.json")
    n = 0
    for c in g["cases"]:
        if not c.get("singular") or c["mode"] != "compat":
            continue
        k, m, L = c["k"], c["m"], c["L"]
        data = [_splitmix(seed_of("sing", k, L, j), L) for j in range(k)]
        coder = RSCoder(k, m)
        par = [np.empty(L, np.uint8) for _ in range(m)]
        coder.encode_host([d.ctypes.data for d in data], [p.ctypes.data for p in par], L)
        units = data + par
        outs = [np.full(L, 0x5A, np.uint8) for _ in c["erased"]]
        st = coder.decode_host([units[i].ctypes.data for i in c["decode_indexes"]], c["decode_indexes"],
                               c["erased"], [o.ctypes.data for o in outs], L)
        assert st == _lib.WARN_SINGULAR
        assert [digest(x) for x in outs] == c["outputs"], c
        n += 1
    assert n >= 12


def test_golden_update_on_gpu(dev):
    from elect_amd.batch import encode_update_batch
    from elect_amd.coder import RSCoder
    g = load("update.json")
    for c in g["cases"]:
        k, m, L, t = c["k"], c["m"], c["L"], c["target"]
        coder = RSCoder(k, m)
        old = torch.from_numpy(_splitmix(seed_of("upd-old", k, L, t), L)[None]).to(dev)
        new = torch.from_numpy(_splitmix(seed_of("upd-new", k, L, t), L)[None]).to(dev)
        pin = torch.from_numpy(np.stack([_splitmix(seed_of("upd-par", k, L, t, r), L) for r in range(m)])[None]).to(dev)
        pout = torch.zeros_like(pin)
        encode_update_batch(coder, t, old, new, pin, pout)
        assert [digest(p) for p in pout.cpu().numpy()[0]] == c["parity_out"], (k, m, L, t)


def test_golden_erasure_code_test_port_on_gpu(dev):
    """ErasureCodeTest.java:31-173 through the Java-API mirror on the GPU host path."""
    from elect_amd.coder import ByteBuffer, ErasureCoderOptions, NativeRSDecoder, NativeRSEncoder
    from tests.golden.java_random import JavaRandom
    g = load("erasure_code_test.json")
    L, k, m = g["codeLength"], 4, 2
    rnd = JavaRandom(123)
    data, modified = [], []
    for _ in range(k):
        tmp = rnd.nextBytes(L)
        data.append(ByteBuffer.allocateDirect(L).put(tmp).rewind())
        modified.append(ByteBuffer.allocateDirect(L).put(tmp).rewind())
    modified[0] = ByteBuffer.allocateDirect(L).put(rnd.nextBytes(L)).rewind()
    parity = [ByteBuffer.allocateDirect(L) for _ in range(m)]
    second = [ByteBuffer.allocateDirect(L) for _ in range(m)]
    upd = [ByteBuffer.allocateDirect(L) for _ in range(m)]
    enc = NativeRSEncoder(ErasureCoderOptions(k, m))
    dec = NativeRSDecoder(ErasureCoderOptions(k, m))
    enc.encode(data, parity)
    enc.encode(modified, second)
    out1, out2 = [ByteBuffer.allocateDirect(L)], [ByteBuffer.allocateDirect(L)]
    dec.decode([parity[0]] + data[1:], [4, 1, 2, 3], [0], out1)
    dec.decode([second[0]] + modified[1:], [4, 1, 2, 3], [0], out2)
    enc.encodeUpdate([data[0], modified[0]] + parity, upd, 0)
    assert [digest(b.array()) for b in data] == g["data"]
    assert [digest(b.array()) for b in parity] == g["parity"]
    assert [digest(b.array()) for b in second] == g["second_parity"]
    assert [digest(b.array()) for b in upd] == g["update_parity"]
    assert out1[0].compareTo(data[0].rewind()) == 0          # :112
    assert out2[0].compareTo(modified[0].rewind()) == 0      # :119
    enc.release()
    dec.release()


def test_cpp_mirror_erasure_code_test_on_gpu(dev, tmp_path):
    """ErasureCodeTest.java through the C++ mirror (include/elect_ec.hpp) on the GPU."""
    import subprocess
    from tests.cpp_build import build
    r = subprocess.run([build(), "gpu", str(tmp_path)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    g = load("erasure_code_test.json")
    rd = lambda n: np.fromfile(tmp_path / n, dtype=np.uint8)  # noqa: E731
    assert [digest(rd(f"data{i}")) for i in range(4)] == g["data"]
    assert [digest(rd(f"parity{r}")) for r in range(2)] == g["parity"]
    assert [digest(rd(f"second{r}")) for r in range(2)] == g["second_parity"]
    assert [digest(rd(f"update{r}")) for r in range(2)] == g["update_parity"]


def test_jni_shim_erasure_code_test_on_gpu(dev, tmp_path):
    """ErasureCodeTest.java through the seven JNI entry points of the drop-in
    libec.so shim (fake JVM, buffers at non-zero positions), on the GPU."""
    import subprocess
    from tests.jni_build import build
    lib, drv = build()
    r = subprocess.run([drv, lib, "gpu", str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    g = load("erasure_code_test.json")
    rd = lambda n: np.fromfile(tmp_path / n, dtype=np.uint8)  # noqa: E731
    assert [digest(rd(f"data{i}")) for i in range(4)] == g["data"]
    assert [digest(rd(f"parity{r}")) for r in range(2)] == g["parity"]
    assert [digest(rd(f"second{r}")) for r in range(2)] == g["second_parity"]
    assert [digest(rd(f"update{r}")) for r in range(2)] == g["update_parity"]
