"""Zero-copy host-memory calls (host_path.cpp ZeroCopy, off by default since
round 5): a lone caller's own buffers are page-locked for the call
(hsa_amd_memory_lock) and the kernel reads and writes them over PCIe.  Every
host entry point that takes the path (encode, decode, update, the padded
encode / update / degraded-read steps, with NULL empty units and an in-place
update) against the CPU oracle, forced on (ELECT_EC_ZEROCOPY=2, so short units
take it too) and as the lone-caller policy (ELECT_EC_ZEROCOPY=1: units of 1 MiB
and up); a unit another party has registered keeps the library from locking
it, and the call must still be right (staged path).  Each mode
runs in its own process: the library reads ELECT_EC_ZEROCOPY once."""
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import ctypes, sys
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd.coder import RSCoder
from oracle import ec_oracle as orc

torch.cuda.init()
rng = np.random.default_rng(SEED)
k, m = 4, 2
c = RSCoder(k, m)
enc = orc.Encoder(k, m)
bad = []

def check(name, got, want):
    for i, (a, b) in enumerate(zip(got, want)):
        if not np.array_equal(a, b):
            bad.append(f"{name} unit {i}")

def zf(x, n):
    return np.concatenate([x[:n], np.zeros(len(x) - n, np.uint8)])

hip = ctypes.CDLL("libamdhip64.so.7")
hip.hipHostRegister.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [ctypes.c_void_p]
for L in LENGTHS:
    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    want = enc.encode(d)
    locked = []
    if PRELOCK:  # someone else holds data unit 1 locked: the library's registration must fail over
        assert hip.hipHostRegister(d[1].ctypes.data, L, 0) == 0
        locked.append(d[1])
    p = [np.zeros(L, np.uint8) for _ in range(m)]
    c.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    check(f"encode L={L}", p, want)
    out = [np.zeros(L, np.uint8) for _ in range(2)]
    c.decode_host([p[0].ctypes.data, d[1].ctypes.data, d[3].ctypes.data, p[1].ctypes.data], [4, 1, 3, 5], [0, 2],
                  [x.ctypes.data for x in out], L)
    check(f"decode L={L}", out, [d[0], d[2]])
    # padded encode: unit 2 empty (NULL), unit 0 short
    lens = [L // 3, L, 0, max(0, L - 7)]
    p2 = [np.full(L, 0xAB, np.uint8) for _ in range(m)]
    c.encode_ex_host([d[0].ctypes.data, d[1].ctypes.data, None, d[3].ctypes.data], [x.ctypes.data for x in p2], L,
                     data_lengths=lens)
    check(f"encode_ex L={L}", p2, enc.encode([zf(x, n) for x, n in zip(d, lens)]))
    # update in place (outputs alias the old parity inputs)
    new = rng.integers(0, 256, L, dtype=np.uint8)
    par = [x.copy() for x in p]
    c.encode_update_host([d[1].ctypes.data, new.ctypes.data] + [x.ctypes.data for x in par], 1,
                         [x.ctypes.data for x in par], L)
    check(f"update L={L}", par, enc.encode([d[0], new, d[2], d[3]]))
    # padded update into separate buffers
    on = [max(0, L - 100), L // 2]
    pu = [np.zeros(L, np.uint8) for _ in range(m)]
    c.encode_update_ex_host([d[1].ctypes.data, new.ctypes.data] + [x.ctypes.data for x in p], 1,
                            [x.ctypes.data for x in pu], L, old_new_lengths=on)
    check(f"update_ex L={L}", pu, enc.encode_update([zf(d[1], on[0]), zf(new, on[1])] + p, 1))
    # degraded read of a prefix, survivors zero padded
    pre = max(1, L - 33)
    ins = [d[1], d[2], d[3], p[0]]
    il = [L, L // 2, L, L]
    r = [np.zeros(pre, np.uint8)]
    c.decode_ex_host([x.ctypes.data for x in ins], [1, 2, 3, 4], [0], [r[0].ctypes.data], pre, input_lengths=il)
    wantd = orc.decode(k, m, [zf(x, n)[:pre] for x, n in zip(ins, il)], [1, 2, 3, 4], [0])[1]
    check(f"decode_ex L={L}", r, wantd)
    for x in locked:
        hip.hipHostUnregister(x.ctypes.data)
from elect_amd import _lib
import json
print("BAD" if bad else "OK", json.dumps(_lib.host_path_stats()))
"""


def _run(env_extra, lengths, prelock=False, seed=7):
    code = (SCRIPT.replace("ROOT", repr(ROOT)).replace("SEED", str(seed)).replace("LENGTHS", repr(lengths))
            .replace("PRELOCK", "True" if prelock else "False"))
    env = {k: v for k, v in os.environ.items() if k != "ELECT_EC_ZEROCOPY"}
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]
    import json
    return json.loads(r.stdout.strip().split(" ", 1)[1])


def test_zero_copy_forced_every_entry_point():
    # forced: short and unaligned units take the zero-copy path too
    st = _run({"ELECT_EC_ZEROCOPY": "2"}, [1, 15, 1007, 65536, 4404020])
    assert st["zero_copy"] == 5 * 6 and st["zero_copy_fallback"] == 0, st  # every call took the path


def test_zero_copy_lone_caller_policy():
    # ELECT_EC_ZEROCOPY=1: a lone caller's units of 1 MiB and up (ELECT's codeLength) go zero-copy
    st = _run({"ELECT_EC_ZEROCOPY": "1"}, [1 << 20, 4404020], seed=8)
    # decode_ex codes a prefix of L - 33 bytes: below 1 MiB at L = 1 MiB, so it is batched
    assert st["zero_copy"] == 11 and st["zero_copy_fallback"] == 0, st


def test_zero_copy_off_by_default():
    # round 5: the batched path (units locked per call, gather / scatter kernels) serves a lone caller
    # faster than zero-copy, so the default is off
    st = _run({}, [4404020], seed=12)
    assert st["zero_copy"] == 0 and st["registered"] + st["batched"] == 6, st


def test_zero_copy_falls_back_when_memory_is_already_locked():
    # the library's hipHostRegister fails on a range another party locked: staged path, same bytes
    st = _run({"ELECT_EC_ZEROCOPY": "2"}, [4404020, 2 << 20], prelock=True, seed=9)
    assert st["zero_copy_fallback"] >= 2 and st["batched"] + st["per_thread"] >= st["zero_copy_fallback"], st


def test_zero_copy_off():
    st = _run({"ELECT_EC_ZEROCOPY": "0"}, [4404020], seed=10)
    # batched: units locked for the call (the default) or staged
    assert st["zero_copy"] == 0 and st["zero_copy_fallback"] == 0 and st["batched"] + st["registered"] == 6, st


PAGE_EDGE = r"""
import json, mmap, sys
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd import _lib
from elect_amd.coder import RSCoder
from oracle import ec_oracle as orc

torch.cuda.init()
k, m, L, P = 4, 2, 65536, mmap.PAGESIZE
rng = np.random.default_rng(11)
maps = []

def unit_at_plus8():
    # an L-byte unit 8 bytes into its own page-aligned mapping (JNI inputOffsets do this)
    mm = mmap.mmap(-1, L + 2 * P)
    maps.append(mm)
    a = np.frombuffer(mm, dtype=np.uint8)[8:8 + L]
    a[:] = rng.integers(0, 256, L, dtype=np.uint8)
    return a

def zf(x, n):
    return np.concatenate([x[:n], np.zeros(len(x) - n, np.uint8)])

d = [unit_at_plus8() for _ in range(k)]
# every content end lands exactly on a page boundary of its mapping: the segment that
# holds it reaches 8 bytes into the next page, which only the content-rounded
# registration covers
lens = [t * P - 8 for t in (2, 3, 5, 16)]
c = RSCoder(k, m)
p = [np.zeros(L, np.uint8) for _ in range(m)]
c.encode_ex_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L, data_lengths=lens)
want = orc.Encoder(k, m).encode([zf(x, n) for x, n in zip(d, lens)])
bad = [r for r in range(m) if not np.array_equal(p[r], want[r])]
ins = [d[1], d[2], d[3], unit_at_plus8()]
ins[3][:] = want[0]
il = [lens[1], lens[2], lens[3], L]
r = np.zeros(L, np.uint8)
c.decode_ex_host([x.ctypes.data for x in ins], [1, 2, 3, 4], [0], [r.ctypes.data], L, input_lengths=il)
wantd = orc.decode(k, m, [zf(x, n) for x, n in zip(ins, il)], [1, 2, 3, 4], [0])[1][0]
if not np.array_equal(r, wantd):
    bad.append("decode_ex")
print("BAD" if bad else "OK", json.dumps(_lib.host_path_stats()))
"""


def test_zero_copy_content_end_on_page_boundary():
    """A padded unit whose pointer is 8 bytes into a page and whose content ends
    exactly on a page boundary: the padded kernel loads the whole segment holding
    the content end (8 bytes past it), so the zero-copy registration must cover
    the content rounded up to 16 bytes (host_path.cpp ZeroCopy::input_span)."""
    code = PAGE_EDGE.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_ZEROCOPY="2")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]
    import json
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["zero_copy"] == 2 and st["zero_copy_fallback"] == 0, st


MIXED_POOL = r"""
import json, sys
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd import _lib
from elect_amd.coder import RSCoder
from oracle import ec_oracle as orc

torch.cuda.init()
rng = np.random.default_rng(21)
k, m, L = 4, 2, 4404020
c = RSCoder(k, m)
enc = orc.Encoder(k, m)
pool = [_lib.HostBuffer(L) for _ in range(2)]  # data unit 1 and parity unit 0 in page-locked pool blocks
bad = []
for it in range(3):
    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    pool[0].array[:] = d[1]
    d[1] = pool[0].array
    p = [pool[1].array, np.zeros(L, np.uint8)]
    p[0][:] = 0
    c.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    want = enc.encode(d)
    bad += [f"encode {it} parity {r}" for r in range(m) if not np.array_equal(p[r], want[r])]
    out = [np.zeros(L, np.uint8)]
    c.decode_host([p[0].ctypes.data, d[1].ctypes.data, d[2].ctypes.data, d[3].ctypes.data], [4, 1, 2, 3], [0],
                  [out[0].ctypes.data], L)
    if not np.array_equal(out[0], d[0]):
        bad.append(f"decode {it}")
# the pool blocks are still page-locked and move right through the batched path afterwards
if not all(_lib.host_pinned(b.addr, L) for b in pool):
    bad.append("pool block no longer pinned")
print("BAD " + "; ".join(bad) if bad else "OK", json.dumps(_lib.host_path_stats()))
"""


def test_zero_copy_pool_units_among_pageable_ones():
    """a zero-copy call whose units mix pool blocks and pageable memory must
    not lock (and later unlock) the pool's pages itself: the pool units are addressed through the
    pool's own device mapping, the pageable ones locked for the call.  No failed unlock, and the
    pool blocks stay locked and usable afterwards (the second and third rounds reuse them)."""
    code = MIXED_POOL.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_ZEROCOPY="2")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-2000:] + r.stderr[-2000:]
    import json
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["zero_copy"] == 6 and st["zero_copy_fallback"] == 0 and st["unregister_failures"] == 0, st
