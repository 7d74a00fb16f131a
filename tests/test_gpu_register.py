"""Per-call registration of batched callers' pageable units (ELECT_EC_REGISTER=1,
host_path.cpp Registrar / RegisterPath), and the round-4 fault it once caused.

Round 4 page-locked each batched caller's page-ROUNDED ranges per call; units
that sit back to back share their end pages, the HIP runtime accepts the
overlapping registrations and the first unregister unmaps pages another call
still uses (profiles/r05/register_overlap.txt); the suite then faulted
(hipErrorIllegalAddress) at a later plain host-to-device copy
(profiles/r04/register_mode_fault.txt).  Here: 8 threads whose units are laid
back to back at odd offsets in ONE buffer, interleaved so that every unit's
first and last pages are shared with another thread's units; every host entry
point ELECT calls, inputs shared by all threads at once (identical
registrations), outputs aliasing inputs (in-place update); each result against
the CPU oracle.  Then, in the same process, device-only work of the kind that
faulted in round 4: fresh pageable arrays copied to the device (also the very
memory that was registered), coded there and checked.  No unregistration may
fail, and calls must really have taken the registered path."""
import json
import os
import subprocess
import sys

import pytest

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import json, sys, threading
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd import _lib
from elect_amd.batch import encode_batch
from elect_amd.coder import RSCoder, java_bytebuffer_hash
from oracle import ec_oracle as orc

torch.cuda.init()
dev = torch.device("cuda", 0)
k, m = 4, 2
L = (1 << 20) + 4099          # >= the register path's 1 MiB floor, ragged ends
T, CALLS, GAP = 8, 3, 7
per = k + m + 2               # data, parity, a rebuilt unit, a new-data unit
block = np.zeros(T * per * (L + GAP) + 2 * 4096, np.uint8)
units, off = {}, 1            # odd start: no unit is page or 16-byte aligned
for i in range(per):
    for t in range(T):        # thread-interleaved: a unit's neighbours belong to other threads
        units[(t, i)] = block[off:off + L]
        off += L + GAP
rng0 = np.random.default_rng(5)
shared = [rng0.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]  # inputs every thread codes at once
errors = []

def zf(x, n):
    return np.concatenate([x[:n], np.zeros(len(x) - n, np.uint8)])

def worker(t):
    try:
        rng = np.random.default_rng(100 + t)
        c, enc = RSCoder(k, m), orc.Encoder(k, m)
        d = [units[(t, j)] for j in range(k)]
        p = [units[(t, k + r)] for r in range(m)]
        rb, new = units[(t, k + m)], units[(t, k + m + 1)]
        a = lambda xs: [x.ctypes.data for x in xs]
        for i in range(CALLS):
            for x in d:
                x[:] = rng.integers(0, 256, L, dtype=np.uint8)
            c.encode_host(a(d), a(p), L)
            want = enc.encode([x.copy() for x in d])
            if not all(np.array_equal(x, y) for x, y in zip(p, want)):
                errors.append(f"t{t} c{i} encode")
            c.decode_host(a([p[0], d[1], d[2], d[3]]), [4, 1, 2, 3], [0], a([rb]), L)
            if not np.array_equal(rb, d[0]):
                errors.append(f"t{t} c{i} decode")
            new[:] = rng.integers(0, 256, L, dtype=np.uint8)
            c.encode_update_host(a([d[1], new] + p), 1, a(p), L)   # in place: outputs alias inputs
            if not all(np.array_equal(x, y) for x, y in zip(p, enc.encode([d[0], new, d[2], d[3]]))):
                errors.append(f"t{t} c{i} update")
            lens = [L // 3, L, L - 4097, L - 9]
            hs = c.encode_ex_host(a(d), a(p), L, data_lengths=lens, hashed=True)
            want2 = enc.encode([zf(x, n) for x, n in zip(d, lens)])
            if not all(np.array_equal(x, y) for x, y in zip(p, want2)) or hs != [java_bytebuffer_hash(x) for x in want2]:
                errors.append(f"t{t} c{i} encode_ex")
            c.encode_host(a(shared), a(p), L)   # every thread registers the same input units at once
            if not all(np.array_equal(x, y) for x, y in zip(p, enc.encode(shared))):
                errors.append(f"t{t} c{i} shared inputs")
    except Exception as e:
        errors.append(f"t{t}: {e!r}")

th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
for x in th:
    x.start()
for x in th:
    x.join()
stats = _lib.host_path_stats()

# device-only work in the same process, of the kind that faulted after round 4's
# register mode: fresh pageable arrays (and the registered block itself) to the device
enc = orc.Encoder(k, m)
c = RSCoder(k, m)
for rep in range(4):
    B, Lc = 64, 65536 + 16 * rep
    host = np.random.default_rng(rep).integers(0, 256, (B, k + m, Lc), dtype=np.uint8)
    st = torch.from_numpy(host).to(dev)
    encode_batch(c, st[:, :k], st[:, k:])
    got = st.cpu().numpy()
    for s in (0, B - 1):
        want = enc.encode([host[s, j] for j in range(k)])
        if not all(np.array_equal(got[s, k + r], want[r]) for r in range(m)):
            errors.append(f"device rep {rep} stripe {s}")
    del host, st
whole = torch.from_numpy(block).to(dev)
if not np.array_equal(whole.cpu().numpy(), block):
    errors.append("registered block round trip")
torch.cuda.synchronize()
print("BAD " + "; ".join(errors[:6]) if errors else "OK", json.dumps(stats))
"""


# Direct batches in one step (round 5's unpipelined batch) and pipelined over
# windows (round 6, Batcher::issue_direct; 256 KiB steps put four windows in
# each 1 MiB unit, so window edges fall inside the units' locked interiors).
@pytest.mark.parametrize("steps", ["1", "8"])
def test_registered_units_back_to_back_then_device_work(steps):
    code = SCRIPT.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_REGISTER="1", ELECT_EC_REGISTER_SLOTS="4", ELECT_EC_ZEROCOPY="0",
               ELECT_EC_PIPELINE_STEPS=steps, ELECT_EC_STEP_KB="256")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["unregister_failures"] == 0, st
    # every call was batched (registered, or staged when no slot was free), none fell to the per-thread engine
    # (a call meeting a shared lock that is being released at that moment is staged)
    assert st["registered"] >= 8 * 3 * 5 // 2 and st["per_thread"] == 0, st
    assert st["registered"] + st["batched"] == 8 * 3 * 5, st


OVERLAP = r"""
import json, sys, threading
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd import _lib
from elect_amd.coder import RSCoder
from oracle import ec_oracle as orc

torch.cuda.init()
k, m, L, P = 4, 2, (1 << 20) + 333, 4096
rng = np.random.default_rng(21)
block = rng.integers(0, 256, 2 * k * (L + 3 * P), dtype=np.uint8)
# caller A's data units and caller B's overlap them shifted by one page and a byte: every B interior
# shares pages with an A interior of another extent, so whichever locks second is refused (staged)
a_in = [block[1 + j * (L + 3 * P):][:L] for j in range(k)]
b_in = [block[1 + P + 1 + j * (L + 3 * P):][:L] for j in range(k)]
enc = orc.Encoder(k, m)
want = {"a": enc.encode([x.copy() for x in a_in]), "b": enc.encode([x.copy() for x in b_in])}
bad = []

def caller(name, ins):
    c = RSCoder(k, m)
    for it in range(12):
        out = [np.zeros(L, np.uint8) for _ in range(m)]
        c.encode_host([x.ctypes.data for x in ins], [x.ctypes.data for x in out], L)
        if not all(np.array_equal(o, w) for o, w in zip(out, want[name])):
            bad.append(f"{name} {it}")

th = [threading.Thread(target=caller, args=("a", a_in)), threading.Thread(target=caller, args=("b", b_in))]
for x in th:
    x.start()
for x in th:
    x.join()
print("BAD " + "; ".join(bad[:4]) if bad else "OK", json.dumps(_lib.host_path_stats()))
"""


def test_partially_overlapping_units_of_concurrent_callers():
    """Two callers whose input units overlap each other's pages at another extent
    (read-only, so both results are defined): the registry never lets the two
    locks coexist; the caller that meets the other's lock is staged, both right."""
    code = OVERLAP.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_REGISTER="1", ELECT_EC_ZEROCOPY="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["unregister_failures"] == 0 and st["per_thread"] == 0, st
    assert st["registered"] + st["batched"] == 24 and st["registered"] >= 1, st


REMAP = r"""
import ctypes, json, sys
import numpy as np
import torch
sys.path.insert(0, ROOT)
from elect_amd import _lib
from elect_amd.coder import RSCoder
from oracle import ec_oracle as orc

torch.cuda.init()
libc = ctypes.CDLL("libc.so.6", use_errno=True)
libc.mmap.restype = ctypes.c_void_p
libc.mmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_long]
libc.munmap.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
PROT_RW, MAP_PRIVATE, MAP_ANON, MAP_FIXED = 3, 0x02, 0x20, 0x10
k, m, L = 4, 2, (1 << 20) + 4099
size = (k + m + 1) * (L + 8192) + (1 << 20)
base = libc.mmap(None, size, PROT_RW, MAP_PRIVATE | MAP_ANON, -1, 0)
c, enc = RSCoder(k, m), orc.Encoder(k, m)
bad = []
for rnd in range(6):
    if rnd:  # new physical pages at the same virtual addresses (a free + malloc can do this)
        libc.munmap(base, size)
        got = libc.mmap(base, size, PROT_RW, MAP_PRIVATE | MAP_ANON | MAP_FIXED, -1, 0)
        assert got == base
    buf = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(base))
    shift = 1 + 1237 * rnd  # each round's units at another extent: locks overlap the last round's, shifted
    rng = np.random.default_rng(rnd)
    units = [buf[shift + i * (L + 8192):][:L] for i in range(k + m + 1)]
    for x in units[:k]:
        x[:] = rng.integers(0, 256, L, dtype=np.uint8)
    a = lambda xs: [x.ctypes.data for x in xs]
    c.encode_host(a(units[:k]), a(units[k:k + m]), L)
    want = enc.encode([x.copy() for x in units[:k]])
    if not all(np.array_equal(x, y) for x, y in zip(units[k:k + m], want)):
        bad.append(f"round {rnd} encode")
    c.decode_host(a([units[k]] + units[1:k]), [k, 1, 2, 3], [0], a([units[k + m]]), L)
    if not np.array_equal(units[k + m], units[0]):
        bad.append(f"round {rnd} decode")
    del buf, units, x
libc.munmap(base, size)
print("BAD " + "; ".join(bad) if bad else "OK", json.dumps(_lib.host_path_stats()))
"""


def test_relocks_after_the_pages_were_replaced():
    """The pattern the relock probe found unsafe for DMA (profiles/r06/relock_probe.txt:
    after a lock, an unlock and new physical pages at the same addresses, an SDMA
    copy through the new lock reads the OLD pages): units whose memory is replaced
    between calls (munmap + mmap at the same address, as free + malloc can do) and
    placed at a shifted extent each round, so every call's locks overlap the last
    round's.  The library moves locked memory only with kernels (the gather /
    scatter copy kernels), whose reads the probe shows right: every round's
    outputs against the oracle, and the locked path really taken."""
    code = REMAP.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_REGISTER="1", ELECT_EC_ZEROCOPY="0")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["unregister_failures"] == 0 and st["per_thread"] == 0 and st["registered"] >= 12, st
