"""Pipelined direct batches of the host path (round 6, host_path.cpp
Batcher::issue_direct): a batch's units are gathered, coded and scattered in
steps over windows of their bytes, a software pipeline of copy stages (gather
of window k+1 and scatter of window k-1 in one launch) and coding launches on
the batch's stream.

Every JNI entry point ELECT calls (encodeImpl, encodeExImpl with content
lengths and parity hashes, decodeImpl, encodeUpdateImpl in place) at ELECT's
codeLength 4,404,020 B and at ragged lengths around the 1 MiB floor of the
locked path, units at odd offsets (no unit page- or 16-byte aligned, so every
unit has partial end pages through the arena), pool units mixed among
pageable ones; a lone caller and concurrent callers; under step counts that put
window and piece boundaries in different places (1 step = round 5's unpipelined
batch, 3, 8, the default) and 16 / 64 KiB pieces.  Each output against the CPU oracle
(oracle/ec_oracle.c), each hash against the JDK's ByteBuffer.hashCode loop.
The step knobs are read once per process, so each configuration runs in a
process of its own."""
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
from elect_amd.coder import RSCoder, java_bytebuffer_hash
from oracle import ec_oracle as orc

torch.cuda.init()
k, m = 4, 2
LENGTHS = [4404020, (1 << 20) + 4099, 2 * (1 << 20) + 13]
errors = []
keep = []

def pool_array(n):
    hb = _lib.HostBuffer(n)
    keep.append(hb)
    return hb.array

def units(L, count, seed, odd, pool_at=()):
    # count units of L bytes at odd offsets inside one pageable block (neighbours share end pages);
    # the indices in pool_at come from the page-locked pool instead
    rng = np.random.default_rng(seed)
    block = np.zeros(count * (L + 21) + 64, np.uint8)
    keep.append(block)
    out = []
    for i in range(count):
        u = pool_array(L) if i in pool_at else block[odd + i * (L + 21):][:L]
        u[:] = rng.integers(0, 256, L, dtype=np.uint8)
        out.append(u)
    return out

def zf(x, n):
    return np.concatenate([x[:n], np.zeros(len(x) - n, np.uint8)])

def check_all(tag, L, seed, pool_at=()):
    a = lambda xs: [x.ctypes.data for x in xs]
    c, enc = RSCoder(k, m), orc.Encoder(k, m)
    u = units(L, k + m + 2, seed, 1 + seed % 7, pool_at)
    d, p, rb, new = u[:k], u[k:k + m], u[k + m], u[k + m + 1]
    c.encode_host(a(d), a(p), L)
    want = enc.encode([x.copy() for x in d])
    if not all(np.array_equal(x, y) for x, y in zip(p, want)):
        errors.append(f"{tag} L={L} encode")
    for e in range(k):  # every data shard rebuilt from the others and parity 0
        surv = [p[0]] + [d[j] for j in range(k) if j != e]
        idx = [k] + [j for j in range(k) if j != e]
        c.decode_host(a(surv), idx, [e], a([rb]), L)
        if not np.array_equal(rb, d[e]):
            errors.append(f"{tag} L={L} decode e={e}")
    c.encode_update_host(a([d[1], new] + p), 1, a(p), L)   # in place: outputs alias inputs
    if not all(np.array_equal(x, y) for x, y in zip(p, enc.encode([d[0], new, d[2], d[3]]))):
        errors.append(f"{tag} L={L} update")
    for lens in ([L // 3, L, L - 4097, L - 9], [0, 1, 65536 * 5 + 3, L - 1]):
        hs = c.encode_ex_host(a(d), a(p), L, data_lengths=lens, hashed=True)
        want2 = enc.encode([zf(x, n) for x, n in zip(d, lens)])
        if not all(np.array_equal(x, y) for x, y in zip(p, want2)):
            errors.append(f"{tag} L={L} encode_ex parity lens={lens}")
        if hs != [java_bytebuffer_hash(x) for x in want2]:
            errors.append(f"{tag} L={L} encode_ex hashes lens={lens}")

def run(tag, fn, threads):
    th = [threading.Thread(target=fn, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()

for L in LENGTHS:
    check_all("lone", L, 3)
    check_all("lone+pool", L, 4, pool_at=(1, 4))      # a pool data unit and a pool parity unit
def caller(t):
    try:
        for L in LENGTHS:
            check_all(f"t{t}", L, 10 + t, pool_at=(2,) if t % 2 else ())
    except Exception as e:
        errors.append(f"t{t}: {e!r}")
run("concurrent", caller, 4)
st = _lib.host_path_stats()
print("BAD " + "; ".join(errors[:6]) if errors else "OK", json.dumps(st))
"""

CONFIGS = {
    "default": {},
    "one_step": {"ELECT_EC_PIPELINE_STEPS": "1"},
    "three_steps": {"ELECT_EC_PIPELINE_STEPS": "3", "ELECT_EC_STEP_KB": "256"},
    "eight_steps_64k_pieces": {"ELECT_EC_PIPELINE_STEPS": "8", "ELECT_EC_STEP_KB": "256", "ELECT_EC_PIECE_KB": "64"},
    "eight_steps_16k_pieces": {"ELECT_EC_PIPELINE_STEPS": "8", "ELECT_EC_STEP_KB": "256", "ELECT_EC_PIECE_KB": "16"},
    "five_equal_windows_whole_table": {"ELECT_EC_PIPELINE_STEPS": "5", "ELECT_EC_TAPER": "0", "ELECT_EC_STAGE_WRITES": "0"},
    # round 5's scheduling: no early issue (no gate counter waits), coarse polls, the default timer slack
    "no_early_issue_coarse_polls": {"ELECT_EC_EARLY_ISSUE": "0", "ELECT_EC_POLL_FINE_US": "0",
                                    "ELECT_EC_TIMER_SLACK_NS": "0"},
    # early issue with a lead longer than a batch: every batch waits on the device for the previous one
    "early_issue_long_lead": {"ELECT_EC_EARLY_US": "5000"},
}


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_pipelined_direct_batches_match_oracle(name):
    code = SCRIPT.replace("ROOT", repr(ROOT))
    env = dict(os.environ, ELECT_EC_ZEROCOPY="0", ELECT_EC_REGISTER="1", **CONFIGS[name])
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0 and r.stdout.strip().startswith("OK"), r.stdout[-3000:] + r.stderr[-3000:]
    st = json.loads(r.stdout.strip().split(" ", 1)[1])
    assert st["unregister_failures"] == 0 and st["per_thread"] == 0, st
    # the locked (pipelined) path really ran: pageable callers' units locked for the call
    assert st["registered"] > 0, st
