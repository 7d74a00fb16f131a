"""Direct batches (host_path.cpp, Batcher with direct = true): callers whose units
lie in elect_ec_host_alloc buffers (page-locked, pooled) are batched with no
staging copies: the dispatcher DMAs each unit straight from the caller's buffer
into the arena and each output straight back.  Every host entry point that ELECT
calls, single and concurrent callers, a mix of direct and staged callers, and a
call with one output outside the pool (staged), all against the CPU oracle."""
import threading

import numpy as np
import pytest

from elect_amd import _lib

pytestmark = pytest.mark.gpu

K, M = 4, 2


def _zf(x, n):
    return np.concatenate([x[:n], np.zeros(len(x) - n, np.uint8)])


def _pinned(n, fill=None, keep=None):
    hb = _lib.HostBuffer(n)
    assert _lib.host_pinned(hb.addr, n), ("elect_ec_host_alloc on a GPU box must be page-locked",
                                          hex(hb.addr), n, _lib.host_pinned(hb.addr, 1))
    if fill is not None:
        hb.array[:] = fill
    if keep is not None:
        keep.append(hb)
    return hb.array


def _delta(before):
    now = _lib.host_path_stats()
    return {k: now[k] - before[k] for k in now if isinstance(now[k], (int, float))}


@pytest.mark.parametrize("L", [4404020, 65536 + 3, 1 << 20, 1000])
def test_direct_entry_points_match_oracle(dev, oracle, L):
    from elect_amd.coder import RSCoder, java_bytebuffer_hash
    rng = np.random.default_rng(L)
    keep = []
    d = [_pinned(L, rng.integers(0, 256, L, dtype=np.uint8), keep) for _ in range(K)]
    c = RSCoder(K, M)
    enc = oracle.Encoder(K, M)
    st = _lib.host_path_stats()
    p = [_pinned(L, 0, keep) for _ in range(M)]
    c.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    want = enc.encode(list(d))
    assert all(np.array_equal(a, b) for a, b in zip(p, want))
    # ELECT's fused encode step: content lengths, parity hashCodes
    lens = [L // 3, L, 0, max(0, L - 9)]
    p2 = [_pinned(L, 0xAB, keep) for _ in range(M)]
    hs = c.encode_ex_host([d[0].ctypes.data, d[1].ctypes.data, None, d[3].ctypes.data], [x.ctypes.data for x in p2],
                          L, data_lengths=lens, hashed=True)
    want2 = enc.encode([_zf(x, n) for x, n in zip(d, lens)])
    assert all(np.array_equal(a, b) for a, b in zip(p2, want2))
    assert hs == [java_bytebuffer_hash(x) for x in want2]
    # parity update in place (outputs alias the old parity inputs)
    new = _pinned(L, rng.integers(0, 256, L, dtype=np.uint8), keep)
    par = [_pinned(L, x, keep) for x in p]
    c.encode_update_host([d[1].ctypes.data, new.ctypes.data] + [x.ctypes.data for x in par], 1,
                         [x.ctypes.data for x in par], L)
    assert all(np.array_equal(a, b) for a, b in zip(par, enc.encode([d[0], new, d[2], d[3]])))
    # degraded read: survivors zero padded
    ins = [d[1], d[2], d[3], p[0]]
    il = [L, L // 2, L, L]
    r = _pinned(L, 0, keep)
    c.decode_ex_host([x.ctypes.data for x in ins], [1, 2, 3, 4], [0], [r.ctypes.data], L, input_lengths=il)
    wantd = oracle.decode(K, M, [_zf(x, n) for x, n in zip(ins, il)], [1, 2, 3, 4], [0])[1][0]
    assert np.array_equal(r, wantd)
    dl = _delta(st)
    # every call in place on the pool buffers: batched by DMA (direct), or, for a lone
    # caller's unhashed calls of 1 MiB and up, read and written by the kernel over PCIe
    assert dl["direct"] + dl["zero_copy"] == 4 and dl["direct"] >= 1, dl
    assert dl["batched"] == 0 and dl["per_thread"] == 0 and dl["zero_copy_fallback"] == 0, dl
    for hb in keep:
        hb.close()


def test_direct_needs_every_unit_in_the_pool(dev, oracle):
    """One output in ordinary memory: the call is not a pool-direct call; it is
    coded with that output's interior pages locked for the call (or staged), and
    right."""
    from elect_amd.coder import RSCoder
    L = 4404020
    rng = np.random.default_rng(5)
    keep = []
    d = [_pinned(L, rng.integers(0, 256, L, dtype=np.uint8), keep) for _ in range(K)]
    p = [_pinned(L, 0, keep), np.zeros(L, np.uint8)]
    st = _lib.host_path_stats()
    RSCoder(K, M).encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    assert all(np.array_equal(a, b) for a, b in zip(p, oracle.Encoder(K, M).encode(list(d))))
    dl = _delta(st)
    assert dl["direct"] == 0 and dl["batched"] + dl["registered"] + dl["zero_copy"] + dl["per_thread"] == 1, dl
    for hb in keep:
        hb.close()


def test_direct_and_staged_callers_concurrently(dev, oracle):
    """16 callers at once, half on pool buffers (direct batches), half on ordinary
    memory (staged batches), pool buffers freed and re-allocated between calls:
    every caller's parity against the oracle."""
    from elect_amd.coder import RSCoder
    L, T, calls = 1 << 20, 16, 3
    enc = oracle.Encoder(K, M)
    errors = []
    st = _lib.host_path_stats()

    def worker(t):
        try:
            rng = np.random.default_rng(100 + t)
            c = RSCoder(K, M)
            for i in range(calls):
                keep = []
                if t % 2 == 0:
                    d = [_pinned(L, rng.integers(0, 256, L, dtype=np.uint8), keep) for _ in range(K)]
                    p = [_pinned(L, 0, keep) for _ in range(M)]
                else:
                    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(K)]
                    p = [np.zeros(L, np.uint8) for _ in range(M)]
                c.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
                if not all(np.array_equal(a, b) for a, b in zip(p, enc.encode(list(d)))):
                    errors.append(f"caller {t} call {i}")
                for hb in keep:
                    hb.close()
        except Exception as e:  # noqa: BLE001
            errors.append(f"caller {t}: {e!r}")

    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:4]
    dl = _delta(st)
    assert dl["direct"] + dl["zero_copy"] >= T // 2 * calls and dl["direct"] >= 1, dl
