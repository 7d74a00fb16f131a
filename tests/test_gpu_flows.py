"""GPU parity of ELECT's two coding-node steps, each fused into one pass.

- encode step, JEC/net/ECMessageVerbHandler.java:283-329: SSTable contents zero
  filled to codeLength, encode, parity hashCode() (names the parity blocks);
- parity-update step, JEC/net/ECParityUpdateVerbHandler.java:634-699: old and
  new SSTable contents zero filled to codeLength, encodeUpdate, new-parity
  hashCode().

Expected values come from the oracle alone: zero fill (oracle.zero_fill), the
L1 coder restatement (oracle.Encoder) and the JDK hashCode loop
(oracle.java_hashcode).  Bar: bit-exact bytes and equal int32 hashes.  The
buffers hold 0xFF garbage past every content length, which must not leak in.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _to(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


def _garbage_past(a, lens):
    """a[..., n:] = 0xFF past each length (last axis)."""
    out = a.copy()
    flat = out.reshape(-1, out.shape[-1])
    for i, n in enumerate(np.asarray(lens).reshape(-1)):
        flat[i, n:] = 0xFF
    return out


def _lengths(rng, B, n, L):
    lens = rng.integers(0, L + 1, size=(B, n)).astype(np.int32)
    lens[0, :] = L          # full units
    if B > 1:
        lens[1, :] = 0      # empty (ELECT's all-zero filler chunks)
    if B > 2:
        lens[2, :] = np.minimum(L, 16 * np.arange(1, n + 1) + 5)
    return lens


ENC_CASES = [(4, 2, 65536), (4, 2, 4099), (4, 2, 1), (4, 2, 1040), (8, 4, 2048), (3, 2, 4404020 // 64),
             (10, 4, 333), (4, 6, 16008), (6, 3, 65536 + 16)]


@pytest.mark.parametrize("k,m,L", ENC_CASES)
@pytest.mark.parametrize("padded,hashed", [(True, True), (True, False), (False, True)])
def test_encode_batch_ex(dev, oracle, k, m, L, padded, hashed):
    from elect_amd.batch import encode_batch_ex
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L + 7 * k + 3 * m)
    B = 5
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    lens = _lengths(rng, B, k, L) if padded else np.full((B, k), L, np.int32)
    par = torch.full((B, m, L), 0x5A, dtype=torch.uint8, device=dev)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev) if hashed else None
    encode_batch_ex(RSCoder(k, m), _to(dev, _garbage_past(data, lens) if padded else data), par,
                    lengths=_to(dev, lens) if padded else None, hashes=hashes)
    got = par.cpu().numpy()
    got_h = hashes.cpu().numpy() if hashed else None
    enc = oracle.Encoder(k, m)
    for s in range(B):
        want = enc.encode([oracle.zero_fill(data[s, j, :lens[s, j]], L) for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[s, r], want[r]), (s, r)
            if hashed:
                assert int(got_h[s, r]) == oracle.java_hashcode(want[r]), (s, r)


UPD_CASES = [(4, 2, 65536), (4, 2, 4099), (4, 2, 17), (8, 4, 1024), (6, 6, 2048), (2, 8, 333), (4, 2, 1040)]


@pytest.mark.parametrize("k,m,L", UPD_CASES)
@pytest.mark.parametrize("padded,hashed", [(True, True), (True, False), (False, True)])
@pytest.mark.parametrize("in_place", [False, True])
def test_encode_update_batch_ex(dev, oracle, k, m, L, padded, hashed, in_place):
    """m = 6, 8: two row groups, the second reading parity the first overwrote in place."""
    from elect_amd.batch import encode_update_batch_ex
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L * 5 + k + m)
    B = 4
    target = int(rng.integers(0, k))
    old = rng.integers(0, 256, (B, L), dtype=np.uint8)
    new = rng.integers(0, 256, (B, L), dtype=np.uint8)
    pin = rng.integers(0, 256, (B, m, L), dtype=np.uint8)
    lens = _lengths(rng, B, 2, L) if padded else np.full((B, 2), L, np.int32)
    d_old = _to(dev, _garbage_past(old, lens[:, 0]) if padded else old)
    d_new = _to(dev, _garbage_past(new, lens[:, 1]) if padded else new)
    d_pin = _to(dev, pin)
    d_pout = d_pin if in_place else torch.full((B, m, L), 0x77, dtype=torch.uint8, device=dev)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev) if hashed else None
    encode_update_batch_ex(RSCoder(k, m), target, d_old, d_new, d_pin, d_pout,
                           lengths=_to(dev, lens) if padded else None, hashes=hashes)
    got = d_pout.cpu().numpy()
    got_h = hashes.cpu().numpy() if hashed else None
    enc = oracle.Encoder(k, m)
    for s in range(B):
        ins = [oracle.zero_fill(old[s, :lens[s, 0]], L), oracle.zero_fill(new[s, :lens[s, 1]], L)]
        want = enc.encode_update(ins + [pin[s, r] for r in range(m)], target)
        for r in range(m):
            assert np.array_equal(got[s, r], want[r]), (s, r)
            if hashed:
                assert int(got_h[s, r]) == oracle.java_hashcode(want[r]), (s, r)


def test_tiled_update_needs_m_le_8(dev):
    """An update of an m >= 9 code is a 2 + m > 10 column product, wider than the
    padded vector kernels that tiled launches ride on: the tiled call refuses it,
    hashed or not, whether its units span one tile or several (up front, not in
    the launcher); the untiled hashed call runs (the byte-granular kernel,
    tests/test_gpu_parity.py::test_hashed_update_of_wide_codes)."""
    from elect_amd import _lib
    from elect_amd.batch import encode_update_batch_ex, encode_update_batch_tiled
    from elect_amd.coder import RSCoder
    B, L, m = 2, 64, 9
    z = torch.zeros((B, L), dtype=torch.uint8, device=dev)
    p = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
    h = torch.zeros((B, m), dtype=torch.int32, device=dev)
    for chunk in (L, 3 * L):  # T = 1 and T = 3 tiles per unit (B = 2 stripes -> 2 / 6 tile rows)
        T = chunk // L
        zt = torch.zeros((B * T, L), dtype=torch.uint8, device=dev)
        pt = torch.zeros((B * T, m, L), dtype=torch.uint8, device=dev)
        with pytest.raises(_lib.ECInvalidArgument):
            encode_update_batch_tiled(RSCoder(4, m), 0, zt, zt, pt, pt, chunk, hashes=h)
        with pytest.raises(_lib.ECInvalidArgument):
            encode_update_batch_tiled(RSCoder(4, m), 0, zt, zt, pt, pt, chunk)
    encode_update_batch_ex(RSCoder(4, m), 0, z, z, p, p, hashes=h)
    torch.cuda.synchronize()
    assert not p.any()  # all-zero units: zero parity, hash 31^L
    assert all(int(x) == _pow31(L) for x in h.view(-1).cpu())


def _pow31(n):
    v = pow(31, n, 1 << 32)
    return v - (1 << 32) if v >= 1 << 31 else v


def test_elect_flow_encode_then_update(dev, oracle):
    """ELECT's lifecycle on one batch of stripes: transition (padded + hashed encode),
    then compaction replaces SSTable `t` (padded + hashed update, in place).  The
    updated parity and its hashes must equal a fresh encode of the new contents."""
    from elect_amd.batch import encode_batch_ex, encode_update_batch_ex
    from elect_amd.coder import RSCoder
    k, m, B, L = 4, 2, 8, 65536 + 4  # codeLength = ceil(1.05 * size) is rarely a multiple of 16
    rng = np.random.default_rng(77)
    c = RSCoder(k, m)
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    lens = rng.integers(L // 2, L + 1, size=(B, k)).astype(np.int32)
    d_data = _to(dev, _garbage_past(data, lens))
    par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
    h0 = torch.empty((B, m), dtype=torch.int32, device=dev)
    encode_batch_ex(c, d_data, par, lengths=_to(dev, lens), hashes=h0)
    t = 2
    new = rng.integers(0, 256, (B, L), dtype=np.uint8)
    new_lens = rng.integers(0, L + 1, size=B).astype(np.int32)
    ul = np.stack([lens[:, t], new_lens], axis=1).astype(np.int32)
    h1 = torch.empty((B, m), dtype=torch.int32, device=dev)
    encode_update_batch_ex(c, t, d_data[:, t], _to(dev, _garbage_past(new, new_lens)), par, par,
                           lengths=_to(dev, ul), hashes=h1)
    lens2 = lens.copy()
    lens2[:, t] = new_lens
    data2 = data.copy()
    data2[:, t] = new
    ref = torch.empty_like(par)
    h2 = torch.empty_like(h1)
    encode_batch_ex(c, _to(dev, _garbage_past(data2, lens2)), ref, lengths=_to(dev, lens2), hashes=h2)
    torch.cuda.synchronize()
    assert torch.equal(par, ref)
    assert torch.equal(h1, h2)
    enc = oracle.Encoder(k, m)
    want = enc.encode([oracle.zero_fill(data2[0, j, :lens2[0, j]], L) for j in range(k)])
    assert int(h1[0, 1]) == oracle.java_hashcode(want[1])


def test_host_encode_ex(dev, oracle):
    """elect_ec_encode_ex: lengths across the 1 MiB pipeline step, NULL empty unit, hashes."""
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    L = (1 << 20) * 2 + 4404020 % 16 + 48
    rng = np.random.default_rng(41)
    lens = [L, (1 << 20) + 7, 0, 5]
    bufs = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    addrs = [b.ctypes.data if n else None for b, n in zip(bufs, lens)]
    par = [np.zeros(L, np.uint8) for _ in range(m)]
    hs = RSCoder(k, m).encode_ex_host(addrs, [p.ctypes.data for p in par], L, data_lengths=lens, hashed=True)
    want = oracle.Encoder(k, m).encode([oracle.zero_fill(b[:n], L) for b, n in zip(bufs, lens)])
    for r in range(m):
        assert np.array_equal(par[r], want[r])
        assert hs[r] == oracle.java_hashcode(want[r])


@pytest.mark.parametrize("L", [4404020, 4099, 1])
@pytest.mark.parametrize("in_place", [False, True])
def test_host_encode_update_ex(dev, oracle, L, in_place):
    """elect_ec_encode_update_ex, as ECParityUpdateVerbHandler calls it: the old and
    new SSTables shorter than codeLength, the new parity written over the old."""
    from elect_amd.coder import RSCoder
    k, m, t = 4, 2, 1
    rng = np.random.default_rng(L + in_place)
    old = rng.integers(0, 256, L, dtype=np.uint8)
    new = rng.integers(0, 256, L, dtype=np.uint8)
    pin = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(m)]
    pin_copy = [p.copy() for p in pin]
    lens = [max(0, L - 1000), L // 3]
    out = pin if in_place else [np.zeros(L, np.uint8) for _ in range(m)]
    hs = RSCoder(k, m).encode_update_ex_host([old.ctypes.data, new.ctypes.data] + [p.ctypes.data for p in pin], t,
                                             [o.ctypes.data for o in out], L, old_new_lengths=lens, hashed=True)
    want = oracle.Encoder(k, m).encode_update(
        [oracle.zero_fill(old[:lens[0]], L), oracle.zero_fill(new[:lens[1]], L)] + pin_copy, t)
    for r in range(m):
        assert np.array_equal(out[r], want[r])
        assert hs[r] == oracle.java_hashcode(want[r])


def test_host_update_ex_empty_old(dev, oracle):
    """A zero-length old SSTable may come as a NULL pointer."""
    from elect_amd.coder import RSCoder
    k, m, L, t = 4, 2, 5000, 3
    rng = np.random.default_rng(3)
    new = rng.integers(0, 256, L, dtype=np.uint8)
    pin = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(m)]
    out = [np.zeros(L, np.uint8) for _ in range(m)]
    RSCoder(k, m).encode_update_ex_host([None, new.ctypes.data] + [p.ctypes.data for p in pin], t,
                                        [o.ctypes.data for o in out], L, old_new_lengths=[0, L])
    want = oracle.Encoder(k, m).encode_update([np.zeros(L, np.uint8), new] + pin, t)
    for r in range(m):
        assert np.array_equal(out[r], want[r])


def test_cross_thread_batching_fused_steps(dev, oracle):
    """ELECT's coding threads issue the fused steps concurrently: padded / hashed /
    both / neither encodes and updates are distinct batch shapes, so batches close
    early and the arenas alternate; every caller must get its own parity and
    hashes.  Plain encodeUpdate batches too (as a product)."""
    import threading
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    errors = []
    _lib.set_batching(True, window_us=300, arena_bytes=8 << 20)
    try:
        def worker(t):
            try:
                L = 65536 + 4 if t % 2 else 4099
                padded, hashed = bool(t & 2), bool(t & 4)
                rng = np.random.default_rng(2000 + t)
                for it in range(3):
                    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
                    lens = [int(x) for x in rng.integers(0, L + 1, k)] if padded else None
                    p = [np.empty(L, np.uint8) for _ in range(m)]
                    hs = coder.encode_ex_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L,
                                              data_lengths=lens, hashed=hashed)
                    full = [oracle.zero_fill(x[:n], L) for x, n in zip(d, lens)] if padded else d
                    want = enc.encode(full)
                    if not all(np.array_equal(a, b) for a, b in zip(p, want)):
                        errors.append(f"t{t} it{it} encode")
                    if hashed and hs != [oracle.java_hashcode(w) for w in want]:
                        errors.append(f"t{t} it{it} encode hashes")
                    tgt = it % k
                    new = rng.integers(0, 256, L, dtype=np.uint8)
                    ul = [lens[tgt], int(rng.integers(0, L + 1))] if padded else None
                    ins = [d[tgt].ctypes.data, new.ctypes.data] + [x.ctypes.data for x in p]
                    if padded or hashed:
                        hs = coder.encode_update_ex_host(ins, tgt, [x.ctypes.data for x in p], L,
                                                         old_new_lengths=ul, hashed=hashed)
                    else:
                        coder.encode_update_host(ins, tgt, [x.ctypes.data for x in p], L)
                    full = list(full)
                    full[tgt] = oracle.zero_fill(new[:ul[1]], L) if padded else new
                    want = enc.encode(full)
                    if not all(np.array_equal(a, b) for a, b in zip(p, want)):
                        errors.append(f"t{t} it{it} update")
                    if hashed and hs != [oracle.java_hashcode(w) for w in want]:
                        errors.append(f"t{t} it{it} update hashes")
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    finally:
        _lib.set_batching(True)
    assert not errors, errors[:5]


DEC_CASES = [(4, 2, 65536), (4, 2, 4099), (4, 2, 1040), (8, 4, 2048), (3, 2, 17), (10, 4, 333)]


@pytest.mark.parametrize("k,m,L", DEC_CASES)
@pytest.mark.parametrize("n_erased", [1, 2])
def test_decode_batch_ex_padded_survivors(dev, oracle, k, m, L, n_erased):
    """ECRecovery's degraded read (:128-141): survivors copied into zero-filled codeLength
    buffers.  Data survivors hold their content lengths (0xFF garbage past them), parity
    survivors are full; strict and compat modes against the oracle's decode."""
    from elect_amd import _lib
    from elect_amd.batch import decode_batch_ex
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L + 11 * k + n_erased)
    B = 4
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    dlens = _lengths(rng, B, k, L)
    enc = oracle.Encoder(k, m)
    stripes = np.zeros((B, k + m, L), np.uint8)
    for s in range(B):
        full = [oracle.zero_fill(data[s, j, :dlens[s, j]], L) for j in range(k)]
        stripes[s, :k] = np.stack(full)
        stripes[s, k:] = np.stack(enc.encode(full))
    erased = list(range(n_erased))                       # data units lost
    surv = list(range(n_erased, k)) + list(range(k, k + n_erased))
    lens = np.array([[dlens[s, u] if u < k else L for u in surv] for s in range(B)], np.int32)
    stored = stripes.copy()
    for s in range(B):
        for u in range(k):
            stored[s, u, dlens[s, u]:] = 0xFF
    out = torch.full((B, n_erased, L), 0x44, dtype=torch.uint8, device=dev)
    for mode in (_lib.DECODE_COMPAT, _lib.DECODE_STRICT):
        decode_batch_ex(RSCoder(k, m), _to(dev, stored), surv, erased, out, lengths=_to(dev, lens), mode=mode,
                        inputs_by_unit=True)
        got = out.cpu().numpy()
        for s in range(B):
            for r, e in enumerate(erased):
                assert np.array_equal(got[s, r], stripes[s, e]), (mode, s, r)


def test_host_decode_ex_prefix(dev, oracle):
    """elect_ec_decode_ex as ECRecovery would call it: only the dataFileSize prefix of the
    rebuilt SSTable is decoded, from survivors shorter than codeLength (one empty, NULL)."""
    from elect_amd.coder import RSCoder
    k, m, L = 4, 2, 4404020
    rng = np.random.default_rng(12)
    lens = [L - 7, 3_000_001, 0, 4_404_000]
    data = [oracle.zero_fill(rng.integers(0, 256, n, dtype=np.uint8), L) for n in lens]
    par = oracle.Encoder(k, m).encode(data)
    raw = [d.copy() for d in data]
    for d, n in zip(raw, lens):
        d[n:] = 0xEE
    want_len = lens[1]
    out = np.full(L, 0x33, np.uint8)
    surv = [0, 2, 3, 4]  # unit 1 lost
    addrs = [raw[0].ctypes.data, None, raw[3].ctypes.data, par[0].ctypes.data]
    RSCoder(k, m).decode_ex_host(addrs, surv, [1], [out.ctypes.data], want_len,
                                 input_lengths=[lens[0], 0, lens[3], L])
    assert np.array_equal(out[:want_len], data[1][:want_len])
    assert (out[want_len:] == 0x33).all()


def test_device_lengths_above_chunk_count_as_full(dev, oracle):
    """A device length array holding values above chunk_size (up to 2^32-1) must not make a
    kernel load past a unit: they count as chunk_size.  Covers the one-segment padded
    kernel (L % 16 != 0, hashed), gf_apply_lens (L % 16 == 0) and the padded decode."""
    from elect_amd.batch import decode_batch_ex, encode_batch_ex
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    for L, hashed, B in ((4099, True, 3), (65536, False, 3), ((20 << 20) + 4, True, 2)):
        rng = np.random.default_rng(L)
        data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
        lens = np.full((B, k), 0xFFFFFFFF, np.uint32).view(np.int32)
        lens[1, 2] = L + 1
        lens[1, 3] = L - 3  # beyond 2^24: lengths must stay exact integers on the device
        par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
        hs = torch.empty((B, m), dtype=torch.int32, device=dev) if hashed else None
        d_data = _to(dev, data)
        encode_batch_ex(RSCoder(k, m), d_data, par, lengths=_to(dev, lens), hashes=hs)
        enc = oracle.Encoder(k, m)
        for s in range(B):
            want = enc.encode([oracle.zero_fill(data[s, j, :min(int(lens[s, j]) & 0xFFFFFFFF, L)], L)
                               for j in range(k)])
            for r in range(m):
                assert np.array_equal(par[s, r].cpu().numpy(), want[r])
                if hashed:
                    assert int(hs[s, r]) == oracle.java_hashcode(want[r])
        if L > 1 << 24:
            continue
        stripe = torch.cat([d_data, par], dim=1)
        out = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
        dl = np.concatenate([lens[:, 1:], np.full((B, 1), -1, np.int32)], axis=1)  # survivors 1, 2, 3, P0
        decode_batch_ex(RSCoder(k, m), stripe, [1, 2, 3, 4], [0], out, lengths=_to(dev, dl), inputs_by_unit=True)
        assert torch.equal(out[:, 0], d_data[:, 0])  # unit 0's lengths are all above L: full


@pytest.mark.parametrize("threads", [12, 24, 80])
def test_concurrent_streams_hashed_device_api(dev, oracle, threads):
    """Many threads, each launching hashed encodes on its own stream (the device API
    leases a per-stream scratch for the hash partials).  Stream-ordered pool scratch
    (hipMallocAsync / hipFreeAsync) corrupted partials in exactly this pattern
    (tools/sanitize/host_stress); every hash must still match the JDK loop.  With 80
    streams the 64 cached buffers change hands (a device-wide synchronize first)."""
    import threading
    from elect_amd.batch import encode_batch_ex
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    errors = []

    from tests.conftest import distinct_hip_streams
    own = distinct_hip_streams(threads, dev.index or 0)  # (torch.cuda.Stream() objects share a pool of 32)

    def worker(t):
        try:
            torch.cuda.set_device(dev)
            s = own[t]
            rng = np.random.default_rng(700 + t)
            for it in range(6):
                B, L = int(rng.integers(1, 5)), int(rng.choice([1500, 4099, 20000, 65536 + 4]))
                data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
                lens = rng.integers(0, L + 1, size=(B, k)).astype(np.int32)
                with torch.cuda.stream(s):
                    d = torch.from_numpy(data).to(dev, non_blocking=False)
                    dl = torch.from_numpy(lens).to(dev)
                    par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
                    hs = torch.empty((B, m), dtype=torch.int32, device=dev)
                    encode_batch_ex(coder, d, par, lengths=dl, hashes=hs, stream=s)
                s.synchronize()
                got_p, got_h = par.cpu().numpy(), hs.cpu().numpy()
                for b in range(B):
                    want = enc.encode([oracle.zero_fill(data[b, j, :lens[b, j]], L) for j in range(k)])
                    for r in range(m):
                        if not np.array_equal(got_p[b, r], want[r]):
                            errors.append(f"t{t} it{it} parity {b} {r}")
                        if int(got_h[b, r]) != oracle.java_hashcode(want[r]):
                            errors.append(f"t{t} it{it} hash {b} {r} L={L}")
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors[:5]


def test_scratch_handoff_waits_for_last_use_only(dev, oracle):
    """More streams than the hash scratch cache holds (64 per device): once 32 or
    more entries are assigned, each use records an event, and a handoff to
    another stream waits for that event on the device (hipStreamWaitEvent)
    instead of synchronizing the device from the calling thread
    (rs_kernels.hip scratch_lease).  80 streams launch hashed
    batches while an unrelated stream reads HBM for ~0.3 s: a device-wide
    synchronize at a handoff would hold the launching call until that work is
    done, so every launch of the last round must return in far less time (the
    launches' completion is not timed: with 4 hardware queues per process,
    streams share queues with the long work), and the hashes stay right."""
    import threading
    import time
    from elect_amd import _lib
    from elect_amd.batch import encode_batch_ex
    from elect_amd.coder import RSCoder
    k, m, B, L, S = 4, 2, 2, 65536 + 4, 80
    coder, enc = RSCoder(k, m), oracle.Encoder(k, m)
    rng = np.random.default_rng(99)
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    d = torch.from_numpy(data).to(dev)
    want = [enc.encode([data[b, j] for j in range(k)]) for b in range(B)]
    from tests.conftest import distinct_hip_streams
    streams = distinct_hip_streams(S, dev.index or 0)  # (torch.cuda.Stream() objects share a pool of 32)
    outs = [(torch.empty((B, m, L), dtype=torch.uint8, device=dev), torch.empty((B, m), dtype=torch.int32, device=dev))
            for _ in range(S)]
    errors, launch_s = [], [0.0] * S

    def round_of_calls():
        def one(i):
            try:
                torch.cuda.set_device(dev)
                par, hs = outs[i]
                t0 = time.perf_counter()
                encode_batch_ex(coder, d, par, hashes=hs, stream=streams[i])
                launch_s[i] = time.perf_counter() - t0
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))
        th = [threading.Thread(target=one, args=(i,)) for i in range(S)]
        for x in th:
            x.start()
        for x in th:
            x.join()

    round_of_calls()
    torch.cuda.synchronize()
    round_of_calls()  # every entry's last use now recorded under pressure
    torch.cuda.synchronize()
    buf = torch.empty(1 << 31, dtype=torch.uint8, device=dev)
    sink = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    long_stream = torch.cuda.Stream(dev)
    t0 = time.perf_counter()
    for _ in range(1000):  # 1,000 x 2 GiB reads: ~0.3 s on an MI355X
        _lib.hbm_probe(0, buf.data_ptr(), sink.data_ptr(), buf.numel(), stream=long_stream.cuda_stream)
    round_of_calls()
    slowest_launch = max(launch_s)
    long_stream.synchronize()
    long_s = time.perf_counter() - t0
    torch.cuda.synchronize()
    assert not errors, errors[:3]
    for par, hs in outs:
        got_p, got_h = par.cpu().numpy(), hs.cpu().numpy()
        for b in range(B):
            for r in range(m):
                assert np.array_equal(got_p[b, r], want[b][r])
                assert int(got_h[b, r]) == oracle.java_hashcode(want[b][r])
    print(f"scratch handoff: slowest launch {slowest_launch * 1e3:.2f} ms beside {long_s * 1e3:.0f} ms of other work")
    assert long_s > 0.15, f"the unrelated work ran only {long_s:.3f} s: no room for the timing check"
    assert slowest_launch < long_s / 3, (f"a hashed launch took {slowest_launch * 1e3:.1f} ms beside {long_s * 1e3:.0f} ms "
                                         "of unrelated work: a scratch handoff synchronized the device")
