"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, byte for byte.

Bar: bit-exact.  Cases follow the reference's coder surface (EC/erasure_coder.c:
encode :74-98, encodeUpdate :100-142, decode :202-226) and the edge cases it
meets in ELECT: odd chunk lengths (codeLength is not a multiple of 16,
StorageService.java:331-339), every erasure pattern up to m, the compat-mode
zero rows, unaligned buffers, and row counts above the fast kernel's 4.
"""
import itertools

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

LENGTHS = [1, 15, 16, 17, 33, 1024, 4099, 65536]


def _rand(rng, *shape):
    return rng.integers(0, 256, size=shape, dtype=np.uint8)


def _to(dev, a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (2, 2), (3, 2), (6, 3), (10, 4), (1, 1), (4, 10)])
@pytest.mark.parametrize("L", LENGTHS)
def test_encode_batch_matches_oracle(dev, oracle, k, m, L):
    from elect_amd.batch import encode_batch
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(1000 * k + 10 * m + L)
    B = 3
    data = _rand(rng, B, k, L)
    c = RSCoder(k, m)
    par = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
    encode_batch(c, _to(dev, data), par)
    got = par.cpu().numpy()
    enc = oracle.Encoder(k, m)
    for s in range(B):
        want = enc.encode([data[s, j] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[s, r], want[r]), (s, r)


def _patterns(k, m, limit=None):
    n = k + m
    pats = []
    for e in range(1, m + 1):
        for er in itertools.combinations(range(n), e):
            pats.append(list(er))
    return pats if limit is None else pats[:limit]


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (3, 2)])
@pytest.mark.parametrize("mode", [0, 1])
def test_decode_all_patterns_match_oracle(dev, oracle, k, m, mode):
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(7 + k + m + mode)
    B, L = 2, 4099
    c = RSCoder(k, m)
    data = _to(dev, _rand(rng, B, k, L))
    stripe = torch.zeros((B, k + m, L), dtype=torch.uint8, device=dev)
    stripe[:, :k] = data
    encode_batch(c, stripe[:, :k], stripe[:, k:])
    st_host = stripe.cpu().numpy()
    pats = _patterns(k, m)
    if len(pats) > 120:
        pats = [pats[i] for i in np.random.default_rng(3).choice(len(pats), 120, replace=False)]
    for erased in pats:
        survivors = [i for i in range(k + m) if i not in erased][:k]
        if mode == 0:
            order = list(rng.permutation(survivors))  # any input order, as ELECT's {4,1,2,3}
        else:
            order = survivors
        out = torch.zeros((B, len(erased), L), dtype=torch.uint8, device=dev)
        decode_batch(c, stripe, order, erased, out, mode=mode, inputs_by_unit=True)
        got = out.cpu().numpy()
        for s in range(B):
            rc, want = oracle.decode(k, m, [st_host[s, i] for i in order], order, erased, strict=bool(mode))
            assert rc == 0
            for r in range(len(erased)):
                assert np.array_equal(got[s, r], want[r]), (erased, order, s, r)
            if mode == 1:  # strict rebuilds every erased unit
                for r, e in enumerate(erased):
                    assert np.array_equal(got[s, r], st_host[s, e])


def test_compat_zero_rows_quirk(dev, oracle):
    """EC/erasure_coder.c:261-281: rows past the erased-DATA count stay zero."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 1000, 2
    rng = np.random.default_rng(5)
    c = RSCoder(k, m)
    stripe = torch.zeros((B, k + m, L), dtype=torch.uint8, device=dev)
    stripe[:, :k] = _to(dev, _rand(rng, B, k, L))
    encode_batch(c, stripe[:, :k], stripe[:, k:])
    h = stripe.cpu().numpy()
    for erased, survivors in (([0, 4], [1, 2, 3, 5]), ([4, 0], [1, 2, 3, 5]), ([4], [0, 1, 2, 3]),
                              ([4, 5], [0, 1, 2, 3])):
        out = torch.full((B, len(erased), L), 0xAB, dtype=torch.uint8, device=dev)
        decode_batch(c, stripe, survivors, erased, out, mode=0, inputs_by_unit=True)
        got = out.cpu().numpy()
        ned = sum(e < k for e in erased)
        for r, e in enumerate(erased):
            if r < ned:
                assert np.array_equal(got[:, r], h[:, e])
            else:
                assert not got[:, r].any()


@pytest.mark.parametrize("L", [1, 17, 4099, 65536])
@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (2, 6)])
def test_encode_update_matches_oracle(dev, oracle, k, m, L):
    from elect_amd.batch import encode_update_batch
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L + k)
    B = 3
    c = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    for target in range(k):
        old = _rand(rng, B, L)
        new = _rand(rng, B, L)
        pin = _rand(rng, B, m, L)
        pout = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
        encode_update_batch(c, target, _to(dev, old), _to(dev, new), _to(dev, pin), pout)
        got = pout.cpu().numpy()
        for s in range(B):
            want = enc.encode_update([old[s], new[s]] + [pin[s, r] for r in range(m)], target)
            for r in range(m):
                assert np.array_equal(got[s, r], want[r])


def test_update_in_place_equals_reencode(dev):
    from elect_amd.batch import encode_batch, encode_update_batch
    from elect_amd.coder import RSCoder
    k, m, B, L = 4, 2, 16, 65536 + 4
    rng = np.random.default_rng(9)
    c = RSCoder(k, m)
    data = _to(dev, _rand(rng, B, k, L))
    par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
    encode_batch(c, data, par)
    new0 = _to(dev, _rand(rng, B, L))
    encode_update_batch(c, 0, data[:, 0], new0, par, par)  # in place, as ELECT updates stored parity
    data[:, 0] = new0
    ref = torch.empty_like(par)
    encode_batch(c, data, ref)
    torch.cuda.synchronize()
    assert torch.equal(par, ref)


def _shifted(dev, a, shift):
    """A device copy of a at a byte offset `shift` from an aligned allocation."""
    big = torch.zeros(a.size + 64, dtype=torch.uint8, device=dev)
    view = big[shift:shift + a.size].view(*a.shape)
    view.copy_(_to(dev, a))
    return view


@pytest.mark.parametrize("shift", [1, 3, 4, 8, 13])
@pytest.mark.parametrize("L", [333, 4096, 4404020 // 256])
def test_unaligned_layouts(dev, oracle, shift, L):
    """Column starts at any byte offset (and strides that are not multiples of
    16, e.g. ELECT's codeLength in a contiguous [B][k+m][L] layout): the dwordx4
    kernels run on unaligned addresses (rs_kernels.hip unaligned_vector_ok);
    encode, decode, update and the fused hash must stay bit-exact."""
    from elect_amd.batch import decode_batch, encode_batch, encode_batch_hashed, encode_update_batch
    from elect_amd.coder import RSCoder
    k, m, B = 4, 2, 5
    rng = np.random.default_rng(shift * 1000 + L)
    c = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    data = _rand(rng, B, k, L)
    view = _shifted(dev, data, shift)
    pv = _shifted(dev, np.zeros((B, m, L), np.uint8), (shift * 5) % 16)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_batch_hashed(c, view, pv, hashes)
    got, gh = pv.cpu().numpy(), hashes.cpu().numpy()
    want = [enc.encode([data[s, j] for j in range(k)]) for s in range(B)]
    for s in range(B):
        for r in range(m):
            assert np.array_equal(got[s, r], want[s][r]), (s, r)
            assert int(gh[s, r]) == oracle.java_hashcode(want[s][r])
    pv2 = _shifted(dev, np.zeros((B, m, L), np.uint8), (shift + 7) % 16)
    encode_batch(c, view, pv2)
    assert np.array_equal(pv2.cpu().numpy(), got)
    # decode from a stripe-resident layout at an odd offset: survivors {1,2,3,4}
    stripe = np.concatenate([data, got], axis=1)
    sv = _shifted(dev, stripe, shift)
    out = _shifted(dev, np.zeros((B, 1, L), np.uint8), (shift + 2) % 16)
    decode_batch(c, sv, [4, 1, 2, 3], [0], out, inputs_by_unit=True)
    assert np.array_equal(out.cpu().numpy()[:, 0], data[:, 0])
    # parity update with every column misaligned
    new = _rand(rng, B, L)
    pout = _shifted(dev, np.zeros((B, m, L), np.uint8), (shift + 9) % 16)
    encode_update_batch(c, 2, view[:, 2], _shifted(dev, new, (shift + 1) % 16), pv, pout)
    gu = pout.cpu().numpy()
    for s in range(B):
        wu = enc.encode_update([data[s, 2], new[s]] + [got[s, r] for r in range(m)], 2)
        for r in range(m):
            assert np.array_equal(gu[s, r], wu[r])


def test_unaligned_probe_reports_vector_path(dev):
    """The one-time per-device check behind the unaligned fast path passes on
    this device (else misaligned layouts would silently take the byte kernel)."""
    from elect_amd import _lib
    assert _lib.unaligned_vector_ok()


def test_apply_batch_many_rows(dev, oracle):
    """rows > 4 runs as row groups of the fast kernel."""
    from elect_amd.batch import apply_batch
    rng = np.random.default_rng(11)
    rows, cols, B, L = 11, 16, 4, 4096 + 7
    coef = _rand(rng, rows, cols)
    coef[0, :] = 0
    coef[1, :] = 1
    src = [_to(dev, _rand(rng, B, L)) for _ in range(cols)]
    dst = [torch.zeros((B, L), dtype=torch.uint8, device=dev) for _ in range(rows)]
    apply_batch(coef, src, dst)
    hs = [t.cpu().numpy() for t in src]
    for s in range(B):
        want = oracle.apply(coef, [h[s] for h in hs])
        for r in range(rows):
            assert np.array_equal(dst[r][s].cpu().numpy(), want[r]), r


def test_host_path_java_api_roundtrip(dev, oracle):
    """NativeRSEncoder/Decoder over host buffers (the JNI convention), incl. a
    chunk longer than the 1 MiB pipeline step and an odd length."""
    from elect_amd.coder import ByteBuffer, ErasureCoderOptions, NativeRSDecoder, NativeRSEncoder
    k, m = 4, 2
    for L in (4099, (1 << 20) * 3 + 5):
        rng = np.random.default_rng(L)
        raw = _rand(rng, k, L)
        data = [ByteBuffer.direct_from(raw[j].copy()) for j in range(k)]
        par = [ByteBuffer.allocateDirect(L) for _ in range(m)]
        enc = NativeRSEncoder(ErasureCoderOptions(k, m))
        enc.encode(data, par)
        want = oracle.Encoder(k, m).encode(list(raw))
        for r in range(m):
            assert np.array_equal(par[r].array(), want[r])
        dec = NativeRSDecoder(ErasureCoderOptions(k, m))
        out = [ByteBuffer.allocateDirect(L)]
        dec.decode([par[0], data[1], data[2], data[3]], [4, 1, 2, 3], [0], out)
        assert out[0].compareTo(data[0].rewind()) == 0
        enc.release()
        dec.release()


def _sample(B, extra=6, seed=0):
    """first, second, middle pair, last two, and a few seeded random stripes"""
    rng = np.random.default_rng(seed)
    picks = {0, 1, B // 2 - 1, B // 2, B - 2, B - 1} | {int(x) for x in rng.integers(0, B, extra)}
    return sorted(p for p in picks if 0 <= p < B)


def test_large_batch_roundtrip_properties(dev, oracle):
    """BASELINE configs[1]/[2] at full size: RS(6,4), 64 KiB, 4096 stripes (1 GiB
    data) in the bench's [B][k+m][L] layout.  Sampled stripes (first, middle,
    last: the grid's first and last blocks) byte-for-byte against the oracle for
    the parity and for every single data erasure's rebuilt unit; every stripe by
    decode(encode(x)) == x; linearity encode(a ^ b) == encode(a) ^ encode(b)."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 65536, 4096
    c = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    g = torch.Generator(device=dev).manual_seed(123)
    stripe = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
    stripe[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    encode_batch(c, stripe[:, :k], stripe[:, k:])
    picks = _sample(B)
    host = {s: stripe[s].cpu().numpy() for s in picks}
    for s, h in host.items():
        want = enc.encode([h[j] for j in range(k)])
        assert all(np.array_equal(h[k + r], want[r]) for r in range(m)), s
    out = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
    for e in range(k):
        surv = [i for i in range(k + m) if i != e][:k]
        decode_batch(c, stripe, surv, [e], out, inputs_by_unit=True)
        assert torch.equal(out[:, 0], stripe[:, e])
        for s in picks:
            rc, want = oracle.decode(k, m, [host[s][i] for i in surv], surv, [e])
            assert rc == 0 and np.array_equal(out[s, 0].cpu().numpy(), want[0]), (e, s)
    del out
    a = stripe[: B // 4, :k].clone()
    b = torch.randint(0, 256, a.shape, dtype=torch.uint8, device=dev, generator=g)
    pa = torch.empty((B // 4, m, L), dtype=torch.uint8, device=dev)
    pb = torch.empty_like(pa)
    pab = torch.empty_like(pa)
    encode_batch(c, a, pa)
    encode_batch(c, b, pb)
    encode_batch(c, a ^ b, pab)
    assert torch.equal(pab, pa ^ pb)


def _zero_padded(data, lens):
    out = data.copy()
    B, k, L = data.shape
    for s in range(B):
        for j in range(k):
            out[s, j, lens[s, j]:] = 0
    return out


@pytest.mark.parametrize("k,m,L", [(4, 2, 65536), (4, 2, 4099), (8, 4, 1000), (3, 2, 17), (10, 4, 333),
                                   (4, 2, 1040), (4, 2, 16), (2, 1, 4096 + 48), (8, 4, 2048), (5, 3, 1056),
                                   (10, 4, 4096)])
def test_encode_batch_padded_ignores_bytes_past_length(dev, oracle, k, m, L):
    """ELECT zero-fills each SSTable to codeLength (ECMessageVerbHandler.java:292-310)
    and pads missing primaries with all-zero chunks (:174-184).  The padded kernel
    must give the parity of the zero-padded stripe whatever the bytes past each
    content length hold: the buffers hold 0xFF garbage there.  L % 16 == 0 cases
    take gf_apply_lens (U segments per lane; L = 1040 makes its waves straddle
    stripes), the others gf_apply_x16<PAD>."""
    from elect_amd.batch import encode_batch_padded
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L * 3 + k)
    B = 6
    data = _rand(rng, B, k, L)
    lens = rng.integers(0, L + 1, size=(B, k)).astype(np.int32)
    lens[0, :] = L
    lens[1, :] = 0
    lens[2, 0] = 0
    lens[3, :] = np.minimum(L, [16 * (j + 1) + 3 for j in range(k)])
    garbage = data.copy()
    for s in range(B):
        for j in range(k):
            garbage[s, j, lens[s, j]:] = 0xFF
    par = torch.full((B, m, L), 0x33, dtype=torch.uint8, device=dev)
    encode_batch_padded(RSCoder(k, m), _to(dev, garbage), _to(dev, lens), par)
    got = par.cpu().numpy()
    want_in = _zero_padded(data, lens)
    enc = oracle.Encoder(k, m)
    for s in range(B):
        want = enc.encode([want_in[s, j] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[s, r], want[r]), (s, r, lens[s])


def test_encode_padded_host_path(dev, oracle):
    """elect_ec_encode_padded: NULL for an all-zero filler unit, lengths below and
    across the 1 MiB pipeline step, ELECT's codeLength-shaped odd total."""
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    L = (1 << 20) * 2 + 4404020 % 16 + 48
    rng = np.random.default_rng(4)
    lens = [L, (1 << 20) + 7, 0, 5]
    bufs = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    addrs = [b.ctypes.data if n else None for b, n in zip(bufs, lens)]
    par = [np.zeros(L, np.uint8) for _ in range(m)]
    RSCoder(k, m).encode_padded_host(addrs, lens, [p.ctypes.data for p in par], L)
    padded = [np.concatenate([b[:n], np.zeros(L - n, np.uint8)]) for b, n in zip(bufs, lens)]
    want = oracle.Encoder(k, m).encode(padded)
    for r in range(m):
        assert np.array_equal(par[r], want[r])


def test_padded_unaligned(dev, oracle):
    from elect_amd.batch import encode_batch_padded
    from elect_amd.coder import RSCoder
    k, m, B, L = 4, 2, 3, 100
    rng = np.random.default_rng(8)
    data = _rand(rng, B, k, L)
    lens = np.array([[100, 50, 0, 99], [1, 2, 3, 4], [100, 100, 100, 100]], np.int32)
    big = torch.zeros(B * k * L + 16, dtype=torch.uint8, device=dev)
    view = big[3:3 + B * k * L].view(B, k, L)
    view.copy_(_to(dev, data))
    par = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
    encode_batch_padded(RSCoder(k, m), view, _to(dev, lens), par)
    want_in = _zero_padded(data, lens)
    enc = oracle.Encoder(k, m)
    for s in range(B):
        want = enc.encode([want_in[s, j] for j in range(k)])
        for r in range(m):
            assert np.array_equal(par[s, r].cpu().numpy(), want[r])


def test_host_path_concurrent_callers(dev, oracle):
    """The C ABI is re-entrant: many threads encoding and decoding at once on ONE
    coder (the reference is safe only with a coder per task, EC/NativeRSEncoder.c:25-29)."""
    import threading
    from elect_amd.coder import RSCoder
    k, m, L = 4, 2, 300001
    coder = RSCoder(k, m)
    errors = []

    def worker(t):
        try:
            rng = np.random.default_rng(100 + t)
            d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
            p = [np.empty(L, np.uint8) for _ in range(m)]
            for _ in range(3):
                coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
                out = np.empty(L, np.uint8)
                coder.decode_host([p[1].ctypes.data, d[1].ctypes.data, d[2].ctypes.data, d[3].ctypes.data],
                                  [5, 1, 2, 3], [0], [out.ctypes.data], L)
                if not np.array_equal(out, d[0]):
                    errors.append(f"thread {t} decode mismatch")
            want = oracle.Encoder(k, m).encode(d)
            if not all(np.array_equal(a, b) for a, b in zip(p, want)):
                errors.append(f"thread {t} parity mismatch")
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(12)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors


@pytest.mark.parametrize("k,m,L", [(4, 2, 65536), (4, 2, 4099), (4, 2, 1), (4, 2, 15), (8, 4, 1024), (4, 2, 1 << 20),
                                   (4, 10, 333), (3, 2, 4404020 // 64), (4, 2, 1040), (6, 3, 16008)])
def test_encode_batch_hashed_matches_java_hashcode(dev, oracle, k, m, L):
    """Fused parity hash == java.nio.ByteBuffer.hashCode() of each parity unit
    (ECMessageVerbHandler.java:326-329), incl. tails, waves straddling stripes
    (1040, 16008: every / some waves; the launch's last wave partial), the
    memset-and-add mode (< 64 segments per stripe) and row groups (m > 4)."""
    from elect_amd.batch import encode_batch_hashed
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L + 13 * k)
    B = 5
    data = _rand(rng, B, k, L)
    par = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_batch_hashed(RSCoder(k, m), _to(dev, data), par, hashes)
    got_p, got_h = par.cpu().numpy(), hashes.cpu().numpy()
    enc = oracle.Encoder(k, m)
    for s in range(B):
        want = enc.encode([data[s, j] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got_p[s, r], want[r])
            assert int(got_h[s, r]) == oracle.java_hashcode(want[r]), (s, r)


def test_encode_hashed_host_path(dev, oracle):
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    for L in (4404020, 17, 0):
        rng = np.random.default_rng(L)
        d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        p = [np.zeros(L, np.uint8) for _ in range(m)]
        hs = RSCoder(k, m).encode_hashed_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
        want = oracle.Encoder(k, m).encode(d) if L else [np.zeros(0, np.uint8)] * m
        for r in range(m):
            assert np.array_equal(p[r], want[r])
            assert hs[r] == oracle.java_hashcode(want[r])


def test_host_device_policy(dev, oracle):
    """elect_ec_set_host_devices: threads pinned round robin to the listed devices
    (one JVM driving every GPU of a node); bad ids rejected; default restored."""
    import threading
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    ndev = torch.cuda.device_count()
    with pytest.raises(_lib.ECInvalidArgument):
        _lib.set_host_devices([ndev])
    _lib.set_host_devices(list(range(ndev)))
    try:
        k, m, L = 4, 2, 70001
        coder = RSCoder(k, m)
        ok = []

        def worker(t):
            rng = np.random.default_rng(t)
            d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
            p = [np.empty(L, np.uint8) for _ in range(m)]
            coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
            want = oracle.Encoder(k, m).encode(d)
            ok.append(all(np.array_equal(a, b) for a, b in zip(p, want)))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(2 * ndev + 1)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert ok and all(ok)
    finally:
        _lib.set_host_devices([])


def test_launch_split_beyond_2pow31_segments(dev):
    """A batch with more than 2^31 16-byte segments is split into several launches
    (per-launch index < 2^31).  RS(2,1) has E[1][0] = 1/(1^0) = 1, so its parity
    must equal the data exactly: a size-independent check at 32 GiB per column."""
    from elect_amd.batch import encode_batch
    from elect_amd.coder import RSCoder
    free, _ = torch.cuda.mem_get_info()
    B, L = (1 << 31) + 4099, 16
    if free < 2 * B * L + (4 << 30):
        pytest.skip("needs ~70 GiB of free HBM")
    data = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
    data.view(-1)[: 1 << 20].random_(0, 256)
    data.view(-1)[-(1 << 20):].random_(0, 256)
    par = torch.zeros((B, 1, L), dtype=torch.uint8, device=dev)
    encode_batch(RSCoder(1, 1), data, par)
    torch.cuda.synchronize()
    assert torch.equal(par.view(-1)[: 1 << 20], data.view(-1)[: 1 << 20])
    assert torch.equal(par.view(-1)[-(1 << 20):], data.view(-1)[-(1 << 20):])  # last launch window
    del data, par
    torch.cuda.empty_cache()


def test_rs12_8_every_double_erasure_at_256k(dev):
    """BASELINE configs[4] shape: RS(12,8), 256 KiB chunks; every 2-erasure
    pattern (66) rebuilt in strict mode from the first 8 survivors must equal the
    lost units (MDS round trip at full size)."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 8, 4, 262144, 32
    c = RSCoder(k, m)
    st = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
    st[:, :k].random_(0, 256)
    encode_batch(c, st[:, :k], st[:, k:])
    out = torch.empty((B, 2, L), dtype=torch.uint8, device=dev)
    for erased in itertools.combinations(range(k + m), 2):
        surv = [i for i in range(k + m) if i not in erased][:k]
        decode_batch(c, st, surv, list(erased), out, mode=1, inputs_by_unit=True)
        assert torch.equal(out[:, 0], st[:, erased[0]]) and torch.equal(out[:, 1], st[:, erased[1]]), erased


def test_mixed_size_batch_properties(dev, oracle):
    """BASELINE configs[3] shape, scaled: 1 KiB / 4 KiB / 1 MiB classes; sampled
    stripes against the oracle, every stripe by the decode round trip."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    c = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    for L, B in ((1024, 8192), (4096, 2048), (1 << 20, 16)):
        st = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
        st[:, :k].random_(0, 256)
        encode_batch(c, st[:, :k], st[:, k:])
        out = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
        decode_batch(c, st, [1, 2, 3, 4], [0], out, inputs_by_unit=True)
        assert torch.equal(out[:, 0], st[:, 0])
        for s in (0, B // 2, B - 1):
            h = st[s].cpu().numpy()
            want = enc.encode([h[j] for j in range(k)])
            assert np.array_equal(h[k], want[0]) and np.array_equal(h[k + 1], want[1])


def test_cross_thread_batching(dev, oracle):
    """Cross-thread batching (on by default): concurrent one-stripe host calls share one arena,
    H2D, launch and D2H.  Mixed shapes (two lengths, encode and decode) force
    batches to close early and the two arenas to alternate; every call must
    still get exactly its own parity / rebuilt unit."""
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
                L = 65536 + 48 if t % 3 else 4099
                rng = np.random.default_rng(1000 + t)
                for it in range(4):
                    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
                    p = [np.empty(L, np.uint8) for _ in range(m)]
                    coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
                    want = enc.encode(d)
                    if not all(np.array_equal(a, b) for a, b in zip(p, want)):
                        errors.append(f"t{t} it{it} parity")
                    out = np.empty(L, np.uint8)
                    coder.decode_host([p[0].ctypes.data] + [x.ctypes.data for x in d[1:]], [4, 1, 2, 3], [0],
                                      [out.ctypes.data], L)
                    if not np.array_equal(out, d[0]):
                        errors.append(f"t{t} it{it} decode")
            except Exception as e:  # noqa: BLE001
                errors.append(repr(e))

        th = [threading.Thread(target=worker, args=(t,)) for t in range(24)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        # a stripe larger than the arena falls back to the direct path (batching is
        # on by default, so the batcher may already run with the default 256 MiB arena)
        L = max(3 << 20, (256 << 20) // k + 4096)
        d = [np.full(L, j + 1, np.uint8) for j in range(k)]
        p = [np.empty(L, np.uint8) for _ in range(m)]
        coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
        want = enc.encode(d)
        assert all(np.array_equal(a, b) for a, b in zip(p, want))
    finally:
        _lib.set_batching(True)  # the library default
    assert not errors, errors[:5]


def test_tiled_layout_equals_contiguous(dev):
    """bench.py's layout for chunks above 64 KiB ([B][L/64K][k+m][64K], coded as
    B*L/64K stripes of 64 KiB): every chunk's parity and rebuilt
    unit are the same bytes as coding the chunk whole in [B][k+m][L]."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, B, L, T = 4, 2, 3, 1 << 20, 1 << 16
    coder = RSCoder(k, m)
    g = torch.Generator(device=dev).manual_seed(31)
    flat = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
    flat[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    tiled = torch.empty((B, L // T, k + m, T), dtype=torch.uint8, device=dev)
    tiled[:, :, :k] = flat[:, :k].reshape(B, k, L // T, T).transpose(1, 2)
    view = tiled.view(B * (L // T), k + m, T)
    encode_batch(coder, flat[:, :k], flat[:, k:])
    encode_batch(coder, view[:, :k], view[:, k:])
    out = torch.empty((B * (L // T), 1, T), dtype=torch.uint8, device=dev)
    decode_batch(coder, view, [1, 2, 3, 4], [0], out, inputs_by_unit=True)
    torch.cuda.synchronize()
    assert torch.equal(tiled[:, :, k:].transpose(1, 2).reshape(B, m, L), flat[:, k:])
    assert torch.equal(out.view(B, L), flat[:, 0])


def test_batcher_arena_failure_falls_back(dev, tmp_path):
    """ELECT_EC_BATCH_ARENA_MB far beyond what can be pinned: the batcher's arena
    allocation fails, it frees what it got and every host call runs on the
    per-thread engine instead of failing (and keeps doing so)."""
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = f"""
import sys, numpy as np
sys.path.insert(0, {ROOT!r})
from elect_amd.coder import RSCoder
from oracle import ec_oracle
k, m = 4, 2
c = RSCoder(k, m)
for L in (4404020, 4099, 65536 * 3):
    for it in range(2):
        rng = np.random.default_rng(L + it)
        d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        p = [np.empty(L, np.uint8) for _ in range(m)]
        c.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
        want = ec_oracle.Encoder(k, m).encode(d)
        assert all(np.array_equal(a, b) for a, b in zip(p, want)), L
print("fallback ok")
"""
    env = dict(__import__("os").environ, ELECT_EC_BATCH_ARENA_MB=str(64 << 20))  # 64 TiB per arena
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "fallback ok" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("k,m", [(3, 9), (2, 12), (5, 9)])
def test_hashed_update_of_wide_codes(dev, oracle, k, m):
    """encode_update_ex with hashes for m >= 9 (2 + m columns, wider than the
    hashed vector kernels): the byte-granular kernel's atomic hash path, on the
    device API and the host path; bit-exact parity and ByteBuffer.hashCode()."""
    from elect_amd.batch import encode_update_batch_ex
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(k * 100 + m)
    B, L, t = 3, 1000 + 7, k - 1
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    old, new = _rand(rng, B, L), _rand(rng, B, L)
    pin = _rand(rng, B, m, L)
    lens = np.array([[L, L], [17, 900], [0, L]], np.int32)
    pout = torch.zeros((B, m, L), dtype=torch.uint8, device=dev)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_update_batch_ex(coder, t, _to(dev, old), _to(dev, new), _to(dev, pin), pout,
                           lengths=_to(dev, lens), hashes=hashes)
    got, gh = pout.cpu().numpy(), hashes.cpu().numpy()
    for s in range(B):
        o = np.where(np.arange(L) < lens[s, 0], old[s], 0).astype(np.uint8)
        n = np.where(np.arange(L) < lens[s, 1], new[s], 0).astype(np.uint8)
        want = enc.encode_update([o, n] + [pin[s, r] for r in range(m)], t)
        for r in range(m):
            assert np.array_equal(got[s, r], want[r]), (s, r)
            assert int(gh[s, r]) == oracle.java_hashcode(want[r]), (s, r)
    # host path (JNI encodeUpdateExImpl convention)
    s = 1
    outs = [np.zeros(L, np.uint8) for _ in range(m)]
    ins = [old[s], new[s]] + [np.ascontiguousarray(pin[s, r]) for r in range(m)]
    hs = coder.encode_update_ex_host([x.ctypes.data for x in ins], t, [x.ctypes.data for x in outs], L,
                                     old_new_lengths=[int(lens[s, 0]), int(lens[s, 1])], hashed=True)
    for r in range(m):
        assert np.array_equal(outs[r], got[s, r])
        assert hs[r] == int(gh[s, r])


@pytest.mark.parametrize("hashed", [False, True])
def test_host_update_of_wide_code_above_tile(dev, oracle, hashed):
    """The host path's batcher stores units above 64 KiB as tiles, but a tiled
    launch needs the padded vector kernels (at most 10 columns): the (2+m)-column
    update of an m = 9 code at ELECT's codeLength (4,404,020 B) must run untiled
    instead of failing its batch.  Two concurrent callers (so the batch is shared);
    against the oracle, bytes and hashCode()."""
    import threading
    from elect_amd.coder import RSCoder
    k, m, L, t = 3, 9, 4404020, 1
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    calls = []
    for c in range(2):
        rng = np.random.default_rng(90 + c)
        old, new = rng.integers(0, 256, L, dtype=np.uint8), rng.integers(0, 256, L, dtype=np.uint8)
        pin = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(m)]
        lens = [L - 1000 * (c + 1), L - 77 * c]
        calls.append((old, new, pin, lens, [np.zeros(L, np.uint8) for _ in range(m)], [None]))

    def run(c):
        torch.cuda.set_device(dev)
        old, new, pin, lens, outs, res = calls[c]
        ins = [old, new] + pin
        res[0] = coder.encode_update_ex_host([x.ctypes.data for x in ins], t, [x.ctypes.data for x in outs], L,
                                             old_new_lengths=lens, hashed=hashed)
    th = [threading.Thread(target=run, args=(c,)) for c in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    for old, new, pin, lens, outs, res in calls:
        o = np.where(np.arange(L) < lens[0], old, 0).astype(np.uint8)
        n = np.where(np.arange(L) < lens[1], new, 0).astype(np.uint8)
        want = enc.encode_update([o, n] + pin, t)
        for r in range(m):
            assert np.array_equal(outs[r], want[r]), r
            if hashed:
                assert res[0][r] == oracle.java_hashcode(want[r]), r


@pytest.mark.parametrize("k,m", [(4, 2), (3, 5)])
def test_encode_decode_batches_equal_per_batch_calls(dev, oracle, k, m):
    """elect_ec_encode_batches / _decode_batches (several chunk sizes, one call):
    the same bytes as one encode_batch / decode_batch per element.  Mixes
    groupable batches (whole segments; more than 8 of them: two launches) with
    ones that launch alone (L % 16 != 0, a misaligned base) and empty ones;
    m = 5: two row groups; sampled stripes against the oracle."""
    from elect_amd.batch import decode_batch, decode_batches, encode_batch, encode_batches
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(31 * k + m)
    coder = RSCoder(k, m)
    shapes = [(64, 1024), (9, 4096), (3, 65536), (5, 4099), (2, 48), (0, 1024), (7, 16), (4, 2048), (3, 1024),
              (2, 8192), (6, 512), (1, 65536 + 16), (5, 160)]
    stripes = []
    for i, (B, L) in enumerate(shapes):
        if i == 4:  # a misaligned base: the vector kernels still run it, alone
            big = torch.zeros(B * (k + m) * L + 16, dtype=torch.uint8, device=dev)
            st = big[3:3 + B * (k + m) * L].view(B, k + m, L)
        else:
            st = torch.zeros((B, k + m, L), dtype=torch.uint8, device=dev)
        st[:, :k] = _to(dev, _rand(rng, B, k, L))
        stripes.append(st)
    encode_batches(coder, [(st[:, :k], st[:, k:]) for st in stripes])
    ref = [torch.zeros_like(st[:, k:]) for st in stripes]
    for st, r in zip(stripes, ref):
        if st.shape[0]:
            encode_batch(coder, st[:, :k], r)
    torch.cuda.synchronize()
    enc = oracle.Encoder(k, m)
    for st, r in zip(stripes, ref):
        assert torch.equal(st[:, k:], r)
        if st.shape[0]:
            h = st[-1].cpu().numpy()
            want = enc.encode([h[j] for j in range(k)])
            assert all(np.array_equal(h[k + q], want[q]) for q in range(m))
    erased = [0, k] if m >= 2 else [0]
    surv = [i for i in range(k + m) if i not in erased][:k]
    outs = [torch.full((st.shape[0], len(erased), st.shape[2]), 0x5A, dtype=torch.uint8, device=dev) for st in stripes]
    decode_batches(coder, list(zip(stripes, outs)), surv, erased, mode=1, inputs_by_unit=True)
    torch.cuda.synchronize()
    for st, o in zip(stripes, outs):
        for q, e in enumerate(erased):
            assert torch.equal(o[:, q], st[:, e])


@pytest.mark.parametrize("helpers", ["0", "1", "16"])
def test_lone_caller_copy_fanout(dev, helpers):
    """The batcher's copy fan-out (host_path.cpp CopyPool: a caller with at most
    one other call in flight shares its staging copies with helper threads):
    one caller, then two racing for the pool, on ELECT's codeLength and a 2 MB
    unit, through encode_ex (padded + hashed), decode_ex and encode_update_ex;
    bit-exact against the oracle with the pool off (0), minimal (1) and widest (16)."""
    import subprocess
    import sys
    from tests.conftest import ROOT
    code = f"""
import sys, threading, numpy as np
sys.path.insert(0, {ROOT!r})
from elect_amd.coder import RSCoder
from oracle import ec_oracle
k, m = 4, 2
c = RSCoder(k, m)
enc = ec_oracle.Encoder(k, m)
bad = []

def one(seed, L):
    rng = np.random.default_rng(seed)
    d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    lens = [L, L - 1000 - seed % 7, L // 3, 0]
    z = [np.where(np.arange(L) < n, x, 0).astype(np.uint8) for x, n in zip(d, lens)]
    p = [np.empty(L, np.uint8) for _ in range(m)]
    hs = c.encode_ex_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L, data_lengths=lens, hashed=True)
    want = enc.encode(z)
    if not all(np.array_equal(a, b) for a, b in zip(p, want)) or hs != [ec_oracle.java_hashcode(w) for w in want]:
        bad.append(("encode_ex", seed, L))
    out = [np.empty(L, np.uint8)]
    c.decode_ex_host([z[1].ctypes.data, z[2].ctypes.data, z[3].ctypes.data, p[0].ctypes.data], [1, 2, 3, 4], [0],
                     [x.ctypes.data for x in out], L)
    if not np.array_equal(out[0], z[0]):
        bad.append(("decode_ex", seed, L))
    new = rng.integers(0, 256, L, dtype=np.uint8)
    q = [np.empty(L, np.uint8) for _ in range(m)]
    c.encode_update_ex_host([z[2].ctypes.data, new.ctypes.data, p[0].ctypes.data, p[1].ctypes.data], 2,
                            [x.ctypes.data for x in q], L)
    z[2] = new
    if not all(np.array_equal(a, b) for a, b in zip(q, enc.encode(z))):
        bad.append(("update", seed, L))

for L in (4404020, 2 << 20):
    one(1, L)  # a lone caller
    th = [threading.Thread(target=one, args=(s, L)) for s in (2, 3)]  # two callers racing for the pool
    [t.start() for t in th]
    [t.join() for t in th]
print("bad", bad)
assert not bad
print("fanout ok")
"""
    env = dict(__import__("os").environ, ELECT_EC_COPY_THREADS=helpers)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0 and "fanout ok" in r.stdout, r.stdout + r.stderr


def test_configs0_literal_every_byte(dev, oracle):
    """BASELINE configs[0] as written: RS(6,4) encode of 1,000 random 64 KiB data
    chunks (250 stripes of k = 4), every parity byte against the oracle, through
    both boundaries ELECT has: the device batch (elect_ec_encode_batch) and the
    JNI calling convention, one synchronous elect_ec_encode per stripe
    (EC/NativeRSEncoder.c:43-61).  Then ErasureCodeTest's decode on every stripe
    (ErasureCodeTest.java:89-109: erase {0}, decodeIndexes {4, 1, 2, 3}, inputs
    [parity 0, data 1, data 2, data 3]), every rebuilt byte against the oracle's
    decode and against the original chunk."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 65536, 250
    rng = np.random.default_rng(0xC0F160)
    data = _rand(rng, B, k, L)  # 1,000 chunks
    enc = oracle.Encoder(k, m)
    want = np.stack([np.stack(enc.encode([data[s, j] for j in range(k)])) for s in range(B)])
    c = RSCoder(k, m)
    stripe = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
    stripe[:, :k] = _to(dev, data)
    encode_batch(c, stripe[:, :k], stripe[:, k:])
    assert np.array_equal(stripe[:, k:].cpu().numpy(), want)
    host_par = np.empty((B, m, L), np.uint8)
    for s in range(B):
        c.encode_host([data[s, j].ctypes.data for j in range(k)], [host_par[s, r].ctypes.data for r in range(m)], L)
    assert np.array_equal(host_par, want)
    surv = [4, 1, 2, 3]
    out = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
    decode_batch(c, stripe, surv, [0], out, inputs_by_unit=True)
    got = out[:, 0].cpu().numpy()
    for s in range(B):
        rc, ref = oracle.decode(k, m, [want[s, 0], data[s, 1], data[s, 2], data[s, 3]], surv, [0])
        assert rc == 0 and np.array_equal(got[s], ref[0]), s
    assert np.array_equal(got, data[:, 0])
