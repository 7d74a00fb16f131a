"""Tiled units (include/elect_ec.h, elect_ec_*_batch_tiled): a unit of L bytes
stored as ceil(L/tile) tiles, each tile coded as a stripe of its own, must give
the bytes of coding the unit whole: parity, parity hashCode() (per STRIPE, over
L bytes), the parity update and the degraded-read decode, with content lengths
per stripe, garbage past every content end and in the pad of the last tile
(never read), and zeros written to the output pad.  Checked against the CPU
oracle on zero-filled units (ECMessageVerbHandler.java:292-310) and against the
untiled _ex calls.  ELECT's codeLength 4,404,020 B in 64 KiB tiles (T = 68) is
the case bench.py --config flows measures."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [  # (k, m, L, tile, B): ELECT's size, odd sizes, hash add mode (< 64 segments per unit), T = 1
    (4, 2, 4404020, 65536, 3),
    (4, 2, 300001, 65536, 5),
    (8, 4, 70000, 4096, 4),
    (3, 2, 1000, 48, 6),
    (4, 2, 200, 256, 7),
    (4, 2, 65536, 65536, 4),
    (6, 3, 131072 + 16, 65536, 3),
]


def _tiled(dev, units, tile):
    """[B, n, L] host bytes -> device [B*T, n, tile] view of a [B][T][n][tile] block, pad = 0xEE."""
    B, n, L = units.shape
    T = max(1, -(-L // tile))
    pad = np.full((B, n, T * tile), 0xEE, np.uint8)
    pad[:, :, :L] = units
    blk = np.ascontiguousarray(pad.reshape(B, n, T, tile).transpose(0, 2, 1, 3))
    return torch.from_numpy(blk).to(dev).view(B * T, n, tile), T


def _untile(view, B, L):
    rows, n, tile = view.shape
    T = rows // B
    h = view.cpu().numpy().reshape(B, T, n, tile).transpose(0, 2, 1, 3).reshape(B, n, T * tile)
    return h[:, :, :L], h[:, :, L:]


def _garbage_past(units, lens):
    g = units.copy()
    for s in range(units.shape[0]):
        for j in range(units.shape[1]):
            g[s, j, lens[s, j]:] = 0xFF
    return g


def _zero_past(units, lens):
    z = units.copy()
    for s in range(units.shape[0]):
        for j in range(units.shape[1]):
            z[s, j, lens[s, j]:] = 0
    return z


@pytest.mark.parametrize("k,m,L,tile,B", CASES)
def test_tiled_encode_hash_equals_whole_unit(dev, oracle, k, m, L, tile, B):
    from elect_amd.batch import encode_batch_ex, encode_batch_tiled
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(L + tile + k)
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    lens = rng.integers(0, L + 1, (B, k)).astype(np.int32)
    lens[0] = L
    lens[-1, 0] = 0
    if B > 2:
        lens[1] = [min(L, tile * (j + 1) + j) for j in range(k)]  # content ends at / near tile edges
    stripe = np.concatenate([_garbage_past(data, lens), np.full((B, m, L), 0x77, np.uint8)], axis=1)
    view, T = _tiled(dev, stripe, tile)
    d_lens = torch.from_numpy(lens).to(dev)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_batch_tiled(coder, view[:, :k], view[:, k:], L, lengths=d_lens, hashes=hashes)
    got, pad = _untile(view, B, L)
    want_in = _zero_past(data, lens)
    h = hashes.cpu().numpy()
    for s in range(B):
        want = enc.encode([want_in[s, j] for j in range(k)])
        for r in range(m):
            assert np.array_equal(got[s, k + r], want[r]), (s, r)
            assert int(h[s, r]) == oracle.java_hashcode(want[r]), (s, r)
    assert not pad[:, k:].any()  # outputs in the last tile's pad are written as zero
    assert (pad[:, :k] == 0xEE).all()  # inputs there untouched
    # the same bytes as the untiled call on a contiguous [B][k+m][L] batch
    flat = torch.from_numpy(np.concatenate([_garbage_past(data, lens), np.zeros((B, m, L), np.uint8)], 1)).to(dev)
    h2 = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_batch_ex(coder, flat[:, :k], flat[:, k:], lengths=d_lens, hashes=h2)
    assert np.array_equal(flat[:, k:].cpu().numpy(), got[:, k:])
    assert torch.equal(h2, hashes)
    # full units, no lengths, no hashes (the plain tiled encode)
    full = np.concatenate([data, np.zeros((B, m, L), np.uint8)], axis=1)
    v2, _ = _tiled(dev, full, tile)
    encode_batch_tiled(coder, v2[:, :k], v2[:, k:], L)
    g2, _ = _untile(v2, B, L)
    for s in (0, B - 1):
        want = enc.encode([data[s, j] for j in range(k)])
        assert all(np.array_equal(g2[s, k + r], want[r]) for r in range(m))


@pytest.mark.parametrize("k,m,L,tile,B", CASES[:4])
def test_tiled_update_and_decode_equal_whole_unit(dev, oracle, k, m, L, tile, B):
    from elect_amd.batch import decode_batch_tiled, encode_update_batch_tiled
    from elect_amd.coder import RSCoder
    rng = np.random.default_rng(3 * L + tile)
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    par = np.stack([np.stack(enc.encode([data[s, j] for j in range(k)])) for s in range(B)])
    t = 1 % k
    new = rng.integers(0, 256, (B, L), dtype=np.uint8)
    ulens = rng.integers(0, L + 1, (B, 2)).astype(np.int32)
    ulens[0] = L
    old_g = _garbage_past(data[:, t:t + 1], ulens[:, :1])[:, 0]
    new_g = _garbage_past(new[:, None], ulens[:, 1:])[:, 0]
    blk = np.concatenate([old_g[:, None], new_g[:, None], par], axis=1)  # [old, new, P...] per stripe
    view, T = _tiled(dev, blk, tile)
    hashes = torch.zeros((B, m), dtype=torch.int32, device=dev)
    encode_update_batch_tiled(coder, t, view[:, 0], view[:, 1], view[:, 2:], view[:, 2:], L,
                              lengths=torch.from_numpy(ulens).to(dev), hashes=hashes)  # in place
    got, pad = _untile(view, B, L)
    old_z = _zero_past(data[:, t:t + 1], ulens[:, :1])[:, 0]
    new_z = _zero_past(new[:, None], ulens[:, 1:])[:, 0]
    h = hashes.cpu().numpy()
    for s in range(B):
        want = enc.encode_update([old_z[s], new_z[s]] + [par[s, r] for r in range(m)], t)
        for r in range(m):
            assert np.array_equal(got[s, 2 + r], want[r]), (s, r)
            assert int(h[s, r]) == oracle.java_hashcode(want[r])
    assert not pad[:, 2:].any()
    # degraded read: rebuild unit t from the other data units + parity 0, survivors zero padded
    surv = [j for j in range(k) if j != t] + [k]
    units = np.concatenate([data, par], axis=1)
    dlens = rng.integers(0, L + 1, (B, k)).astype(np.int32)
    dlens[0] = L
    ins = _garbage_past(units[:, surv], dlens)
    iview, _ = _tiled(dev, ins, tile)
    out = torch.full((B * T, 1, tile), 0x11, dtype=torch.uint8, device=dev)
    decode_batch_tiled(coder, iview, surv, [t], out, L, lengths=torch.from_numpy(dlens).to(dev))
    rebuilt, opad = _untile(out, B, L)
    zin = _zero_past(units[:, surv], dlens)
    for s in range(B):
        rc, want = oracle.decode(k, m, [zin[s, i] for i in range(k)], surv, [t])
        assert rc == 0 and np.array_equal(rebuilt[s, 0], want[0]), s
    assert not opad.any()


def test_tiled_rejects_bad_geometry(dev):
    from elect_amd import _lib
    from elect_amd.batch import encode_batch_tiled
    from elect_amd.coder import RSCoder
    coder = RSCoder(4, 2)
    v = torch.zeros((6, 6, 40), dtype=torch.uint8, device=dev)  # tile 40: not a multiple of 16
    with pytest.raises(_lib.ECInvalidArgument):
        encode_batch_tiled(coder, v[:, :4], v[:, 4:], 100)
    v = torch.zeros((5, 6, 64), dtype=torch.uint8, device=dev)  # 5 rows, T = 2
    with pytest.raises(ValueError):
        encode_batch_tiled(coder, v[:, :4], v[:, 4:], 100)
