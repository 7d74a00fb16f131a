"""BASELINE configs[3] and configs[4] at their full sizes, in the exact HBM
layouts bench.py measures (bench.alloc_stripes / layout_for), checked two ways:
every stripe by a size-independent property (decode(encode(x)) == x, compat
zero rows), and sampled stripes (first, middle, last, seeded random) byte for
byte against the CPU oracle on the WHOLE chunk, reassembled from 64 KiB tiles
where the layout tiles it.

configs[3]: RS(6,4) encode + decode (erase 0), 1 KiB x 262,144 + 4 KiB x
65,536 + 1 MiB x 256 stripes (1 GiB of data per class).
configs[4]: RS(12,8), 256 KiB x 512 stripes, every 2-erasure pattern (66) in
COMPAT mode (the drop-in's default, EC/erasure_coder.c:261-281), decoded from
the first 8 survivors; ELECT's own {0,1} pattern is the bench's.
"""
import importlib.util
import itertools
import os
import types

import numpy as np
import pytest
import torch

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench():
    spec = importlib.util.spec_from_file_location("bench_layouts", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args():
    return types.SimpleNamespace(layout="auto", no_tiles=False)


def _sample(B, seed, extra=5):
    rng = np.random.default_rng(seed)
    picks = {0, B // 2, B - 1} | {int(x) for x in rng.integers(0, B, extra)}
    return sorted(picks)


def _chunk(view, Bc, B, s, unit):
    """Unit `unit` of logical stripe s as one array, from the coding view
    (tiled layouts code B*t stripes of 64 KiB: stripe s is rows s*t .. s*t+t-1)."""
    t = Bc // B
    return np.concatenate([view[s * t + i, unit].cpu().numpy() for i in range(t)])


def test_mixed_config_full_size(dev, oracle):
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    bench = _bench()
    k, m = 4, 2
    coder = RSCoder(k, m)
    enc = oracle.Encoder(k, m)
    for L, B in ((1024, 262144), (4096, 65536), (1 << 20, 256)):
        g = torch.Generator(device=dev).manual_seed(L)
        view, Bc, Lc = bench.alloc_stripes(_args(), B, L, k, m, dev, generator=g)
        encode_batch(coder, view[:, :k], view[:, k:])
        out = torch.empty((Bc, 1, Lc), dtype=torch.uint8, device=dev)
        decode_batch(coder, view, [1, 2, 3, 4], [0], out, inputs_by_unit=True)
        assert torch.equal(out[:, 0], view[:, 0]), L  # every stripe
        for s in _sample(B, L):
            units = [_chunk(view, Bc, B, s, j) for j in range(k + m)]
            assert all(u.size == L for u in units)
            want = enc.encode(units[:k])
            assert np.array_equal(units[k], want[0]) and np.array_equal(units[k + 1], want[1]), (L, s)
            rc, rebuilt = oracle.decode(k, m, units[1:k + 1], [1, 2, 3, 4], [0])
            t = Bc // B
            got = np.concatenate([out[s * t + i, 0].cpu().numpy() for i in range(t)])
            assert rc == 0 and np.array_equal(got, rebuilt[0]), (L, s)
        del view, out
        torch.cuda.empty_cache()


def test_rs12_config_full_size_compat_every_pattern(dev, oracle):
    from elect_amd import _lib
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    bench = _bench()
    k, m, L, B = 8, 4, 262144, 512
    coder = RSCoder(k, m)
    g = torch.Generator(device=dev).manual_seed(12)
    view, Bc, Lc = bench.alloc_stripes(_args(), B, L, k, m, dev, generator=g)
    assert (Bc, Lc) == (B * 4, 65536)  # the bench's 64 KiB tiles
    encode_batch(coder, view[:, :k], view[:, k:])
    enc = oracle.Encoder(k, m)
    samples = _sample(B, 12, extra=2)
    host = {s: [_chunk(view, Bc, B, s, j) for j in range(k + m)] for s in samples}
    for s, units in host.items():
        want = enc.encode(units[:k])
        assert all(np.array_equal(units[k + r], want[r]) for r in range(m)), s
    out = torch.empty((Bc, 2, Lc), dtype=torch.uint8, device=dev)
    zero = torch.zeros((), dtype=torch.uint8, device=dev)
    pats = [list(p) for p in itertools.combinations(range(k + m), 2)]
    pats += [[9, 0], [11, 3], [5, 1]]  # list order matters in compat mode
    for n, erased in enumerate(pats):
        surv = [i for i in range(k + m) if i not in erased][:k]
        out.fill_(0xA5)
        st = decode_batch(coder, view, surv, erased, out, mode=_lib.DECODE_COMPAT, inputs_by_unit=True)
        assert st == _lib.OK
        ned = sum(e < k for e in erased)
        for r, e in enumerate(erased):  # every stripe: rows < nED rebuilt, the rest zero
            if r < ned:
                assert torch.equal(out[:, r], view[:, e]), (erased, r)
            else:
                assert torch.equal(out[:, r], zero.expand_as(out[:, r])), (erased, r)
        for s in (samples[n % len(samples)], samples[-1]):  # the whole 256 KiB chunks vs the oracle
            rc, want = oracle.decode(k, m, [host[s][i] for i in surv], surv, erased, False)
            assert rc == 0
            for r in range(2):
                got = np.concatenate([out[s * 4 + i, r].cpu().numpy() for i in range(4)])
                assert np.array_equal(got, want[r]), (erased, s, r)
