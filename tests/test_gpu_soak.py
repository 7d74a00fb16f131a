"""Soak: the device batch path over and over, every iteration verified.

For ELECT_EC_SOAK_SECONDS of wall time (default 8), cycles through the layouts
bench.py measures (stripe-major 64 KiB, unit-major 1 KiB and 4 KiB, 64 KiB
tiles of 1 MiB, unit-major with a column skew) and codes (RS(6,4) erasing
unit 0, 2 or 3; RS(12,8) erasing {0, 1}).  Each iteration draws fresh random
data, encodes, decodes the erased units into a buffer pre-filled with a
sentinel, and checks decode == data on every stripe (a size-independent
property); every 8th iteration also compares two whole coding stripes' parity
with the CPU oracle."""
import importlib.util
import os
import time
import types

import numpy as np
import pytest
import torch

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu

CASES = [  # (k, m, L, B, layout, column skew, erased)
    (4, 2, 65536, 2048, "stripe", 0, [0]),
    (4, 2, 65536, 2048, "stripe", 0, [3]),
    (4, 2, 1024, 131072, "unit", 0, [0]),
    (4, 2, 4096, 32768, "unit", 0, [2]),
    (4, 2, 1 << 20, 128, "tiled", 0, [0]),
    (4, 2, 1024, 131072, "unit", 69632, [0]),
    (8, 4, 262144, 256, "tiled", 0, [0, 1]),
]


def _bench():
    spec = importlib.util.spec_from_file_location("bench_soak", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_soak_every_iteration_verified(dev, oracle):
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    bench = _bench()
    seconds = float(os.environ.get("ELECT_EC_SOAK_SECONDS", "8"))
    coders = {}
    fails = []
    it = 0
    t0 = last = time.perf_counter()
    while time.perf_counter() - t0 < seconds or it < len(CASES):
        if time.perf_counter() - last > 20:  # a long soak reports progress (a silent run looks hung)
            last = time.perf_counter()
            print(f"soak: {it} iterations, {last - t0:.0f} s, {len(fails)} failures", flush=True)
        k, m, L, B, layout, skew, era = CASES[it % len(CASES)]
        coder = coders.setdefault((k, m), RSCoder(k, m))
        args = types.SimpleNamespace(layout=layout, no_tiles=False, column_skew=skew)
        st, Bc, Lc = bench.alloc_stripes(args, B, L, k, m, dev)
        encode_batch(coder, st[:, :k], st[:, k:])
        surv = [j for j in range(k + m) if j not in era][:k]
        out = torch.full((Bc, len(era), Lc), 0xA5, dtype=torch.uint8, device=dev)
        decode_batch(coder, st, surv, era, out, inputs_by_unit=True)
        for i, e in enumerate(era):
            bad = (out[:, i] != st[:, e]).any(dim=1)
            if bool(bad.any()):
                fails.append((it, k, m, L, layout, skew, e, int(bad.sum()), int(bad.nonzero()[0])))
        if it % 8 == 0:
            enc = oracle.Encoder(k, m)
            for s in (0, Bc - 1):
                want = enc.encode([st[s, j].cpu().numpy() for j in range(k)])
                for r in range(m):
                    if not np.array_equal(st[s, k + r].cpu().numpy(), want[r]):
                        fails.append((it, k, m, L, layout, skew, "parity", s, r))
        it += 1
        del st, out
    torch.cuda.synchronize()
    print(f"soak: {it} iterations in {time.perf_counter() - t0:.1f} s")
    assert not fails, fails[:10]
