"""Decode access-pattern probe (dev tooling): which survivor columns a
single-erasure RS(6,4) decode reads, and where it writes, in the [B][6][L]
stripe layout, timed through the product library (ELECT_EC_LIB selects an A/B
build).  Median of 25 launches per case, cases interleaved over 3 rounds.

  python tools/tune/decode_pattern.py [L] [B]
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from elect_amd import _lib  # noqa: E402
from elect_amd.batch import decode_batch, encode_batch  # noqa: E402
from elect_amd.coder import RSCoder  # noqa: E402


def main():
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda", 0)
    k, m = 4, 2
    c = RSCoder(k, m)
    stripe = torch.randint(0, 256, (B, k + m, L), dtype=torch.uint8, device=dev)
    encode_batch(c, stripe[:, :k], stripe[:, k:])
    sep = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
    big = torch.empty((B, 2, L), dtype=torch.uint8, device=dev)
    cases = {
        # name: (survivors, erased, mode, output tensor, outputs_by_unit)
        "erase0 surv1234 ->sep": ([1, 2, 3, 4], [0], _lib.DECODE_COMPAT, sep, False),
        "erase4 surv0123 ->sep (strict)": ([0, 1, 2, 3], [4], _lib.DECODE_STRICT, sep, False),
        "erase5 surv0123 ->sep (strict)": ([0, 1, 2, 3], [5], _lib.DECODE_STRICT, sep, False),
        "erase0 surv1234 ->[B][2][L] row0": ([1, 2, 3, 4], [0], _lib.DECODE_COMPAT, big, False),
        "erase3 surv0124 ->sep": ([0, 1, 2, 4], [3], _lib.DECODE_COMPAT, sep, False),
    }
    alg = B * (k + 1) * L
    res = {n: [] for n in cases}
    for _ in range(3):
        for name, (surv, er, mode, out, by_unit) in cases.items():
            ts = []
            for i in range(30):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                decode_batch(c, stripe, surv, er, out, mode=mode, inputs_by_unit=True, outputs_by_unit=by_unit)
                e1.record()
                e1.synchronize()
                if i >= 5:
                    ts.append(e0.elapsed_time(e1))
            res[name].append(statistics.median(ts))
    want = stripe[:, 0].clone()
    decode_batch(c, stripe, [1, 2, 3, 4], [0], sep, inputs_by_unit=True)
    ok = torch.equal(sep[:, 0], want)
    print(f"decode pattern probe L={L} B={B} lib={os.environ.get('ELECT_EC_LIB') or 'in-tree'} verified={ok}")
    for name, v in res.items():
        ms = statistics.median(v)
        print(f"  {name:36s} {ms:.4f} ms  {alg / (ms * 1e-3) / 8e12 * 100:5.1f}% of 8 TB/s")


if __name__ == "__main__":
    main()
