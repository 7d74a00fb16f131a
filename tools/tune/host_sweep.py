#!/usr/bin/env python3
"""Host-inclusive sweep (dev tooling): PCIe ceilings, the pinned H2D -> encode
-> D2H pipeline over stream counts and transfer sizes, and the JNI-style
pageable path over caller thread counts.  Prints one line per variant."""
import os
import sys
import threading
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from elect_amd.batch import encode_batch  # noqa: E402
from elect_amd.coder import RSCoder  # noqa: E402

GIB = float(1 << 30)
dev = torch.device("cuda:0")
k, m, L = 4, 2, 65536
coder = RSCoder(k, m)


def pcie():
    n = 1 << 30
    h = torch.empty(n, dtype=torch.uint8).pin_memory()
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    for name, fn in (("H2D", lambda: d.copy_(h, non_blocking=True)),
                     ("D2H", lambda: h.copy_(d, non_blocking=True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        print(f"pinned {name} 1 GiB: {3 * n / (time.perf_counter() - t0) / 1e9:.1f} GB/s", flush=True)
    # both directions at once on two streams
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
    d2 = torch.empty(n, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        with torch.cuda.stream(s1):
            d.copy_(h, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    print(f"pinned H2D+D2H concurrently: {6 * n / (time.perf_counter() - t0) / 1e9:.1f} GB/s total", flush=True)


def pinned_pipeline(nstreams, chunk, total_stripes=2048):
    nch = total_stripes // chunk
    h_data = torch.randint(0, 256, (total_stripes, k, L), dtype=torch.uint8).pin_memory()
    h_par = torch.empty((total_stripes, m, L), dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream() for _ in range(nstreams)]
    dd = [torch.empty((chunk, k, L), dtype=torch.uint8, device=dev) for _ in range(nstreams)]
    dp = [torch.empty((chunk, m, L), dtype=torch.uint8, device=dev) for _ in range(nstreams)]

    def run():
        for c in range(nch):
            s = c % nstreams
            with torch.cuda.stream(streams[s]):
                dd[s].copy_(h_data[c * chunk:(c + 1) * chunk], non_blocking=True)
                encode_batch(coder, dd[s], dp[s], stream=streams[s])
                h_par[c * chunk:(c + 1) * chunk].copy_(dp[s], non_blocking=True)
        torch.cuda.synchronize()

    run()
    t0 = time.perf_counter()
    run()
    run()
    dt = time.perf_counter() - t0
    return 2 * total_stripes * k * L / dt / GIB


def pageable(threads, Lc=4404020, calls=8):
    bufs = []
    for t in range(threads):
        d = [np.random.default_rng(t * 8 + j).integers(0, 256, Lc, dtype=np.uint8) for j in range(k)]
        p = [np.empty(Lc, np.uint8) for _ in range(m)]
        bufs.append(([x.ctypes.data for x in d], [x.ctypes.data for x in p], d, p))

    def worker(t, n):
        da, pa = bufs[t][0], bufs[t][1]
        for _ in range(n):
            coder.encode_host(da, pa, Lc)

    def run(n):
        th = [threading.Thread(target=worker, args=(t, n)) for t in range(threads)]
        [x.start() for x in th]
        [x.join() for x in th]

    run(1)
    t0 = time.perf_counter()
    run(calls)
    return threads * calls * k * Lc / (time.perf_counter() - t0) / GIB


if __name__ == "__main__":
    pcie()
    for ns in (1, 2, 3, 4):
        for ch in (32, 128, 512):
            print(f"pinned pipeline streams={ns} chunk={ch} stripes ({ch * k * L >> 20} MiB data): "
                  f"{pinned_pipeline(ns, ch):.2f} GiB/s data", flush=True)
    for t in (1, 2, 4, 8, 16, 32):
        print(f"pageable JNI path threads={t}: {pageable(t):.2f} GiB/s data", flush=True)
