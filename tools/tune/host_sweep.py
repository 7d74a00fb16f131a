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


def _cpulist(spec):
    cpus = set()
    for part in spec.strip().split(","):
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


if os.environ.get("HOST_NUMA"):  # run (and first-touch pinned memory) on one NUMA node's CPUs
    node = os.environ["HOST_NUMA"]
    os.sched_setaffinity(0, _cpulist(open(f"/sys/devices/system/node/node{node}/cpulist").read()))
    print(f"affinity: NUMA node {node}", flush=True)
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


def staged_pipeline(chunk, ring, total_stripes=4096):
    """Three streams (H2D, compute, D2H) over a ring of device buffers, chained
    by events: the copy engines of both directions stay busy continuously."""
    nch = total_stripes // chunk
    h_data = torch.randint(0, 256, (total_stripes, k, L), dtype=torch.uint8).pin_memory()
    h_par = torch.empty((total_stripes, m, L), dtype=torch.uint8).pin_memory()
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    dd = [torch.empty((chunk, k, L), dtype=torch.uint8, device=dev) for _ in range(ring)]
    dp = [torch.empty((chunk, m, L), dtype=torch.uint8, device=dev) for _ in range(ring)]

    def run():
        ev_in = [None] * nch
        ev_cmp = [None] * nch
        ev_out = [None] * nch
        for c in range(nch):
            r = c % ring
            with torch.cuda.stream(s_in):
                if c >= ring:
                    s_in.wait_event(ev_cmp[c - ring])  # buffer r's data consumed
                dd[r].copy_(h_data[c * chunk:(c + 1) * chunk], non_blocking=True)
                ev_in[c] = torch.cuda.Event()
                ev_in[c].record(s_in)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(ev_in[c])
                if c >= ring:
                    s_cmp.wait_event(ev_out[c - ring])  # buffer r's parity drained
                encode_batch(coder, dd[r], dp[r], stream=s_cmp)
                ev_cmp[c] = torch.cuda.Event()
                ev_cmp[c].record(s_cmp)
            with torch.cuda.stream(s_out):
                s_out.wait_event(ev_cmp[c])
                h_par[c * chunk:(c + 1) * chunk].copy_(dp[r], non_blocking=True)
                ev_out[c] = torch.cuda.Event()
                ev_out[c].record(s_out)
        torch.cuda.synchronize()

    run()
    t0 = time.perf_counter()
    run()
    run()
    dt = time.perf_counter() - t0
    ref = torch.empty((chunk, m, L), dtype=torch.uint8, device=dev)
    encode_batch(coder, h_data[-chunk:].to(dev), ref)
    assert torch.equal(ref.cpu(), h_par[-chunk:]), "staged pipeline parity mismatch"
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
    if "copysizes" in sys.argv:  # raw pinned copy rate by transfer size, each direction alone and both
        big = 1 << 30
        h = torch.empty(big, dtype=torch.uint8).pin_memory()
        h2 = torch.empty(big, dtype=torch.uint8).pin_memory()
        d = torch.empty(big, dtype=torch.uint8, device=dev)
        d2 = torch.empty(big, dtype=torch.uint8, device=dev)
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for mib in (1, 2, 4, 8, 12, 16, 24, 32, 48, 64):
            n = mib << 20
            cnt = big // n
            res = []
            for mode in ("H2D", "D2H", "both"):
                for warm in (0, 1):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for i in range(cnt):
                        if mode in ("H2D", "both"):
                            with torch.cuda.stream(s1):
                                d[i * n:(i + 1) * n].copy_(h[i * n:(i + 1) * n], non_blocking=True)
                        if mode in ("D2H", "both"):
                            with torch.cuda.stream(s2):
                                h2[i * n:(i + 1) * n].copy_(d2[i * n:(i + 1) * n], non_blocking=True)
                    torch.cuda.synchronize()
                    dt = time.perf_counter() - t0
                res.append(f"{mode} {(2 if mode == 'both' else 1) * big / dt / 1e9:.1f}")
            print(f"copy {mib:3d} MiB: " + "  ".join(res) + " GB/s", flush=True)
        sys.exit(0)
    if "staged" in sys.argv:
        pcie()
        for ch in (16, 64, 128):
            for ring in (3,):
                print(f"staged pipeline chunk={ch} stripes ({ch * k * L >> 20} MiB data) ring={ring}: "
                      f"{staged_pipeline(ch, ring):.2f} GiB/s data", flush=True)
        sys.exit(0)
    pcie()
    for ns in (1, 2, 3, 4):
        for ch in (32, 128, 512):
            print(f"pinned pipeline streams={ns} chunk={ch} stripes ({ch * k * L >> 20} MiB data): "
                  f"{pinned_pipeline(ns, ch):.2f} GiB/s data", flush=True)
    for t in (1, 2, 4, 8, 16, 32):
        print(f"pageable JNI path threads={t}: {pageable(t):.2f} GiB/s data", flush=True)
