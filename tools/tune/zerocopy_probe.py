#!/usr/bin/env python3
"""Zero-copy probe for the JNI host path (dev tooling, GPU box).

Today a host-memory call copies its pageable units into a pinned arena, DMAs
them over, codes, DMAs the parity back and copies it out: ~4.5 host-DRAM bytes
per data byte.  The alternative measured here: page-lock the caller's own
buffers (hipHostRegister), let the kernel read the data units and write the
parity units over PCIe directly, unregister.  Per call: register cost, kernel
time, unregister cost; then the rate with 1 / 16 / 64 concurrent callers,
against the product's host path (elect_ec_encode, batching on) in the same
process.  RS(6,4), ELECT's codeLength 4,404,020 B."""
import ctypes
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from elect_amd import _lib  # noqa: E402
from elect_amd.coder import RSCoder  # noqa: E402
from oracle import ec_oracle  # noqa: E402  (checker only)

GIB = float(1 << 30)
torch.cuda.init()
hip = ctypes.CDLL("libamdhip64.so.7")  # the runtime torch already loaded (same soname)
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipHostRegister.argtypes = [vp, sz, ctypes.c_uint]
hip.hipHostUnregister.argtypes = [vp]
hip.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(vp), vp, ctypes.c_uint]
hip.hipStreamCreateWithFlags.argtypes = [ctypes.POINTER(vp), ctypes.c_uint]
hip.hipStreamSynchronize.argtypes = [vp]
hip.hipSetDevice.argtypes = [ctypes.c_int]

k, m, L = 4, 2, int(os.environ.get("ZC_LEN", 4404020))
coder = RSCoder(k, m)
coef = np.ascontiguousarray(ec_oracle.cauchy_matrix(k, m)[k:], np.uint8)


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


class Caller:
    def __init__(self, seed):
        rng = np.random.default_rng(seed)
        self.d = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
        self.p = [np.zeros(L, np.uint8) for _ in range(m)]
        self.stream = vp()
        ok(hip.hipStreamCreateWithFlags(ctypes.byref(self.stream), 1), "stream")
        self.t = {"reg": 0.0, "kern": 0.0, "unreg": 0.0}

    def zero_copy(self, register=True):
        bufs = self.d + self.p
        t0 = time.perf_counter()
        if register:
            for b in bufs:
                ok(hip.hipHostRegister(b.ctypes.data, L, 0), "register")
        dptr = []
        for b in bufs:
            q = vp()
            ok(hip.hipHostGetDevicePointer(ctypes.byref(q), b.ctypes.data, 0), "devptr")
            dptr.append(q.value)
        t1 = time.perf_counter()
        src = (_lib.ColumnT * k)(*[_lib.ColumnT(x, 0) for x in dptr[:k]])
        dst = (_lib.ColumnT * m)(*[_lib.ColumnT(x, 0) for x in dptr[k:]])
        _lib.check(_lib.lib.elect_ec_apply_batch(coef.ctypes.data_as(_lib._u8p), m, k, L, 1, src, dst,
                                                 self.stream.value), "apply")
        ok(hip.hipStreamSynchronize(self.stream), "sync")
        t2 = time.perf_counter()
        if register:
            for b in bufs:
                ok(hip.hipHostUnregister(b.ctypes.data), "unregister")
        t3 = time.perf_counter()
        self.t["reg"] += t1 - t0
        self.t["kern"] += t2 - t1
        self.t["unreg"] += t3 - t2

    def product(self):
        coder.encode_host([x.ctypes.data for x in self.d], [x.ctypes.data for x in self.p], L)


def run(T, calls, mode):
    callers = [Caller(s) for s in range(T)]
    if mode == "registered":  # buffers stay page-locked: the kernel's PCIe rate alone
        for c in callers:
            for b in c.d + c.p:
                ok(hip.hipHostRegister(b.ctypes.data, L, 0), "register")

    def work(c):
        ok(hip.hipSetDevice(0), "setdevice")
        for _ in range(calls):
            if mode == "product":
                c.product()
            else:
                c.zero_copy(register=(mode == "zerocopy"))

    work(callers[0])  # warm
    for c in callers:
        c.t = {"reg": 0.0, "kern": 0.0, "unreg": 0.0}
    th = [threading.Thread(target=work, args=(c,)) for c in callers]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    dt = time.perf_counter() - t0
    want = ec_oracle.Encoder(k, m).encode(callers[-1].d)
    good = all(np.array_equal(a, b) for a, b in zip(callers[-1].p, want))
    n = T * calls
    per = {key: round(sum(c.t[key] for c in callers) / n * 1e3, 3) for key in ("reg", "kern", "unreg")}
    print(f"{mode:10s} T={T:3d} calls={calls}: {n * k * L / dt / GIB:7.2f} GiB/s  per call ms {per}  verified={good}",
          flush=True)
    if mode == "registered":
        for c in callers:
            for b in c.d + c.p:
                hip.hipHostUnregister(b.ctypes.data)


if __name__ == "__main__":
    for T in [int(x) for x in os.environ.get("ZC_THREADS", "1 16 64").split()]:
        calls = max(4, 256 // T)
        for mode in os.environ.get("ZC_MODES", "product zerocopy registered").split():
            run(T, calls, mode)
