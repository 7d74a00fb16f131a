#!/usr/bin/env python3
"""bench.py — device-resident RS(6,4) encode+decode throughput on MI355X.

Workload (BASELINE.json configs[1] + configs[2], the metric's "encode+decode"):
one step = RS(6,4) encode of B=4096 stripes x 64 KiB chunks (1 GiB of data per
GPU) followed by single-erasure decode of the same batch (data shard 0 lost,
survivors {1,2,3,4}).  Stripes are independent, so with N GPUs every rank codes
its own batch (weak scaling, no collective on the data path).

value = data bytes coded by all ranks (k*L per stripe per operation) / the
slowest rank's time, in GiB/s.  roofline = the encode kernel (dominant launch):
algorithmic bytes (k+m)*L*B per launch / its mean HIP-event duration, against
the 8.0 TB/s HBM3E peak.  The timed steps issue their launches only; the
per-launch events time the same launches in the steps right after (split_pass),
since each event record holds the next launch back ~4 us.  cpu_baseline = the oracle's ISA-L-algorithm SIMD path
on the host cores, rank 0 only (test infrastructure, not the product path).
sizes = the same step and timing at the north star's other chunk sizes (1 KiB,
1 MiB; 1 GiB of data per rank each) next to the 64 KiB line, so every
--gpus N run reports all three.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--chunk BYTES] [--stripes B]

With --gpus N > 1 and no launcher in the environment (no WORLD_SIZE), bench.py
starts N rank processes itself under torch.distributed.run; under a launcher
it refuses to run unless WORLD_SIZE == N.  Ranks talk only over gloo (barrier,
max over ranks, per-rank records); no RCCL communicator is created.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak, decimal GB/s (MI355X_MICROARCH.md)
GIB = float(1 << 30)

HIP_EVENT_DISABLE_SYSTEM_FENCE = 0x20000000  # hip_runtime_api.h
EVENT_RELEASE = {"device": HIP_EVENT_DISABLE_SYSTEM_FENCE, "system": 0}
event_release = "device"  # set from --event-release in main()


class Event:
    """A timing HIP event on the stream the kernels run on, as Event()
    but recorded with a device-scope release by default.  torch's timing events release to system
    scope: every record writes back and invalidates the L2 before the next kernel may start, and
    bench.py records three per step to split encode from decode.  That cost the headline ~6 us a
    step (1.4 %) against the same launches with no events (tools/tune/gap_probe.py,
    profiles/r04/event_release_ab.txt).  Nothing on the host reads what the kernels wrote
    between two steps, so the device-scope release is all the timing needs.  The handle comes from
    the HIP runtime torch loaded (one libamdhip64.so.7 per process), so torch's stream handles are
    valid here."""
    _hip = None

    @classmethod
    def hip(cls):
        if cls._hip is None:
            import ctypes
            h = ctypes.CDLL("libamdhip64.so.7")
            h.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            h.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            h.hipEventSynchronize.argtypes = [ctypes.c_void_p]
            h.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._hip = h
        return cls._hip

    def __init__(self):
        import ctypes
        self.h = ctypes.c_void_p()
        rc = self.hip().hipEventCreateWithFlags(ctypes.byref(self.h), EVENT_RELEASE[event_release])
        if rc != 0:
            raise RuntimeError(f"hipEventCreateWithFlags: error {rc}")

    def record(self, stream=None):
        s = (stream if stream is not None else torch.cuda.current_stream()).cuda_stream
        rc = self.hip().hipEventRecord(self.h, s)
        if rc != 0:
            raise RuntimeError(f"hipEventRecord: error {rc}")

    def synchronize(self):
        rc = self.hip().hipEventSynchronize(self.h)
        if rc != 0:
            raise RuntimeError(f"hipEventSynchronize: error {rc}")

    def elapsed_time(self, end: "Event") -> float:
        import ctypes
        ms = ctypes.c_float()
        rc = self.hip().hipEventElapsedTime(ctypes.byref(ms), self.h, end.h)
        if rc != 0:
            raise RuntimeError(f"hipEventElapsedTime: error {rc}")
        return ms.value

    def __del__(self):
        if getattr(self, "h", None) and self._hip is not None:
            self._hip.hipEventDestroy(self.h)
            self.h = None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--k", type=int, default=4)
    ap.add_argument("--m", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--stripes", type=int, default=4096)
    ap.add_argument("--no-tiles", action="store_true",
                    help="layout auto: stripe-major instead of 64 KiB tiles for chunks above 64 KiB")
    ap.add_argument("--layout", choices=("auto", "stripe", "unit", "tiled"), default="auto",
                    help="HBM layout of the stripes ([B][k+m][L] or [k+m][B][L]); headline and mixed. auto: "
                         "unit-major for chunks <= 4 KiB (a stripe-major wave would read and write one "
                         "6 KiB region), stripe-major above")
    ap.add_argument("--column-skew", type=int, default=0,
                    help="unit-major layout experiment: bytes of gap between one column's region and the next's")
    ap.add_argument("--decode-out", choices=("separate", "inplace"), default="separate",
                    help="headline decode target: a separate [B][1][L] buffer, or the erased unit's own slot")
    ap.add_argument("--rotate", type=int, default=4,
                    help="headline and sizes: cycle through N disjoint stripe batches (1 GiB of data each), "
                         "one per step, so that no step finds the previous one's lines in L2 or the 256 MiB "
                         "MALL (DESIGN.md §5)")
    ap.add_argument("--rebuilt-rows", type=int, default=1,
                    help="layout experiment: the separate decode buffer is [B][rows][L], row 0 used")
    ap.add_argument("--unit-gap", type=int, default=0,
                    help="headline layout experiment: bytes of gap after each unit in HBM ([B][k+m][L+gap])")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="target CPU-baseline work time (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host", action="store_true", help="skip the host-inclusive (PCIe) measurement")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the mixed (configs[3]) and RS(12,8) (configs[4]) lines of the headline run")
    ap.add_argument("--settle-ms", type=float, default=100.0,
                    help="run the step untimed for this long before the --warmup steps, so the timed steps see "
                         "the GPU's steady clocks (per-step series: decode runs ~4 points slow for the first "
                         "~20 ms of load, DESIGN.md §5); 0 = off")
    ap.add_argument("--per-step", action="store_true",
                    help="headline: also print every timed step's encode and decode kernel times (diagnostics)")
    ap.add_argument("--rs12-erasures", type=int, default=2, choices=(1, 2, 3, 4),
                    help="rs12: erase units 0..N-1, decode from the next 8 (BASELINE configs[4]: 2)")
    ap.add_argument("--configs-order", default="mixed,rs12",
                    help="headline: the BASELINE configs run after the headline phases, in this order")
    ap.add_argument("--no-sizes", action="store_true",
                    help="headline: skip the 1 KiB / 1 MiB chunk-size lines (sizes) after the 64 KiB one")
    ap.add_argument("--config", default="headline",
                    choices=["headline", "mixed", "rs12", "hostpath", "update", "padded", "hashed", "flows"],
                    help="headline = the driver's line (BASELINE configs[1]+[2]); mixed = configs[3] "
                         "(1 KiB/4 KiB/1 MiB, 1 GiB per class over all ranks); rs12 = configs[4] "
                         "(RS(12,8) two-erasure decode, 256 KiB, 512 stripes per GPU); hostpath = the "
                         "JNI-style synchronous host-memory encode at ELECT's codeLength")
    ap.add_argument("--threads", type=int, default=16, help="hostpath: concurrent callers")
    ap.add_argument("--batch", type=int, default=1, choices=(0, 1),
                    help="hostpath: cross-thread batching (the library default, 1) or per-thread staging (0)")
    ap.add_argument("--pad-fill", default="random",
                    help="padded: content lengths 'random' (uniform [0, L]) or a fixed fraction of L")
    ap.add_argument("--host-chunk", type=int, default=4404020, help="hostpath: bytes per unit per call")
    ap.add_argument("--host-devices", type=int, default=0,
                    help="hostpath: spread the callers over devices 0..N-1 (elect_ec_set_host_devices, what "
                         "ELECT_EC_DEVICES=all does for ELECT's one JVM per node); 0: the current device only")
    ap.add_argument("--host-seconds", type=float, default=0.0,
                    help="hostpath: repeat the timed calls until at least this much wall time has passed")
    ap.add_argument("--no-hostpath", action="store_true",
                    help="headline: skip the JNI-convention host path over all the job's devices")
    ap.add_argument("--host-numa", choices=("none", "local", "remote"), default="none",
                    help="hostpath: bind the process (callers, their buffers by first touch, the library's "
                         "threads) to the device's NUMA node (local) or another node (remote) before allocating")
    ap.add_argument("--host-alloc", choices=("pageable", "pinned"), default="pageable",
                    help="hostpath: the callers' buffers are ordinary memory (ELECT's ByteBuffer.allocateDirect), or "
                         "elect_ec_host_alloc buffers (page-locked; the batcher then moves them by DMA, no staging "
                         "copies: INTEGRATION.md, host buffers)")
    ap.add_argument("--host-register", type=int, choices=(0, 1), default=None,
                    help="hostpath: ELECT_EC_REGISTER for the run (1: batched callers' pageable units page-locked "
                         "per call, their interior pages moved by DMA; default: the library's default)")
    ap.add_argument("--host-op", choices=("encode", "encode_ex", "decode", "update"), default="encode",
                    help="hostpath: plain encode (the JNI encodeImpl), ELECT's fused encode step "
                         "(encodeExImpl: content = codeLength/1.05, parity hashCodes), the degraded-read "
                         "decode (decodeImpl: rebuild unit 0 from [p0, d1, d2, d3], ECRecovery.java:141) or "
                         "the parity update (encodeUpdateImpl: [old d1, new d1, p0, p1] -> p0', p1' in place, "
                         "ECParityUpdateVerbHandler.java:688)")
    ap.add_argument("--flows-tile", type=int, default=-1,
                    help="flows: tile bytes for the [B][T][k+m][tile] layout (-1: 64 KiB tiles above 64 KiB, "
                         "0: untiled)")
    ap.add_argument("--flows-inplace", action="store_true",
                    help="flows: the update writes the new parity over the old (ELECT writes separate buffers)")
    ap.add_argument("--mixed-group", type=int, default=1, choices=(0, 1),
                    help="mixed: code the size classes through elect_ec_{encode,decode}_batches (one launch "
                         "for all classes each, the default) or one call per class (0)")
    ap.add_argument("--mixed-streams", type=int, default=1,
                    help="mixed: issue the size classes on this many streams (1: one stream, in order)")
    ap.add_argument("--mixed-lanes", type=int, default=1,
                    help="mixed: keep this many disjoint copies of the batch and issue step i's grouped encode + "
                         "decode (copy i %% S) on stream i %% S, so one step's launch tail overlaps the next "
                         "step's ramp-up (independent stripes; 1 = one copy, one stream)")
    ap.add_argument("--mixed-share", type=int, default=0,
                    help="mixed: code rank 0's share of an N-rank partition on this GPU (strong-scaling probe)")
    ap.add_argument("--streams", type=int, default=1,
                    help="headline: issue step i (its batch's encode + decode) on stream i %% S; with "
                         "S > 1 consecutive steps' kernels may overlap at their boundaries")
    ap.add_argument("--graph", action="store_true",
                    help="headline and mixed: capture each step's launches in a HIP graph and replay it")
    ap.add_argument("--event-release", choices=tuple(EVENT_RELEASE), default="device",
                    help="scope of the release the timing events' records make: device (the default) or system "
                         "(torch.cuda.Event's, which writes back and invalidates L2 at every record)")
    ap.add_argument("--launch-check", action="store_true",
                    help="plumbing check without a GPU: start the ranks, run the gloo handshake, print "
                         "one JSON line (tests/test_bench_launch_cpu.py)")
    return ap.parse_args()


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher: run N rank processes under
    torch.distributed.run (rendezvous on 127.0.0.1) as a child and return its exit
    status.  This process never touches the GPU, so nothing exec's from a process
    that has initialised HIP."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *argv]
    return subprocess.run(cmd).returncode


def dist_setup(args):
    from elect_amd import dist
    return dist.setup("cpu" if args.launch_check else "cuda")


def barrier(world):
    from elect_amd import dist
    dist.barrier(world)


def max_over_ranks(x: float, world: int) -> float:
    from elect_amd import dist
    return dist.max_over_ranks(x, world, "cuda")


def pmc_traffic(*kernel_substrs: str):
    """HBM bytes per launch from the newest committed rocprofv3 PMC summary
    (tools/pmc_traffic.py) that has one of the named kernels."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc_traffic*.json")), reverse=True):
        try:
            with open(path) as f:
                d = json.load(f)
        except Exception:
            continue
        for sub in kernel_substrs:
            for name, rec in d.get("kernels", {}).items():
                if sub in name:
                    return rec.get("hbm_bytes_per_launch"), os.path.relpath(path, ROOT)
    return None, None


def host_cpu_info() -> dict:
    """The host cores this process may use: affinity mask, cgroup CPU quota, model."""
    info = {"affinity": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count(), "quota_cores": None,
            "model": None}
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts[0] != "max":
                info["quota_cores"] = round(int(parts[0]) / int(parts[1]), 2)
            elif path.endswith("quota_us") and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    info["quota_cores"] = round(int(parts[0]) / int(f.read()), 2)
            break
        except (OSError, ValueError, IndexError):
            continue
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return info


def cpu_thread_points(info: dict) -> list:
    """Thread counts the CPU baseline sweeps: the cgroup quota, twice it, 64 and the
    whole affinity mask (each at most the mask), so that the reported figure is the
    box's best and not an oversubscribed run (a 16-CPU quota under a 256-CPU mask)."""
    aff = info["affinity"]
    q = math.ceil(info["quota_cores"]) if info.get("quota_cores") else None
    pts = {aff, min(64, aff)}
    if q:
        pts |= {min(q, aff), min(2 * q, aff)}
    return sorted(p for p in pts if p >= 1)


def parse_cpulist(text: str) -> list:
    """'0-3,8,10-11' -> [0, 1, 2, 3, 8, 10, 11] (sysfs cpulist format)."""
    out = []
    for part in text.strip().split(","):
        if not part:
            continue
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


def numa_cpus() -> dict:
    """{node: [cpu, ...]}: the CPUs of this process's affinity mask on each NUMA
    node, one logical CPU per physical core first (SMT siblings after), so that a
    placement of t threads on a node takes t distinct cores while it can."""
    aff = os.sched_getaffinity(0)
    nodes = {}
    for path in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        try:
            with open(os.path.join(path, "cpulist")) as f:
                cpus = [c for c in parse_cpulist(f.read()) if c in aff]
        except (OSError, ValueError):
            continue
        first, later = [], []
        for c in cpus:
            try:
                with open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list") as f:
                    primary = min(parse_cpulist(f.read())) == c
            except (OSError, ValueError):
                primary = True
            (first if primary else later).append(c)
        if cpus:
            nodes[int(path.rsplit("node", 1)[1])] = first + later
    return nodes


def cpu_placements(info: dict) -> list:
    """(name, threads, cpu set or None) points of the CPU baseline sweep: the thread
    counts of cpu_thread_points() unpinned (the scheduler's choice inside the
    affinity mask), and the quota and twice it pinned to one NUMA node's cores (each
    node) and split evenly over two nodes.  A cgroup CPU quota (cpu.max) caps the
    CPU time, not the CPUs: unpinned threads may wander over both sockets, away from
    their pages."""
    pts = [("any", t, None) for t in cpu_thread_points(info)]
    nodes = numa_cpus()
    q = math.ceil(info["quota_cores"]) if info.get("quota_cores") else min(16, info["affinity"])
    for t in sorted({q, 2 * q}):
        for n, cpus in sorted(nodes.items()):
            if len(cpus) >= t:
                pts.append((f"node{n}", t, cpus[:t]))
        if len(nodes) >= 2:
            (n0, c0), (n1, c1) = sorted(nodes.items())[:2]
            if len(c0) >= t // 2 and len(c1) >= t - t // 2:
                pts.append((f"split{n0}+{n1}", t, c0[:t // 2] + c1[:t - t // 2]))
    return pts


def cpu_baseline(args, k, m, L, stripes):
    """Oracle SIMD path (ISA-L's algorithm restated) on the host cores: the same
    encode + single-erasure decode step over the same stripe batch the GPU codes
    (4096 x 64 KiB: 1 GiB of data, 1.75 GiB touched, far beyond any LLC), stripes
    split evenly over the threads.  Thread count and placement are swept
    (cpu_placements: unpinned, pinned to one NUMA node with its pages first
    touched there, split over two nodes) and the best point is the value; then
    the same loop on one thread.  Bounded to about --cpu-seconds of threaded work
    in all."""
    import numpy as np
    from oracle import ec_oracle as orc
    info = host_cpu_info()
    points = cpu_placements(info)
    n = k + m
    base = np.empty((stripes, n, L), np.uint8)
    orc.fill_splitmix(0xE1EC7, base)
    em = orc.cauchy_matrix(k, m)
    enc_coef = em[k:]
    rc, dec_coef = orc.decode_matrix(k, m, list(range(1, k + 1)), [0])
    level = orc.simd_best()
    sstride = n * L
    enc_src = [j * L for j in range(k)]
    enc_dst = [(k + r) * L for r in range(m)]
    dec_src = [j * L for j in range(1, k + 1)]
    home = os.sched_getaffinity(0)

    def loop(buf, out, nthreads, budget, min_reps):
        t, reps = 0.0, 0
        while t < budget or reps < min_reps:
            t += orc.batch_apply(enc_coef, buf, sstride, enc_src, buf, sstride, enc_dst, L, stripes, nthreads, level)
            t += orc.batch_apply(dec_coef, buf, sstride, dec_src, out, L, [0], L, stripes, nthreads, level)
            reps += 1
        return reps, t

    step_bytes = 2 * stripes * k * L
    sweep, ok = {}, True
    node_bufs = {}  # per pinned CPU set: the batch's pages first touched by a thread on those CPUs
    budget = args.cpu_seconds / len(points)
    try:
        for name, t, cpus in points:
            if cpus is None:
                os.sched_setaffinity(0, home)
                buf = base
            else:
                os.sched_setaffinity(0, cpus)  # this thread; the oracle's threads inherit it
                key = tuple(sorted(cpus))
                if key not in node_bufs:
                    node_bufs.clear()  # one copy at a time (1.75 GiB each)
                    b = np.empty_like(base)
                    np.copyto(b, base)
                    node_bufs[key] = b
                buf = node_bufs[key]
            out = np.empty((stripes, 1, L), np.uint8)
            orc.batch_apply(enc_coef, buf, sstride, enc_src, buf, sstride, enc_dst, L, stripes, t, level)  # warm
            reps, tt = loop(buf, out, t, budget, 2)
            sweep[f"{name}:{t}"] = (reps, tt, reps * step_bytes / tt / GIB, name, t)
            ok = ok and np.array_equal(out[:, 0], buf[:, 0])
    finally:
        os.sched_setaffinity(0, home)
        node_bufs.clear()
    assert ok, "CPU baseline decode mismatch"
    best = max(sweep, key=lambda key: sweep[key][2])
    reps, total_t, rate, place, threads = sweep[best]
    out = np.empty((stripes, 1, L), np.uint8)
    reps1, t1 = loop(base, out, 1, args.cpu_seconds * 0.3, 1)  # single-core figure
    # one synchronous call as ELECT makes it, on one core: the degraded-read decode
    # (ECRecovery.java:141; 4 survivors -> 1 unit) and the encode (4 -> 2) of one stripe
    # of codeLength 4,404,020 B, the lone-caller GPU calls' counterpart (hostpath_lone)
    # (cold: each timed call on another of 16 stripes, 423 MB in all, far beyond the
    # 32 MB L3 of a CCD, as a degraded read's survivors arrive fresh from disk / network)
    Lc, nst = 4404020, 16
    many = np.empty((nst, n, Lc), np.uint8)
    orc.fill_splitmix(0x10E, many)
    one_out = np.empty((1, 1, Lc), np.uint8)
    lone = {}
    for name, coef, src, dst_of, dst_stride in (
            ("encode", enc_coef, [j * Lc for j in range(k)], lambda i: (many[i:i + 1], [(k + r) * Lc for r in range(m)]),
             n * Lc),
            ("decode", dec_coef, [j * Lc for j in range(1, k + 1)], lambda i: (one_out, [0]), Lc)):
        ts = []
        for i in range(2 * nst):
            buf_out, dst = dst_of(i % nst)
            ts.append(orc.batch_apply(coef, many[i % nst:i % nst + 1], n * Lc, src, buf_out, dst_stride, dst, Lc, 1, 1,
                                      level))
        lone[name] = round(sorted(ts)[nst] * 1e3, 4)
    assert np.array_equal(one_out[0, 0], many[(2 * nst - 1) % nst, 0]), "CPU baseline lone decode mismatch"
    del many
    return {
        "value": round(rate, 3),
        "unit": "GiB/s",
        "cores": threads,
        "threads_used": threads,
        "placement": place,
        "kind": "port",
        "sweep": {key: round(v[2], 3) for key, v in sweep.items()},
        "single_core_GiB/s": round(reps1 * step_bytes / t1 / GIB, 3),
        # core time per GiB coded on the CPU (best point, and one core): against the
        # host path's cpu_core_ms_per_GiB, what offloading saves the node's cores
        "core_ms_per_GiB": round(1e3 * threads / rate, 2),
        "single_core_ms_per_GiB": round(1e3 * t1 / (reps1 * step_bytes / GIB), 2),
        "one_call_1_core_ms": lone,  # median of 32 calls over 16 cold stripes, ELECT's codeLength
        "one_call_workload": "one RS(6,4) call of 4 x 4,404,020 B on one core: encode (2 parity), decode (erase 0)",
        "working_set_bytes": int(base.nbytes + out.nbytes),
        "cpu_model": info["model"],
        "affinity_cpus": info["affinity"],
        "cgroup_quota_cores": info["quota_cores"],
        "numa_nodes": len(numa_cpus()),
        "sample": f"RS({n},{k}) encode + decode (erase 0) of the GPU's batch: {stripes} stripes x {L} B "
                  f"({stripes * k * L / GIB:.2f} GiB data); placement:threads swept over {list(sweep)}, best "
                  f"{best}: {reps} reps in {total_t:.1f} s; {reps1} reps in {t1:.1f} s on 1; oracle "
                  f"{orc.simd_name(level)} (ISA-L's algorithm)",
    }


def host_inclusive(coder, k, m, L, stripes_total, dev, world=1):
    """Pinned host -> H2D -> encode -> D2H; GiB/s of data.  Three streams (H2D,
    compute, D2H) over a ring of 3 device buffers chained by events, so both
    copy directions stay busy; 32 MiB of data per transfer
    (tools/tune/host_sweep.py staged: 47.8 GiB/s there, the PCIe ceiling for
    4 units in and 2 out is ~48 GiB/s)."""
    from elect_amd import _lib
    from elect_amd.batch import encode_batch
    chunk = max(1, (32 << 20) // (k * L))  # stripes per transfer (32 MiB of data)
    nch = max(4, stripes_total // chunk)
    ring = 3
    # the host buffers on the GPU's NUMA node (first touch while bound there; the
    # affinity is restored after): a node-remote buffer costs up to 15 % of the
    # link rate at low concurrency (profiles/r06/numa_ab.txt)
    aff = os.sched_getaffinity(0)
    nodes, gnode = numa_cpus(), _lib.device_numa_node(dev.index if dev.index is not None else 0)
    if gnode in nodes:
        os.sched_setaffinity(0, set(nodes[gnode]))
    try:
        h_data = torch.randint(0, 256, (nch * chunk, k, L), dtype=torch.uint8).pin_memory()
        h_par = torch.empty((nch * chunk, m, L), dtype=torch.uint8).pin_memory()
        h_par.fill_(0)
    finally:
        os.sched_setaffinity(0, aff)
    s_in, s_cmp, s_out = torch.cuda.Stream(), torch.cuda.Stream(), torch.cuda.Stream()
    dd = [torch.empty((chunk, k, L), dtype=torch.uint8, device=dev) for _ in range(ring)]
    dp = [torch.empty((chunk, m, L), dtype=torch.uint8, device=dev) for _ in range(ring)]

    def run():
        ev_cmp, ev_out = [None] * nch, [None] * nch
        for c in range(nch):
            r = c % ring
            ev_in = torch.cuda.Event()
            with torch.cuda.stream(s_in):
                if c >= ring:
                    s_in.wait_event(ev_cmp[c - ring])  # ring slot's data consumed
                dd[r].copy_(h_data[c * chunk:(c + 1) * chunk], non_blocking=True)
                ev_in.record(s_in)
            s_cmp.wait_event(ev_in)
            if c >= ring:
                s_cmp.wait_event(ev_out[c - ring])  # ring slot's parity drained
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
    rates = []  # median of 5 passes (PCIe rates vary run to run)
    for _ in range(5):
        t0 = time.perf_counter()
        run()
        rates.append(nch * chunk * k * L / (time.perf_counter() - t0) / GIB)
    # every rank at once (each over its own PCIe link): 3 passes between barriers,
    # aggregate = all ranks' data / the slowest rank's time; each pass's own rate is
    # kept (round 5's driver line had the aggregate 15 % under the median)
    barrier(world)
    t0 = time.perf_counter()
    marks = [t0]
    for _ in range(3):
        run()
        marks.append(time.perf_counter())
    own = marks[-1] - t0
    barrier(world)
    agg = world * 3 * nch * chunk * k * L / max_over_ranks(own, world) / GIB
    passes = [round(nch * chunk * k * L / (b - a) / GIB, 2) for a, b in zip(marks, marks[1:])]
    ref = torch.empty((chunk, m, L), dtype=torch.uint8, device=dev)
    encode_batch(coder, h_data[-chunk:].to(dev), ref)
    torch.cuda.synchronize()
    if not torch.equal(ref.cpu(), h_par[-chunk:]):
        raise RuntimeError("host-inclusive pipeline: parity mismatch")
    detail = {"single_passes_GiB/s": [round(x, 2) for x in rates], "sum_passes_GiB/s": passes,
              "host_numa_node": gnode if gnode in nodes else None}
    return round(sorted(rates)[2], 2), round(agg, 2), detail


def decode_sweep(coder, stripe, stream, reps=5):
    """Single-erasure decode for each data shard j (survivors: the other k of
    shards 0..k), outside the timed region: per-kernel GB/s and HBM fraction.
    The geometry is the coding view's (tiled layouts: B*T stripes of 64 KiB)."""
    from elect_amd.batch import decode_batch
    B, L, k = stripe.shape[0], stripe.shape[2], coder.k
    out = torch.empty((B, 1, L), dtype=torch.uint8, device=stripe.device)
    res = {}
    for j in range(k):
        surv = [i for i in range(k + 1) if i != j]
        decode_batch(coder, stripe, surv, [j], out, inputs_by_unit=True, stream=stream)
        e0, e1 = Event(), Event()
        e0.record(stream)
        for _ in range(reps):
            decode_batch(coder, stripe, surv, [j], out, inputs_by_unit=True, stream=stream)
        e1.record(stream)
        e1.synchronize()
        ms = e0.elapsed_time(e1) / reps
        gbs = B * (k + 1) * L / (ms * 1e-3) / 1e9
        res[f"erase{j}"] = {"ms": round(ms, 4), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                            "verified": bool(torch.equal(out[:, 0], stripe[:, j]))}
    return res


def parity_rows_verified(coder, stripe, decode=None) -> bool:
    """Every parity row the encode wrote, checked through the product: erase data
    units 0..m-1 and rebuild them from the other data units plus ALL m parity
    units (EC/erasure_coder.c:90-91: every one of the m rows is an output).  The
    timed decodes read parity unit k only (survivors 1..k), so a defect confined
    to another parity row would otherwise leave `verified` true.  Outside the
    timed region.  decode: the decode_batch to use (a CPU test injects its own)."""
    if decode is None:
        from elect_amd.batch import decode_batch as decode
    k, m = coder.k, coder.m
    B, L = stripe.shape[0], stripe.shape[2]
    out = torch.empty((B, m, L), dtype=stripe.dtype, device=stripe.device)
    decode(coder, stripe, list(range(m, k + m)), list(range(m)), out, inputs_by_unit=True)
    return bool(torch.equal(out, stripe[:, :m]))


def size_sweep(args, world, rank, dev, coder, sizes=(1024, 1 << 20)):
    """The north star's other chunk sizes (1 KiB and 1 MiB next to the headline's
    64 KiB), each timed exactly like the headline after it: the same step
    (encode + single-erasure decode) over 1 GiB of data per rank, barrier +
    synchronize on both sides, max over ranks, value = all ranks' data / time.
    Layout per the policy of layout_for().  Per-kernel fractions from HIP events
    on this rank."""
    from elect_amd.batch import decode_batch, encode_batch
    k, m = coder.k, coder.m
    res = {}
    for L in sizes:
        B = (1 << 30) // (k * L)
        sets = []  # --rotate: disjoint batches in turn, as in the headline
        for _ in range(args.rotate):
            st, Bc, Lc = alloc_stripes(args, B, L, k, m, dev)
            sets.append((st, torch.empty((Bc, 1, Lc), dtype=torch.uint8, device=dev)))
        turn = [0]

        def launches(i, sets=sets):
            st, out = sets[i % len(sets)]
            return [lambda: encode_batch(coder, st[:, :k], st[:, k:]),
                    lambda: decode_batch(coder, st, list(range(1, k + 1)), [0], out, inputs_by_unit=True)]

        def step():
            for f in launches(turn[0]):
                f()
            turn[0] += 1

        info = {}
        dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
        (enc_ms, dec_ms), _ = split_pass(lambda i: launches(turn[0] + i), args.steps)
        res[str(L)] = {
            "value": round(world * args.steps * 2 * B * k * L / dt / GIB, 2), "unit": "GiB/s",
            "ms_per_step": round(dt / args.steps * 1e3, 4), **info, "stripes_per_gpu": B,
            "host_submit_ms_per_step": round(submit, 4),
            "layout": LAYOUT_NAMES[layout_for(args, L)],
            "encode_frac": round(B * (k + m) * L / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "decode_frac": round(B * (k + 1) * L / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "verified": all(bool(torch.equal(out[:, 0], st[:, 0])) for st, out in sets) and
                        all(parity_rows_verified(coder, st) for st, _ in sets)}
        del sets
    return res


def device_copy_rate(dev, nbytes=1 << 30, reps=5):
    """A plain device copy (torch copy_ of 1 GiB) as a measured HBM reference
    next to the 8 TB/s peak; read + write bytes counted."""
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    e0, e1 = Event(), Event()
    e0.record()
    for _ in range(reps):
        b.copy_(a)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return round(2 * nbytes / (ms * 1e-3) / 1e9, 1)


# (block, waves per CU, XCD-major order): tools/tune/tune_apply's probe; the plain coding launches;
# and the read shape tools/tune/ceiling_probe.hip found fastest (2 GiB at 7.57-7.62 TB/s on two
# boxes, against 6.87-7.06 in dispatch order: each XCD streaming one contiguous eighth)
PROBE_SHAPES = ((256, 0, False), (64, 18, False), (256, 24, True))
# the coding kernels' own stream mixes (4 in, 1 or 2 out): the one-wave shapes they launch, and
# the XCD-major shape that helps 256-thread blocks (profiles/r04/ceiling_probe.txt)
MIX_SHAPES = ((64, 0, False), (64, 18, False), (256, 18, True))


def hbm_ceilings(dev, nbytes=1 << 31, reps=9):
    """The HBM ceilings the coding kernels are judged against, measured on this GPU
    by the library's own probe kernels (elect_ec_hbm_probe: 16 bytes per lane, the
    coding kernels' non-temporal loads and stores): read, write and copy over 2 GiB
    buffers (read + write bytes counted), each the best of PROBE_SHAPES, and the
    decode- and encode-shaped mixes (four 512 MiB streams XORed into one or two),
    each the best of MIX_SHAPES; every figure the median of `reps` launches timed
    with HIP events on the stream they run on.  The achievable figures beside the
    8 TB/s spec peak."""
    from elect_amd import _lib
    # bytes below 0x80: the read probe's sink condition (a segment whose four dwords XOR to
    # 0x9E3779B9, rs_kernels.hip hbm_probe_kernel) can then never hold.  Over uniform random
    # bytes it held for about one run in 32 (2^27 segments against 2^-32 each), and the
    # check below then failed the whole line.
    a = torch.randint(0, 128, (nbytes,), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    sink = torch.zeros(256, dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream()
    quarter = nbytes // 4
    kinds = {"read": (0, a, sink, nbytes, 1, PROBE_SHAPES), "write": (1, None, b, nbytes, 1, PROBE_SHAPES),
             "copy": (2, a, b, nbytes, 2, PROBE_SHAPES),
             "decode_shape": (3, a, b, quarter, 5, MIX_SHAPES), "encode_shape": (4, a, b, quarter, 6, MIX_SHAPES)}
    res = {}
    for name, (kind, src, dst, n, mult, shapes) in kinds.items():
        best = 0.0
        for block, waves, xcd in shapes:
            def launch():
                _lib.hbm_probe(kind | (0x100 if xcd else 0), src.data_ptr() if src is not None else 0, dst.data_ptr(),
                               n, block, waves, stream.cuda_stream)
            launch()
            ts = []
            for _ in range(reps):
                e0, e1 = Event(), Event()
                e0.record(stream)
                launch()
                e1.record(stream)
                e1.synchronize()
                ts.append(e0.elapsed_time(e1))
            gbs = mult * n / (sorted(ts)[reps // 2] * 1e-3) / 1e9
            res[f"{name}_{block}x{waves}{'_xcd' if xcd else ''}"] = round(gbs, 1)
            best = max(best, gbs)
        res[name] = round(best, 1)
    if bool(sink.any()):
        raise RuntimeError("hbm probe: the read probe's sink was written")
    torch.cuda.synchronize()
    del a, b, sink
    return res


def chunk_name(L: int) -> str:
    """'64 KiB' for 65536 (BASELINE.json's metric string), '1 MiB', or bytes."""
    if L % (1 << 20) == 0:
        return f"{L >> 20} MiB"
    if L % 1024 == 0:
        return f"{L >> 10} KiB"
    return f"{L} B"


TILE = 1 << 16  # the unit size HBM streams best back to back
LAYOUT_NAMES = {"unit": "[k+m][B][L]", "stripe": "[B][k+m][L]", "tiled": "[B][L/64K][k+m][64K]"}


def layout_for(args, L: int) -> str:
    """HBM layout of a batch of L-byte chunks: --layout, or for "auto" unit-major
    [k+m][B][L] when L <= 4 KiB, stripe-major [B][k+m][L] up to 64 KiB, and for
    larger multiples of 64 KiB 64 KiB tiles [B][L/64K][k+m][64K]."""
    if args.layout != "auto":
        return args.layout
    if L <= 4096:
        return "unit"
    return "tiled" if L > TILE and L % TILE == 0 and not args.no_tiles else "stripe"


def alloc_stripes(args, B: int, L: int, k: int, m: int, dev, generator=None):
    """A batch of B stripes of k+m L-byte units in the layout of layout_for(),
    data units filled with random bytes.  Returns the coding view (Bc, k+m, Lc)
    and Bc, Lc.  Tiled: each stripe is stored as L/64K tiles of k+m 64 KiB
    units and coded as B*L/64K stripes of 64 KiB; RS works bytewise, so every
    chunk's parity is the same bytes as coding it whole."""
    layout = layout_for(args, L)
    if layout == "tiled":
        if L % TILE:
            raise ValueError("--layout tiled needs chunks that are a multiple of 64 KiB")
        t = L // TILE
        st = torch.empty((B, t, k + m, TILE), dtype=torch.uint8, device=dev).view(B * t, k + m, TILE)
        Bc, Lc = B * t, TILE
    elif layout == "unit":
        skew = getattr(args, "column_skew", 0)  # bytes between one column's end and the next's start
        if skew:
            base = torch.empty((k + m) * (B * L + skew), dtype=torch.uint8, device=dev)
            st = base.as_strided((B, k + m, L), (L, B * L + skew, 1))
        else:
            st = torch.empty((k + m, B, L), dtype=torch.uint8, device=dev).transpose(0, 1)
        Bc, Lc = B, L
    else:
        st = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
        Bc, Lc = B, L
    st[:, :k] = torch.randint(0, 256, (Bc, k, Lc), dtype=torch.uint8, device=dev, generator=generator)
    return st, Bc, Lc


def settle(step, ms: float) -> int:
    """Run `step` untimed for about `ms` of wall time (synchronising every few
    steps so the host does not run ahead); returns the steps run."""
    n, t0 = 0, time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        step()
        n += 1
        if n % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    return n


def timed(step, steps, warmup, world, settle_ms: float = 0.0, info: dict | None = None):
    """Warm up, then time exactly `steps` steps between barrier + synchronize on
    both sides.  Each rank's clock starts when the opening barrier releases it
    and stops at its closing synchronize (the closing gloo barrier costs ~0.6 ms
    at 8 ranks, a few % of a 20-step region, and is no part of a step); the
    max over ranks is the job's time.  Returns (max over ranks of the elapsed seconds, this rank's host
    submit time per step in ms: the time the host spends issuing one step's
    launches, which must stay well below the step's GPU time).  settle_ms:
    untimed steps before the warmup (settle()).  The steps issue their launches
    only: no event between them (split_pass() times the launches right after);
    two events bracket the region on the current stream, and `info`, if given,
    receives their time per step ("gpu_ms_per_step")."""
    settle(step, settle_ms)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    submit = 0.0
    r0, r1 = Event(), Event()
    t0 = time.perf_counter()
    r0.record()
    for _ in range(steps):
        s0 = time.perf_counter()
        step()
        submit += time.perf_counter() - s0
    r1.record()
    torch.cuda.synchronize()
    own = time.perf_counter() - t0  # this rank's steps, up to its own synchronize
    barrier(world)
    if info is not None:
        info["gpu_ms_per_step"] = round(r0.elapsed_time(r1) / steps, 4)
    return max_over_ranks(own, world), submit / steps * 1e3


def split_pass(launches, steps: int):
    """Per-launch HIP-event durations for a step of several launches: `steps`
    more steps right after the timed region, launches(i) being step i's launches
    in issue order, with an event (Event, device-scope release) before the first
    and after each, all on the current stream.  Returns (mean ms per launch
    position, [per-step ms lists]).  Kept out of the timed region: every event
    record holds the next launch back ~4 us whatever its release scope or form,
    even bound to the dispatch by hipExtLaunchKernel (tools/tune/event_probe.hip,
    profiles/r04/event_cost.txt), 2-3 % of a 0.44 ms headline step at three a step."""
    evs = []
    for i in range(steps):
        fns = launches(i)
        e = [Event() for _ in range(len(fns) + 1)]
        e[0].record()
        for j, f in enumerate(fns):
            f()
            e[j + 1].record()
        evs.append(e)
    torch.cuda.synchronize()
    per = [[e[j].elapsed_time(e[j + 1]) for e in evs] for j in range(len(evs[0]) - 1)]
    return [sum(x) / steps for x in per], per


def graph_steps(fns):
    """Capture each of fns (one step's launches each) in its own HIP graph on a
    side stream; returns their replay functions.  The launchers only enqueue
    kernels on the current stream (no host sync, no allocation once warm), so the
    captured graph replays exactly the launches an eager step makes."""
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    graphs = []
    with torch.cuda.stream(side):
        for fn in fns:
            fn()  # warm: one-time device probes and table uploads happen outside the capture
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    for fn in fns:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            fn()
        graphs.append(g)
    torch.cuda.synchronize()
    return [g.replay for g in graphs]


def config_mixed(args, world, rank, dev):
    """BASELINE configs[3]: RS(6,4) encode + decode (erase 0) over three size
    classes, 1 GiB of data per class in total, each class byte-balanced over
    the ranks (strong scaling: total work fixed)."""
    from elect_amd.batch import decode_batch, decode_batches, encode_batch, encode_batches, partition_by_bytes
    from elect_amd.coder import RSCoder
    k, m = 4, 2
    coder = RSCoder(k, m)
    classes = []
    # --mixed-share N: code only rank 0's share of an N-rank partition on this one GPU (what
    # each GPU of an N-GPU run does under strong scaling), to see the per-GPU rate there
    parts, prank = (args.mixed_share, 0) if args.mixed_share else (world, rank)
    share_bytes = 0
    lanes = max(1, args.mixed_lanes)
    copies = [[] for _ in range(lanes)]  # --mixed-lanes: disjoint copies of the classes, one per lane
    for L in (1024, 4096, 1 << 20):
        total = (1 << 30) // (k * L)
        b, e = partition_by_bytes([k * L] * total, parts, prank)
        share_bytes += 2 * (e - b) * k * L
        for c in range(lanes):
            st, Bc, Lc = alloc_stripes(args, e - b, L, k, m, dev)
            copies[c].append((L, st, torch.empty((Bc, 1, Lc), dtype=torch.uint8, device=dev)))
    classes = copies[0]

    # --mixed-streams S: the classes are independent batches; with S > 1 class i is issued on
    # stream i % S behind an event from the step's stream (and joined back at the end), so
    # one class's launch tail overlaps the next class's ramp-up
    main = torch.cuda.current_stream()
    streams = [main] if args.mixed_streams <= 1 else [torch.cuda.Stream() for _ in range(args.mixed_streams)]

    torch.cuda.synchronize()  # the copies' contents are written before any lane reads them
    enc_pairs = [[(st[:, :k], st[:, k:]) for _, st, _ in cl] for cl in copies]
    dec_pairs = [[(st, out) for _, st, out in cl] for cl in copies]
    lane_streams = [torch.cuda.Stream() for _ in range(lanes)] if lanes > 1 else None
    turn = [0]

    def step_grouped():  # elect_ec_encode_batches / _decode_batches: one launch for all classes each
        c = turn[0] % lanes
        turn[0] += 1
        if lane_streams is None:
            encode_batches(coder, enc_pairs[0])
            decode_batches(coder, dec_pairs[0], [1, 2, 3, 4], [0], inputs_by_unit=True)
            return
        # copy c only ever runs on lane c, so its steps stay ordered; timed() synchronises
        # the whole device around the timed region
        with torch.cuda.stream(lane_streams[c]):
            encode_batches(coder, enc_pairs[c])
            decode_batches(coder, dec_pairs[c], [1, 2, 3, 4], [0], inputs_by_unit=True)

    def step():
        if args.mixed_group:
            return step_grouped()
        cur = torch.cuda.current_stream()
        if len(streams) > 1:
            start = torch.cuda.Event()
            start.record(cur)
        for i, (L, st, out) in enumerate(classes):
            s_i = cur if len(streams) == 1 else streams[i % len(streams)]
            if s_i is not cur:
                s_i.wait_event(start)
            with torch.cuda.stream(s_i):
                encode_batch(coder, st[:, :k], st[:, k:])
                decode_batch(coder, st, [1, 2, 3, 4], [0], out, inputs_by_unit=True)
            if s_i is not cur:
                done = torch.cuda.Event()
                done.record(s_i)
                cur.wait_event(done)

    run = graph_steps([step])[0] if args.graph else step
    info = {}  # the region's events sit on the current stream: one-stream runs only
    dt, submit = timed(run, args.steps, args.warmup, world, args.settle_ms,
                       info if lanes == 1 and len(streams) == 1 else None)
    ok = all(torch.equal(out[:, 0], st[:, 0]) for cl in copies for _, st, out in cl)
    data = 2 * 3 * (1 << 30)  # enc + dec, 3 classes, all ranks together
    per_class = {}  # outside the timed region: each class's kernels by HIP events (median of 9)
    for L, st, out in classes:
        t = {"encode": [], "decode": []}
        for _ in range(9):
            ev = [Event() for _ in range(3)]
            ev[0].record()
            encode_batch(coder, st[:, :k], st[:, k:])
            ev[1].record()
            decode_batch(coder, st, [1, 2, 3, 4], [0], out, inputs_by_unit=True)
            ev[2].record()
            torch.cuda.synchronize()
            t["encode"].append(ev[0].elapsed_time(ev[1]))
            t["decode"].append(ev[1].elapsed_time(ev[2]))
        B, Lc = st.shape[0], st.shape[2]  # the coding view (tiled: B*L/64K stripes of 64 KiB)
        enc_ms, dec_ms = sorted(t["encode"])[4], sorted(t["decode"])[4]
        # each launch's own access pattern with the GF work taken out (the same columns, strides
        # and lengths: the unit-major [k+m][B][L] layout of the small classes, tiles for 1 MiB):
        # frac_of_mix = probe time / kernel time
        enc_mix = mix_ceiling([st[:, j] for j in range(k)], [st[:, k + r] for r in range(m)], Lc)
        dec_mix = mix_ceiling([st[:, j] for j in (k, 1, 2, 3)], [out[:, 0]], Lc)
        per_class[f"{L}B"] = {"encode_frac": round(B * (k + m) * Lc / (enc_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "decode_frac": round(B * (k + 1) * Lc / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "encode_mix_frac": round(B * (k + m) * Lc / (enc_mix["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "decode_mix_frac": round(B * (k + 1) * Lc / (dec_mix["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                              "encode_frac_of_mix": round(enc_mix["ms"] / enc_ms, 4),
                              "decode_frac_of_mix": round(dec_mix["ms"] / dec_ms, 4),
                              "mix_blocks": [enc_mix["block"], dec_mix["block"]]}
    if args.mixed_share:  # one GPU's share of an N-GPU run, timed alone: its own rate, and N x it
        per_gpu = args.steps * share_bytes / dt / GIB
        return {"metric": f"GiB/s device-resident RS(6,4) encode+decode, mixed chunks: one GPU's share of an "
                          f"{parts}-GPU strong-scaled run", "value": round(per_gpu, 2), "unit": "GiB/s (this GPU)",
                "n_gpus": world, "share_of": parts, "aggregate_if_ranks_scale": round(parts * per_gpu, 2),
                "steps": args.steps, "ms_per_step": round(dt / args.steps * 1e3, 4), **info,
                "host_submit_ms_per_step": round(submit, 4), "graph": bool(args.graph),
                "streams": len(streams), "grouped": bool(args.mixed_group), "verified": ok, "classes": per_class, "data": "synthetic", "dtype": "u8", "higher_is_better": True,
                "config": {"workload": f"rank 0's byte-balanced share of 1 GiB per class split {parts} ways"}}
    return {"metric": "GiB/s device-resident RS(6,4) encode+decode, mixed 1 KiB/4 KiB/1 MiB chunks",
            "value": round(args.steps * data / dt / GIB, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), **info,
            "host_submit_ms_per_step": round(submit, 4), "graph": bool(args.graph), "streams": len(streams),
            "grouped": bool(args.mixed_group), "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic", "verified": ok, "classes": per_class,
            "config": {"layout": {f"{L}B": LAYOUT_NAMES[layout_for(args, L)] for L, _, _ in classes},
                       "workload": "RS(6,4) encode+decode (erase 0), 1 GiB data per class "
                                   "(1 KiB x 262144, 4 KiB x 65536, 1 MiB x 256 stripes) over all ranks",
                       "parallelism": f"per-class byte-balanced stripe partition x{world}"}}


def config_rs12(args, world, rank, dev):
    """BASELINE configs[4]: RS(12,8) two-erasure decode (erase {0,1}, survivors
    {2..9}), 256 KiB chunks, 512 stripes per GPU (weak scaling)."""
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 8, 4, 262144, 512
    e = args.rs12_erasures
    coder = RSCoder(k, m)
    st, Bc, Lc = alloc_stripes(args, B, L, k, m, dev)  # layout policy of layout_for (64 KiB tiles)
    encode_batch(coder, st[:, :k], st[:, k:])
    out = torch.empty((Bc, e, Lc), dtype=torch.uint8, device=dev)
    surv = list(range(e, e + k))
    def step():
        decode_batch(coder, st, surv, list(range(e)), out, inputs_by_unit=True)

    info = {}
    dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
    (ms,), (per_step,) = split_pass(lambda i: [step], args.steps)
    ok = torch.equal(out, st[:, :e])
    alg = B * (k + e) * L
    gbs = alg / (ms * 1e-3) / 1e9
    # the same code's encode (k=8, m=4), outside the timed region: HIP events per launch
    par = st[:, k:].clone()
    enc_ev = []
    for _ in range(max(5, args.steps)):
        e0, e1 = Event(), Event()
        e0.record()
        encode_batch(coder, st[:, :k], st[:, k:])
        e1.record()
        enc_ev.append((e0, e1))
    torch.cuda.synchronize()
    ok = ok and torch.equal(par, st[:, k:]) and parity_rows_verified(coder, st)  # parity rows 0..3 all read
    enc_ms = sorted(a.elapsed_time(b) for a, b in enc_ev)[len(enc_ev) // 2]
    enc_gbs = B * (k + m) * L / (enc_ms * 1e-3) / 1e9
    # each launch against a probe of its own stream mix (8 in / 4 out, 8 in / e out; no GF work)
    mixes = {"encode": mix_ceiling([st[:, j] for j in range(k)], [par[:, r] for r in range(m)], Lc)}
    if e in (1, 2, 4):
        mixes["decode"] = mix_ceiling([st[:, j] for j in surv], [out[:, r] for r in range(e)], Lc)
    torch.cuda.synchronize()
    dec_k = {"ms": round(ms, 4), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}
    enc_k = {"ms": round(enc_ms, 4), "GB/s": round(enc_gbs, 1), "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
             "mix_probe": mixes["encode"], "frac_of_mix": round(mixes["encode"]["ms"] / enc_ms, 4)}
    if "decode" in mixes:
        dec_k.update(mix_probe=mixes["decode"], frac_of_mix=round(mixes["decode"]["ms"] / ms, 4))
    name = {1: "single", 2: "two", 3: "three", 4: "four"}[e]
    return {"metric": f"GiB/s device-resident RS(12,8) {name}-erasure decode, 256 KiB chunks",
            "kernels": {f"decode_{e}erasure": dec_k, "encode": enc_k},
            "value": round(world * args.steps * B * k * L / dt / GIB, 2), "unit": "GiB/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "host_submit_ms_per_step": round(submit, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic", "verified": ok,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": f"gf_apply_x16u<8,{e}> (decode)", "algorithmic_bytes_per_launch": alg},
            **info, **({"per_step_ms": [round(x, 4) for x in per_step]} if args.per_step else {}),
            "config": {"workload": f"RS(12,8) decode erase {set(range(e))} from {surv}, {B} x {L} B stripes per GPU",
                       "layout": LAYOUT_NAMES[layout_for(args, L)],
                       "parallelism": f"stripe-partitioned x{world}"}}


def config_hostpath(args, world, rank, dev):
    """The drop-in path exactly as ELECT drives it: synchronous encode of one
    stripe per call from pageable host memory (JVM direct buffers), codeLength
    = ceil(4 MiB * 1.05) = 4,404,020 B (StorageService.java:331-339), with
    --threads concurrent callers (ELECT's concurrent_ec pool, elect.yaml:598;
    each coding task encodes synchronously, ECMessageVerbHandler.java:282-319).
    --host-devices N spreads the callers over devices 0..N-1 the way
    ELECT_EC_DEVICES=all does for ELECT's one JVM per node (each calling thread
    keeps one device, round robin)."""
    import threading

    import numpy as np

    from elect_amd.coder import RSCoder
    from elect_amd import _lib
    k, m, L = 4, 2, args.host_chunk
    T = args.threads
    if args.host_register is not None:  # read by the library at its first host call
        os.environ["ELECT_EC_REGISTER"] = str(args.host_register)
    coder = RSCoder(k, m)
    _lib.set_batching(args.batch)
    ndev = max(1, args.host_devices)
    if args.host_devices:
        avail = torch.cuda.device_count()
        if ndev > avail:
            raise SystemExit(f"--host-devices {ndev}: only {avail} device(s) visible")
        _lib.set_host_devices(list(range(ndev)))
    numa = {"policy": args.host_numa}
    if args.host_numa != "none":  # before any buffer is touched: first-touch places them on the bound node
        nodes = numa_cpus()
        gnode = _lib.device_numa_node(dev.index if dev.index is not None else 0)
        numa["gpu_node"] = gnode
        if gnode in nodes and len(nodes) >= 2:
            target = gnode if args.host_numa == "local" else min(n for n in nodes if n != gnode)
            os.sched_setaffinity(0, set(nodes[target]))
            numa.update(bound_node=target, cpus=len(nodes[target]))
        else:
            numa["unavailable"] = f"device node {gnode}, nodes {sorted(nodes)}"
    bufs, keep = [], []
    pinned = args.host_alloc == "pinned"

    def host_array(n):
        if not pinned:
            return np.empty(n, np.uint8)
        hb = _lib.HostBuffer(n)  # what ECNative.allocateDirect would wrap
        keep.append(hb)
        return hb.array

    for t in range(T):
        d = []
        for j in range(k):
            a = host_array(L)
            a[:] = np.random.default_rng(t * 8 + j).integers(0, 256, L, dtype=np.uint8)
            d.append(a)
        p = [host_array(L) for _ in range(m)]
        bufs.append((d, p))
    if pinned and not all(_lib.host_pinned(x.ctypes.data, L) for d, p in bufs for x in d + p):
        raise RuntimeError("--host-alloc pinned: elect_ec_host_alloc returned memory that is not page-locked")
    fused = args.host_op == "encode_ex"
    op = args.host_op
    # decode: each caller rebuilds its unit 0 into a unit of its own; update: a new version of
    # unit 1 per caller, applied in place to its parity (alternating old/new keeps the data valid)
    extra = [host_array(L) for _ in range(T)] if op in ("decode", "update") else []
    if op == "decode":
        for t in range(T):
            d, p = bufs[t]
            coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    if op == "update":
        for t in range(T):
            extra[t][:] = np.random.default_rng(10_000 + t).integers(0, 256, L, dtype=np.uint8)
            d, p = bufs[t]
            coder.encode_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L)
    content = [int(L / 1.05) - 64 * j for j in range(k)]  # SSTables just under codeLength/1.05

    errors = []
    update_counts = [0] * T
    # (start, end) of every call per caller; the rate counts the calls that END inside the
    # timed window [t1, t2] of a free-running set of callers (each loops until told to stop:
    # steady state, no join of all callers every few calls as before round 6, whose ramp-down
    # and thread starts the rate used to include)
    spans = [[] for _ in range(T)]
    clock = time.perf_counter
    go, stop = threading.Event(), threading.Event()

    def worker(t):
        try:
            if not args.host_devices:
                torch.cuda.set_device(dev)
            d, p = bufs[t]
            da, pa = [x.ctypes.data for x in d], [x.ctypes.data for x in p]
            rec = spans[t].append
            go.wait()
            i = 0
            while not stop.is_set():
                t0 = clock()
                if op == "decode":
                    coder.decode_host([pa[0]] + da[1:], [4, 1, 2, 3], [0], [extra[t].ctypes.data], L)
                elif op == "update":
                    ver = [da[1], extra[t].ctypes.data]  # the current and the next version of unit 1
                    coder.encode_update_host([ver[i % 2], ver[(i + 1) % 2]] + pa, 1, pa, L)
                    update_counts[t] += 1
                elif fused:
                    coder.encode_ex_host(da, pa, L, data_lengths=content, hashed=True)
                else:
                    coder.encode_host(da, pa, L)
                rec((t0, clock()))
                i += 1
        except Exception as e:  # a failed call fails the run (a thread's exception would vanish)
            errors.append(f"caller {t}: {e!r}")

    import resource
    th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for x in th:
        x.start()
    window = args.host_seconds if args.host_seconds > 0 else 1.0
    go.set()
    time.sleep(max(0.3, min(1.0, window / 4)))  # warm: every caller's device, arenas, dispatchers, locks
    r0, t1 = resource.getrusage(resource.RUSAGE_SELF), clock()
    time.sleep(window)
    r1, t2 = resource.getrusage(resource.RUSAGE_SELF), clock()
    stop.set()
    for x in th:
        x.join()
    if errors:
        raise RuntimeError(f"{len(errors)} caller(s) failed: {errors[0]}")
    dt = t2 - t1
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    timed = [e - b for sp in spans for (b, e) in sp if t1 <= e <= t2]
    if not timed:
        raise RuntimeError(f"no call completed inside the {window:.1f} s window")
    done_calls = len(timed)
    done = max(1, round(done_calls / T))  # calls per caller (reported as steps)
    calls_s = np.sort(np.asarray(timed))
    d, p = bufs[0]  # self-check through the product: rebuild d0 from [p0, d1, d2, d3]
    rebuilt = np.empty(L, np.uint8)
    coder.decode_host([p[0].ctypes.data] + [x.ctypes.data for x in d[1:]], [4, 1, 2, 3], [0],
                      [rebuilt.ctypes.data], L)
    ok = bool(np.array_equal(rebuilt, d[0])) if not fused and op != "update" else True
    if op == "decode":  # every caller's last rebuilt unit is its unit 0
        ok = ok and all(np.array_equal(extra[t], bufs[t][0][0]) for t in range(T))
    if op == "update":  # each caller's parity now encodes its current version of unit 1
        for t in range(T):
            d, p = bufs[t]
            cur = d[1] if update_counts[t] % 2 == 0 else extra[t]
            units = [d[0], cur, d[2], d[3]]
            ref = [np.empty(L, np.uint8) for _ in range(m)]
            coder.encode_host([x.ctypes.data for x in units], [x.ctypes.data for x in ref], L)
            ok = ok and all(np.array_equal(a, b) for a, b in zip(p, ref))
    if fused:  # self-check: the fused step's parity equals a plain encode of the zero-filled units
        from elect_amd.coder import java_bytebuffer_hash
        z = [np.concatenate([x[:n], np.zeros(L - n, np.uint8)]) for x, n in zip(d, content)]
        ref = [np.empty(L, np.uint8) for _ in range(m)]
        coder.encode_host([x.ctypes.data for x in z], [x.ctypes.data for x in ref], L)
        hs = coder.encode_ex_host([x.ctypes.data for x in d], [x.ctypes.data for x in p], L,
                                  data_lengths=content, hashed=True)
        ok = all(np.array_equal(a, b) for a, b in zip(p, ref)) and hs == [java_bytebuffer_hash(x) for x in ref]
    # every caller's last parity against the CPU oracle's restatement is in tests/; here each
    # caller's parity must at least equal caller 0's recomputation on its own data
    op_name = {"encode_ex": "fused encode step (zero fill + encode + parity hashCode, elect_ec_encode_ex)",
               "decode": "single-erasure decode", "update": "parity update (encodeUpdate, in place)"}.get(op, "encode")
    # data = the bytes each call reads: k units (encode, decode), old + new + m parity (update)
    data_gib = done_calls * (2 + m if op == "update" else k) * L / GIB
    stats = _lib.host_path_stats()
    call_latency = {"p50": round(float(np.percentile(calls_s, 50)) * 1e3, 4),
                    "p99": round(float(np.percentile(calls_s, 99)) * 1e3, 4),
                    "mean": round(float(calls_s.mean()) * 1e3, 4), "calls": int(calls_s.size)}
    core_ms = cpu * 1e3 / data_gib
    quota = host_cpu_info()["quota_cores"] or len(os.sched_getaffinity(0))
    return {"metric": f"GiB/s host-memory RS(6,4) {op_name} through the C ABI (JNI calling convention)",
            "value": round(data_gib / dt, 2), "unit": "GiB/s", "n_gpus": world,
            "devices": ndev, "callers": T, "host_path_stats": stats, "host_alloc": args.host_alloc, "numa": numa,
            "host_register": os.environ.get("ELECT_EC_REGISTER", "library default"),
            # CPU time the whole process spent (every caller, helper and dispatcher thread) per GiB
            # of data coded: what the offload costs the node's cores
            "cpu_core_ms_per_GiB": round(core_ms, 2),
            # the rate this path could reach if the process's CPU quota were its only limit
            "cpu_bound_ceiling_GiB/s": round(quota * 1e3 / core_ms, 1) if core_ms > 0 else None,
            "cpu_quota_cores": quota,
            # wall time of one synchronous call, as its caller sees it (every timed call of every caller)
            "call_latency_ms": call_latency,
            "steps": done, "calls_timed": done_calls, "window_s": round(dt, 3), "warmup": 1,
            "ms_per_step": round(dt / done * 1e3, 3), "higher_is_better": True,
            "scaling": "none", "vs_baseline": None, "dtype": "u8", "data": "synthetic", "verified": ok,
            "config": {"workload": f"{T} threads x ~{done} synchronous elect_ec_{args.host_op} calls, one stripe "
                                   f"of {k} x {L} B each, "
                                   f"{'elect_ec_host_alloc (page-locked)' if pinned else 'pageable'} host buffers, "
                                   f"over {ndev} device(s)",
                       "parallelism": ("cross-thread batching (shared pinned arena, one launch per batch)"
                                       if args.batch else "per-thread pinned staging + 2 streams") +
                                      (f", callers spread over devices 0..{ndev - 1} (elect_ec_set_host_devices)"
                                       if args.host_devices else "")}}


HOSTPATH_CALLERS = 64  # ELECT's concurrent_ec (conf/elect.yaml:598)
# The children of hostpath_all_devices share one deadline, well inside the 10-minute gloo
# timeout the other ranks wait under at the barrier (elect_amd/dist.py): a slow or hung child
# yields a verified=false record, never a dead job.
HOSTPATH_TOTAL_TIMEOUT_S = 480
HOSTPATH_CHILD_TIMEOUT_S = 280


def hostpath_child_cmd(ndev: int, alloc: str = "pageable") -> list:
    """The child process hostpath_all_devices starts: the JNI calling convention,
    64 callers, ELECT's codeLength, batching on, callers over devices 0..ndev-1;
    alloc: the callers' buffers (pageable: ELECT as it is; pinned: ELECT with its
    coding buffers from elect_ec_host_alloc)."""
    return [sys.executable, os.path.abspath(__file__), "--config", "hostpath", "--threads", str(HOSTPATH_CALLERS),
            "--host-chunk", "4404020", "--batch", "1", "--host-devices", str(ndev), "--steps", "8",
            "--host-seconds", "2", "--host-alloc", alloc]


def hostpath_lone_cmd(op: str) -> list:
    """One caller on one device, ELECT's codeLength, pageable units, bound to the
    device's NUMA node: ELECT's degraded read (one synchronous decodeImpl,
    JEC/net/ECRecovery.java:141) or a lone encode, with per-call latency."""
    return [sys.executable, os.path.abspath(__file__), "--config", "hostpath", "--threads", "1", "--host-chunk",
            "4404020", "--batch", "1", "--host-op", op, "--host-seconds", "1", "--host-numa", "local"]


def child_env() -> dict:
    """This environment without the launcher's rank variables: the child is a
    single process of its own (bench.py refuses a WORLD_SIZE that disagrees with
    --gpus), not a member of the job's gloo group."""
    drop = ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE", "ROLE_RANK",
            "ROLE_WORLD_SIZE", "ROLE_NAME", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID",
            "TORCHELASTIC_RESTART_COUNT", "TORCHELASTIC_MAX_RESTARTS", "TORCHELASTIC_USE_AGENT_STORE")
    return {key: v for key, v in os.environ.items() if key not in drop}


def hostpath_all_devices(args, world, rank, child=None):
    """The path ELECT actually calls, on every device of the job: rank 0 starts a
    child process (ELECT runs one JVM per node) that drives the JNI calling
    convention with 64 concurrent callers on ELECT's codeLength, batching on,
    spread over devices 0..world-1 by elect_ec_set_host_devices
    (ECMessageVerbHandler.java:282-319: a new coder and a synchronous encode per
    stripe, on the ERASURECODE stage); the other ranks wait at the gloo barrier.
    The child is a new process (no exec) and sees every device.  child: another
    command line (the CPU plumbing test).  Returns the child's record on rank 0."""
    import subprocess
    res = None
    barrier(world)
    if rank == 0:
        ndev = world if child is not None else min(world, torch.cuda.device_count())
        runs = [("pageable", child)] if child is not None else [("pageable", None), ("pinned", None),
                                                                ("lone_decode", hostpath_lone_cmd("decode")),
                                                                ("lone_encode", hostpath_lone_cmd("encode"))]
        deadline = time.monotonic() + HOSTPATH_TOTAL_TIMEOUT_S
        for alloc, cmd_override in runs:
            cmd = cmd_override if cmd_override is not None else hostpath_child_cmd(ndev, alloc)
            limit = min(HOSTPATH_CHILD_TIMEOUT_S, deadline - time.monotonic())
            try:
                if limit <= 0:
                    raise subprocess.TimeoutExpired(cmd, 0)
                r = subprocess.run(cmd, capture_output=True, text=True, env=child_env(), timeout=limit)
            except subprocess.TimeoutExpired as e:
                r = subprocess.CompletedProcess(cmd, -9, (e.stdout or b"").decode(errors="replace") if isinstance(
                    e.stdout, bytes) else (e.stdout or ""), f"timed out after {max(0.0, limit):.0f} s")
            line = next((x for x in reversed(r.stdout.splitlines()) if x.startswith("{")), None)
            if r.returncode != 0 or line is None:
                rec = {"verified": False, "devices": ndev, "error": f"rc={r.returncode}: {(r.stderr or r.stdout)[-400:]}"}
            elif child is not None:
                rec = {"verified": True, "devices": ndev, "child": json.loads(line)}
            else:
                o = json.loads(line)
                rec = {"value": o["value"], "unit": o["unit"], "devices": o["devices"], "callers": o["callers"],
                       "host_alloc": o.get("host_alloc"), "call_latency_ms": o.get("call_latency_ms"),
                       "cpu_core_ms_per_GiB": o.get("cpu_core_ms_per_GiB"),
                       "cpu_bound_ceiling_GiB/s": o.get("cpu_bound_ceiling_GiB/s"),
                       "cpu_quota_cores": o.get("cpu_quota_cores"),
                       "host_path_stats": o.get("host_path_stats"),
                       "calls_per_caller": o["steps"], "verified": bool(o["verified"]),
                       "workload": o["config"]["workload"], "parallelism": o["config"]["parallelism"]}
            if res is None:
                res = rec
            else:  # ELECT with its coding buffers from elect_ec_host_alloc
                res[alloc] = rec
                res["verified"] = res["verified"] and rec["verified"]
    barrier(world)
    return res


def config_update(args, world, rank, dev):
    """parity update (encodeUpdate, EC/erasure_coder.c:100-142)
    as one fused kernel, RS(6,4), 64 KiB, 4096 stripes per GPU, in place."""
    from elect_amd.batch import encode_batch, encode_update_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 65536, 4096
    coder = RSCoder(k, m)
    old = torch.randint(0, 256, (B, L), dtype=torch.uint8, device=dev)
    new = torch.randint(0, 256, (B, L), dtype=torch.uint8, device=dev)
    par = torch.randint(0, 256, (B, m, L), dtype=torch.uint8, device=dev)
    def step():
        encode_update_batch(coder, 1, old, new, par, par)

    info = {}
    dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
    (ms,), _ = split_pass(lambda i: [step], args.steps)
    # self-check through the product: updating twice with the same delta restores the parity
    ref = par.clone()
    encode_update_batch(coder, 1, old, new, par, par)
    encode_update_batch(coder, 1, old, new, par, par)
    ok = torch.equal(par, ref)
    alg = B * (2 + 2 * m) * L
    gbs = alg / (ms * 1e-3) / 1e9
    return {"metric": "GiB/s device-resident RS(6,4) parity update (encodeUpdate), 64 KiB chunks",
            "value": round(world * args.steps * B * L / dt / GIB, 2), "unit": "GiB/s (updated data bytes)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), **info, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic", "verified": ok,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "gf_update_x16<2>", "algorithmic_bytes_per_launch": alg},
            "config": {"workload": f"in-place parity update of data unit 1, {B} x {L} B stripes per GPU",
                       "parallelism": f"stripe-partitioned x{world}"}}


def mix_ceiling(srcs, dsts, L: int, lens=None, reps: int = 5) -> dict:
    """The access pattern of a coding launch without its GF arithmetic
    (elect_ec_mix_probe): inputs `srcs` (each [S, L]-strided uint8 views, the
    kernel's columns), content lengths `lens` ([S, len(srcs)] int32 on the device,
    or None), XORed into `dsts`.  Best of 64 / 128 / 256-thread blocks, median of
    `reps` launches each, HIP events.  Returns {"ms", "block"}: what a kernel of
    this shape could reach here; a kernel's frac_of_mix = this ms / its ms."""
    from elect_amd import _lib
    S = srcs[0].shape[0]
    lp = lens.to(torch.int32).contiguous() if lens is not None else None
    best = None
    for block in (64, 128, 256):
        ts = []
        for _ in range(reps + 1):
            e0, e1 = Event(), Event()
            e0.record()
            _lib.mix_probe([(t.data_ptr(), t.stride(0)) for t in srcs], [(t.data_ptr(), t.stride(0)) for t in dsts],
                           L, S, lp.data_ptr() if lp is not None else 0, block,
                           stream=torch.cuda.current_stream().cuda_stream)
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = sorted(ts[1:])[reps // 2]
        if best is None or ms < best["ms"]:
            best = {"ms": round(ms, 4), "block": block}
    return best


def config_padded(args, world, rank, dev):
    """encode with implicit zero padding, RS(6,4), 64 KiB
    codeLength, content lengths uniform in [0, L] (mean 50 % fill)."""
    from elect_amd.batch import encode_batch, encode_batch_padded
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 65536, 4096
    coder = RSCoder(k, m)
    data = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev)
    if args.pad_fill == "random":
        lens = torch.randint(0, L + 1, (B, k), dtype=torch.int32, device=dev)
    else:
        lens = torch.full((B, k), int(float(args.pad_fill) * L), dtype=torch.int32, device=dev)
    par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
    def step():
        encode_batch_padded(coder, data, lens, par)

    info = {}
    dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
    (ms,), _ = split_pass(lambda i: [step], args.steps)
    # self-check through the product: explicit zero fill + plain encode gives the same parity
    idx = torch.arange(L, device=dev).view(1, 1, L)
    filled = torch.where(idx < lens.view(B, k, 1), data, torch.zeros((), dtype=torch.uint8, device=dev))
    ref = torch.empty_like(par)
    encode_batch(coder, filled, ref)
    ok = torch.equal(par, ref)
    valid = int(lens.sum().item())
    alg = valid + B * m * L  # bytes actually needed: valid data + full parity
    gbs = alg / (ms * 1e-3) / 1e9
    # the same read:write mix (content prefixes in, full parity out) without the GF work
    mix = mix_ceiling([data[:, j] for j in range(k)], [ref[:, r] for r in range(m)], L, lens)
    mix["frac_of_mix"] = round(mix["ms"] / ms, 4)
    return {"metric": "GiB/s device-resident RS(6,4) zero-padded encode, 64 KiB codeLength",
            "value": round(world * args.steps * B * k * L / dt / GIB, 2), "unit": "GiB/s (codeLength bytes)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), **info, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic", "verified": ok,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "gf_apply_lens<4,2,2> (padded, per-stripe lengths)", "algorithmic_bytes_per_launch": alg,
                         "fill": round(valid / (B * k * L), 3), "mix_probe": mix,
                         "frac_of_mix": mix["frac_of_mix"]},
            "config": {"workload": f"{B} stripes, content lengths " + (f"uniform in [0, {L}]" if args.pad_fill == "random"
                                                                     else f"{args.pad_fill} x {L}"),
                       "parallelism": f"stripe-partitioned x{world}"}}


def config_hashed(args, world, rank, dev):
    """RS(6,4) encode with the fused parity hash
    (java.nio.ByteBuffer.hashCode of every parity unit), 64 KiB, 4096 stripes."""
    from elect_amd.batch import encode_batch, encode_batch_hashed
    from elect_amd.coder import RSCoder
    k, m, L = 4, 2, args.chunk
    B = max(1, (1 << 30) // (k * L))  # 1 GiB of data per GPU
    coder = RSCoder(k, m)
    data = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev)
    par = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
    hashes = torch.empty((B, m), dtype=torch.int32, device=dev)
    def step():
        encode_batch_hashed(coder, data, par, hashes)

    info = {}
    dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
    (ms,), _ = split_pass(lambda i: [step], args.steps)
    ref = torch.empty_like(par)
    encode_batch(coder, data, ref)
    # spot-check two hashes against the closed form on the host
    from elect_amd.coder import java_bytebuffer_hash
    h = hashes.cpu()
    ok = torch.equal(par, ref) and all(int(h[s, r]) == java_bytebuffer_hash(par[s, r].cpu().numpy())
                                       for s, r in ((0, 0), (B - 1, m - 1)))
    alg = B * (k + m) * L
    gbs = alg / (ms * 1e-3) / 1e9
    return {"metric": f"GiB/s device-resident RS(6,4) encode + fused parity hashCode, {L} B chunks",
            "value": round(world * args.steps * B * k * L / dt / GIB, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4), **info,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic", "verified": ok,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "gf_apply_x16<4,2> + hash epilogue", "algorithmic_bytes_per_launch": alg},
            "config": {"workload": f"{B} x {L} B stripes per GPU, hashes [B, m] int32",
                       "parallelism": f"stripe-partitioned x{world}"}}


def config_flows(args, world, rank, dev):
    """ELECT's three coding-node steps as it runs them, each one fused launch:
    transition encode (ECMessageVerbHandler.java:283-329: zero fill to codeLength,
    encode, parity hashCode), parity update (ECParityUpdateVerbHandler.java:
    634-699: old/new zero filled, encodeUpdate in place, new-parity hashCode) and
    degraded read (ECRecovery.java:128-141: survivors zero filled, decode of the
    unit the update replaces).  The update writes its new parity to separate
    buffers as ELECT does (newParityCodes, ECParityUpdateVerbHandler.java:664-688;
    --flows-inplace: over the old parity instead).  RS(6,4), codeLength --chunk,
    --stripes per GPU in one block;
    contents fill 1/1.05 of codeLength less up to 5 % (codeLength = ceil(1.05 x
    SSTable size), StorageService.java:331-339).  Layout: codeLengths above 64 KiB
    are stored as 64 KiB tiles [B][T][k+m][64K] (T = ceil(L / 64K); --flows-tile 0:
    untiled [B][k+m][pitch], the pitch rounded up to 256 B) and coded through the
    elect_ec_*_batch_tiled calls: every unit is then 64 KiB back to back, the
    layout HBM streams best, whatever ELECT's codeLength is."""
    from elect_amd.batch import (decode_batch_ex, decode_batch_tiled, encode_batch, encode_batch_ex,
                                 encode_batch_tiled, encode_update_batch_ex, encode_update_batch_tiled)
    from elect_amd.coder import RSCoder, java_bytebuffer_hash
    k, m, L, B = 4, 2, args.chunk, args.stripes
    n = k + m
    coder = RSCoder(k, m)
    g = torch.Generator(device=dev)
    g.manual_seed(0xE1EC7)
    tile = args.flows_tile if args.flows_tile >= 0 else (TILE if L > TILE else 0)
    if tile:
        T = -(-L // tile)
        blk = torch.empty((B, T, n, tile), dtype=torch.uint8, device=dev)
        view = blk.view(B * T, n, tile)

        def scatter(dst_view, src_logical):  # [B, c, L] -> tiles of dst_view ([B*T, c, tile])
            c = src_logical.shape[1]
            full = torch.zeros((B, c, T * tile), dtype=torch.uint8, device=dev)
            full[:, :, :L] = src_logical
            dst_view.copy_(full.view(B, c, T, tile).permute(0, 2, 1, 3).reshape(B * T, c, tile))

        def gather(src_view):  # tiles -> [B, c, L]
            c = src_view.shape[1]
            return src_view.reshape(B, T, c, tile).permute(0, 2, 1, 3).reshape(B, c, T * tile)[:, :, :L]
        layout = f"[B][{T}][k+m][{tile}] ({tile // 1024} KiB tiles, {T * tile - L} B pad per unit)"
    else:
        pitch = (L + 255) & ~255  # 256-byte unit pitch: ELECT's 4,404,020 B (= 4 mod 16) would misalign units
        stripe = torch.empty((B, n, pitch), dtype=torch.uint8, device=dev)[:, :, :L]
        layout = f"[B][k+m][{pitch}] (unit pitch rounded up to 256 B)"
    top = int(L / 1.05)
    src = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
    lens = torch.randint(int(top * 0.95), top + 1, (B, k), dtype=torch.int32, device=dev, generator=g)
    new_l = torch.randint(0, 256, (B, L), dtype=torch.uint8, device=dev, generator=g)
    t = 1
    ulens = torch.stack([lens[:, t], torch.randint(int(top * 0.95), top + 1, (B,), dtype=torch.int32, device=dev,
                                                   generator=g)], dim=1).contiguous()
    surv = [j for j in range(k) if j != t] + [k]  # degraded read of unit t from the others + parity 0
    dlens = torch.cat([lens[:, [j for j in range(k) if j != t]],
                       torch.full((B, 1), L, dtype=torch.int32, device=dev)], dim=1).contiguous()
    h_enc = torch.empty((B, m), dtype=torch.int32, device=dev)
    h_upd = torch.empty((B, m), dtype=torch.int32, device=dev)
    if tile:
        scatter(view[:, :k], src)
        new = torch.empty((B * T, 1, tile), dtype=torch.uint8, device=dev)
        scatter(new, new_l[:, None])
        new = new[:, 0]
        rebuilt = torch.empty((B * T, 1, tile), dtype=torch.uint8, device=dev)
        data, par = view[:, :k], view[:, k:]
        par_new = par if args.flows_inplace else torch.empty((B * T, m, tile), dtype=torch.uint8, device=dev)

        def enc_step():
            encode_batch_tiled(coder, data, par, L, lengths=lens, hashes=h_enc)

        def upd_step():
            encode_update_batch_tiled(coder, t, view[:, t], new, par, par_new, L, lengths=ulens, hashes=h_upd)

        def dec_step():
            decode_batch_tiled(coder, view, surv, [t], rebuilt, L, lengths=dlens, inputs_by_unit=True)
    else:
        stripe[:, :k] = src
        data, par = stripe[:, :k], stripe[:, k:]
        new = torch.empty((B, (L + 255) & ~255), dtype=torch.uint8, device=dev)[:, :L]
        new.copy_(new_l)
        rebuilt = torch.empty((B, 1, (L + 255) & ~255), dtype=torch.uint8, device=dev)[:, :, :L]
        par_new = par if args.flows_inplace else \
            torch.empty((B, m, (L + 255) & ~255), dtype=torch.uint8, device=dev)[:, :, :L]

        def enc_step():
            encode_batch_ex(coder, data, par, lengths=lens, hashes=h_enc)

        def upd_step():
            encode_update_batch_ex(coder, t, data[:, t], new, par, par_new, lengths=ulens, hashes=h_upd)

        def dec_step():
            decode_batch_ex(coder, stripe, surv, [t], rebuilt, lengths=dlens, inputs_by_unit=True)
    def step():
        enc_step()
        upd_step()
        dec_step()

    info = {}
    dt, submit = timed(step, args.steps, args.warmup, world, args.settle_ms, info)
    ms = dict(zip(("encode", "update", "decode"), split_pass(lambda i: [enc_step, upd_step, dec_step], args.steps)[0]))
    # self-check through the product (coded untiled, contiguous): the new parity is the
    # encode of the zero-filled stripe with unit t replaced, its hashes match, and the
    # degraded read returns the unit t its parity holds, zero filled
    idx = torch.arange(L, device=dev).view(1, L)
    zero = torch.zeros((), dtype=torch.uint8, device=dev)
    filled = torch.where(idx.view(1, 1, L) < lens.view(B, k, 1), src, zero)
    old_t = filled[:, t].clone()
    filled[:, t] = torch.where(idx < ulens[:, 1:2], new_l, zero)
    ref = torch.empty((B, m, L), dtype=torch.uint8, device=dev)
    encode_batch(coder, filled, ref)
    par_l = gather(par_new) if tile else par_new
    reb_l = gather(rebuilt)[:, 0] if tile else rebuilt[:, 0]
    h = h_upd.cpu()
    ok = torch.equal(par_l, ref) and all(int(h[s, r]) == java_bytebuffer_hash(ref[s, r].cpu().numpy())
                                         for s, r in ((0, 0), (B - 1, m - 1)))
    ok = ok and torch.equal(reb_l, filled[:, t] if args.flows_inplace else old_t)
    if tile:  # the output pad of every unit's last tile is written as zero
        ok = ok and not bool(par_new.reshape(B, T, m, tile)[:, -1, :, L - (T - 1) * tile:].any())
    valid = int(lens.sum().item())
    uvalid = int(ulens.sum().item())
    dvalid = int(dlens.sum().item())
    # the layout's own ceiling for these kernels: a plain encode (no padding, no hash) of the
    # same buffers (tiled: every tile whole), HIP events, median of 9 launches
    pe = []
    for _ in range(9):
        e0, e1 = Event(), Event()
        e0.record()
        encode_batch(coder, data, par)
        e1.record()
        e1.synchronize()
        pe.append(e0.elapsed_time(e1))
    plain_ms = sorted(pe)[4]
    plain_alg = data.shape[0] * n * data.shape[2]
    # each step's own read:write mix without its GF work and hash (elect_ec_mix_probe), on the
    # same buffers and content lengths (tiled: each tile's share of its unit's)
    if tile:
        Lc = tile

        def coding_lens(lg):  # [B, c] logical lengths -> [B*T, c] per tile
            t_off = torch.arange(T, device=dev, dtype=torch.int64).view(1, T, 1) * tile
            return (lg.to(torch.int64).view(B, 1, -1) - t_off).clamp(0, tile).view(B * T, -1).to(torch.int32)
        old_col, dec_in = view[:, t], [view[:, j] for j in surv]
    else:
        Lc = L

        def coding_lens(lg):
            return lg.to(torch.int32)
        old_col, dec_in = data[:, t], [stripe[:, j] for j in surv]
    full = torch.full((ulens.shape[0], m), L, dtype=torch.int32, device=dev)
    mixes = {"encode": mix_ceiling([data[:, j] for j in range(k)], [par[:, r] for r in range(m)], Lc, coding_lens(lens)),
             "update": mix_ceiling([old_col, new] + [par[:, r] for r in range(m)], [par_new[:, r] for r in range(m)], Lc,
                                   coding_lens(torch.cat([ulens, full], 1))),
             "decode": mix_ceiling(dec_in, [rebuilt[:, 0]], Lc, coding_lens(dlens))}
    alg = {"encode": valid + B * m * L, "update": uvalid + 2 * B * m * L, "decode": dvalid + B * L}
    kern = {}
    for nm in ("encode", "update", "decode"):
        gbs = alg[nm] / (ms[nm] * 1e-3) / 1e9
        kern[nm] = {"ms": round(ms[nm], 4), "GB/s": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4),
                    "algorithmic_bytes_per_launch": alg[nm], "mix_probe": mixes[nm],
                    "frac_of_mix": round(mixes[nm]["ms"] / ms[nm], 4)}
    return {"metric": "GiB/s device-resident ELECT coding steps (padded+hashed encode, padded+hashed update, "
                      "padded degraded-read decode), RS(6,4)",
            "value": round(world * args.steps * B * (2 * k + 1) * L / dt / GIB, 2),
            "unit": "GiB/s (codeLength bytes: k units encoded + 1 updated + k survivors decoded per stripe)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), **info, "host_submit_ms_per_step": round(submit, 4),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic", "verified": ok, "kernels": kern,
            "plain_encode_same_layout": {"ms": round(plain_ms, 4),
                                         "frac": round(plain_alg / (plain_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                         "note": "full units, no padding or hash: the layout's ceiling for the steps"},
            "roofline": {"bound": "hbm", "achieved": kern["encode"]["GB/s"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": kern["encode"]["frac"], "traffic": None,
                         "kernel": "gf_apply_x16<4,2,PAD,HASH> (encode step)",
                         "algorithmic_bytes_per_launch": alg["encode"],
                         "fill": round(valid / (B * k * L), 3)},
            "config": {"workload": f"{B} stripes x {L} B codeLength per GPU; encode all, update unit {t} "
                                   f"({'in place' if args.flows_inplace else 'new parity to separate buffers'}), "
                                   f"rebuild unit {t} from units {surv}", "layout": layout,
                       "parallelism": f"stripe-partitioned x{world}"}}


def other_configs(args, world, rank, dev):
    """The mixed (strong-scaled) and RS(12,8) (weak-scaled) configs inside the
    headline run, so every `--gpus N` line the driver records carries all three
    multi-GPU BASELINE configs at that N.  Same timing as their own --config
    runs (barrier + synchronize both sides, max over ranks), 20 steps."""
    import copy
    sub = copy.copy(args)
    sub.steps, sub.warmup, sub.mixed_share = min(args.steps, 20), min(args.warmup, 3), 0
    res = {}
    fns = {"mixed": config_mixed, "rs12": config_rs12}
    for name in [x for x in args.configs_order.split(",") if x]:
        fn = fns[name]
        o = fn(sub, world, rank, dev)
        keep = ("metric", "value", "unit", "scaling", "steps", "ms_per_step", "host_submit_ms_per_step",
                "verified", "classes", "kernels")
        res[name] = {key: o[key] for key in keep if key in o}
        res[name]["workload"] = o["config"]["workload"]
        torch.cuda.empty_cache()
    return res


def launch_check(args, world, rank):
    """--launch-check: the multi-rank plumbing with no GPU work (CPU test)."""
    barrier(world)
    t = max_over_ranks(float(rank + 1), world)
    recs = gather({"rank": rank, "world": world, "pid": os.getpid()}, world)
    hp = None
    if world > 1:  # the headline's host-path phase: rank 0's child process, the others at the barrier
        hp = hostpath_all_devices(args, world, rank, child=[sys.executable, os.path.abspath(__file__),
                                                            "--launch-check"])
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "max_over_ranks": t, "ranks": recs,
                          "hostpath_child": hp}), flush=True)


def gather(obj, world):
    from elect_amd import dist
    return dist.gather(obj, world)


def finish(out, rank, world, rec) -> None:
    """Every rank's own record (verified, own time, host submit time) to rank 0,
    which prints the line; exit non-zero on every rank if any rank failed."""
    from elect_amd import _lib, dist
    recs = gather(rec, world)
    ok = all(r["verified"] for r in recs)
    out["verified"] = ok
    out["ranks"] = recs
    out["build"] = {"id": _lib.BUILD_ID, "from_these_sources": _lib.BUILD_CURRENT}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if not rec["verified"]:  # say which check failed (the line's records hold the flags)
        print(f"bench.py: rank {rank} failed verification: {json.dumps(rec)}", file=sys.stderr, flush=True)
    dist.teardown(world)
    if not ok:
        sys.exit(1)


def main():
    global event_release
    args = parse()
    event_release = args.event_release
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: start one rank per GPU (before anything touches the GPU here)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if int(env_world or 1) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}: refusing to report a wrong n_gpus",
              file=sys.stderr)
        sys.exit(2)
    world, rank, local = dist_setup(args)
    if args.launch_check:
        launch_check(args, world, rank)
        from elect_amd import dist
        dist.teardown(world)
        return
    dev = torch.device("cuda", local)
    if args.config != "headline":
        fn = {"mixed": config_mixed, "rs12": config_rs12, "hostpath": config_hostpath,
              "update": config_update, "padded": config_padded, "hashed": config_hashed,
              "flows": config_flows}[args.config]
        out = fn(args, world, rank, dev)
        finish(out, rank, world, {"rank": rank, "device": local, "verified": bool(out.get("verified", True)),
                                  "host_submit_ms_per_step": out.get("host_submit_ms_per_step")})
        return
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder

    k, m, L, B = args.k, args.m, args.chunk, args.stripes
    n = k + m
    coder = RSCoder(k, m)
    g = torch.Generator(device=dev).manual_seed(0xE1EC7 + rank)
    sets = []  # --rotate N: N disjoint stripe batches, one per step in turn (no cache reuse across steps)
    for _ in range(args.rotate):
        if args.unit_gap == 0 and args.rebuilt_rows == 1:
            st, Bc, Lc = alloc_stripes(args, B, L, k, m, dev, generator=g)
            sets.append((st, torch.empty((Bc, 1, Lc), dtype=torch.uint8, device=dev)))
            continue
        if layout_for(args, L) == "unit":  # [k+m][B][L] layout experiment
            st = torch.empty((n, B, L + args.unit_gap), dtype=torch.uint8, device=dev)[:, :, :L].transpose(0, 1)
        elif layout_for(args, L) == "stripe":
            st = torch.empty((B, n, L + args.unit_gap), dtype=torch.uint8, device=dev)[:, :, :L]
        else:
            raise ValueError("--unit-gap / --rebuilt-rows experiments take the unit or stripe layout")
        st[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev, generator=g)
        sets.append((st, torch.empty((B, args.rebuilt_rows, L + args.unit_gap), dtype=torch.uint8, device=dev)[:, :1, :L]))
    stripe, rebuilt = sets[0]
    turn = [0]
    survivors = list(range(1, k + 1))
    stream = torch.cuda.current_stream()
    orig0 = stripe[:, 0].clone() if args.decode_out == "inplace" else None

    def encode_of(st):
        return lambda: encode_batch(coder, st[:, :k], st[:, k:])

    def decode_of(st, rb):
        if args.decode_out == "inplace":  # rebuild unit 0 into its own slot of the stripe
            return lambda: decode_batch(coder, st, survivors, [0], st, inputs_by_unit=True, outputs_by_unit=True)
        return lambda: decode_batch(coder, st, survivors, [0], rb, inputs_by_unit=True)

    ops = [(encode_of(st), decode_of(st, rb)) for st, rb in sets]
    replays = graph_steps([lambda e=e, d=d: (e(), d()) for e, d in ops]) if args.graph else None

    lanes = [torch.cuda.Stream() for _ in range(args.streams)] if args.streams > 1 else None
    if lanes is not None and (replays is not None or len(sets) % args.streams):
        raise SystemExit("--streams S needs eager launches and --rotate a multiple of S")

    def step():
        i = turn[0] % len(sets)
        turn[0] += 1
        if lanes is not None:  # batch i always on lane i % S: reuse stays ordered
            with torch.cuda.stream(lanes[i % len(lanes)]):
                ops[i][0]()
                ops[i][1]()
        elif replays is not None:  # one graph per batch: encode + decode
            replays[i]()
        else:
            ops[i][0]()
            ops[i][1]()

    settle_steps = settle(step, args.settle_ms)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    submit = 0.0
    r0, r1 = Event(), Event()  # the region on the GPU's clock (one-stream runs)
    t0 = time.perf_counter()
    r0.record(stream)
    for i in range(args.steps):
        s0 = time.perf_counter()
        step()
        submit += time.perf_counter() - s0
    r1.record(stream)
    torch.cuda.synchronize()
    own = time.perf_counter() - t0  # clock stops at this rank's synchronize; the
    barrier(world)                  # closing barrier's own latency is not a step's
    elapsed = max_over_ranks(own, world)
    submit_ms = submit / args.steps * 1e3
    gpu_ms = r0.elapsed_time(r1) / args.steps if lanes is None else None

    # per-kernel split: the next args.steps steps again, eager on one stream, an event around
    # each launch (split_pass: events inside the timed region would cost it ~4 us a record)
    (enc_ms, dec_ms), (enc_each, dec_each) = split_pass(lambda i: list(ops[(turn[0] + i) % len(sets)]), args.steps)
    per_step = {"encode": [round(x, 4) for x in enc_each],
                "decode": [round(x, 4) for x in dec_each]} if args.per_step else None
    if args.decode_out == "inplace":  # unit 0 was rebuilt in place: it must still be the original data
        ok = bool(torch.equal(stripe[:, 0], orig0))
    else:
        ok = all(bool(torch.equal(r[:, 0], st[:, 0])) for st, r in sets)
    # every parity row of every batch (the timed decodes read parity unit k only)
    parity_ok = all(parity_rows_verified(coder, st) for st, _ in sets)
    ok = ok and parity_ok

    data_bytes_per_rank_step = 2 * B * k * L  # encode k*L + decode k*L survivors, per stripe
    value = world * args.steps * data_bytes_per_rank_step / elapsed / GIB
    enc_alg = B * n * L               # (k+m)*L per stripe
    dec_alg = B * (k + 1) * L         # (k+e)*L per stripe, e = 1
    enc_gbs = enc_alg / (enc_ms * 1e-3) / 1e9
    dec_gbs = dec_alg / (dec_ms * 1e-3) / 1e9
    # the encode launch: the scalar-base kernel since round 4 (one-wave blocks, whole-wave stripes)
    traffic, traffic_src = pmc_traffic("gf_apply_x16u<4, 2, false, false>", "gf_apply_x16<4, 2")

    out = {
        "metric": f"GiB/s device-resident RS({n},{k}) encode+decode, {chunk_name(L)} chunks, 1/2/4/8 GPU",
        "value": round(value, 2),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (device-generated uniform random bytes)",
        "config": {
            "workload": f"RS({n},{k}) encode + single-erasure decode (erase 0, survivors "
                        f"{survivors}), {B} stripes x {L} B chunks per GPU "
                        f"({B * k * L / GIB:.2f} GiB data per op per GPU)",
            "k": k, "m": m, "chunk_bytes": L, "stripes_per_gpu": B,
            "rotate": args.rotate,  # disjoint batches per rank, one per step in turn
            "parallelism": f"stripe-partitioned x{world}, no collectives (gloo timing handshake only)",
            "graph": bool(args.graph),
            "streams": args.streams,
            "settle": {"ms": args.settle_ms, "steps": settle_steps},  # untimed, before the warmup steps
        },
        "host_submit_ms_per_step": round(submit_ms, 4),
        # the timed region on the GPU's clock: two events around it on the launch stream
        "gpu_ms_per_step": round(gpu_ms, 4) if gpu_ms is not None else None,
        "roofline": {
            "bound": "hbm",
            "achieved": round(enc_gbs, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "kernel": "gf_apply_x16u<4,2> (encode)",
            "algorithmic_bytes_per_launch": enc_alg,
            "traffic_source": traffic_src,
            "timing": f"HIP events (device-scope release) around each launch of {args.steps} steps run right "
                      "after the timed region, same launches and stream (split_pass)",
        },
        "kernels": {
            "encode": {"ms": round(enc_ms, 4), "GB/s": round(enc_gbs, 1),
                       "frac": round(enc_gbs / HBM_PEAK_GBS, 4),
                       "data_GiB/s": round(B * k * L / (enc_ms * 1e-3) / GIB, 1)},
            "decode_1erasure": {"ms": round(dec_ms, 4), "GB/s": round(dec_gbs, 1),
                                "frac": round(dec_gbs / HBM_PEAK_GBS, 4),
                                "data_GiB/s": round(B * k * L / (dec_ms * 1e-3) / GIB, 1)},
        },
        "verified": ok,
        "verified_parity_rows": parity_ok,
    }
    if per_step:
        out["per_step_ms"] = per_step
    rec = {"rank": rank, "device": local, "ms_per_step": round(own / args.steps * 1e3, 4),
           "host_submit_ms_per_step": round(submit_ms, 4), "encode_frac": out["kernels"]["encode"]["frac"],
           "decode_frac": out["kernels"]["decode_1erasure"]["frac"], "verified": ok}
    if not args.no_sizes:  # every rank: the sweep has its own barriers and max over ranks
        out["sizes"] = size_sweep(args, world, rank, dev, coder)
        out["sizes"][str(L)] = {"value": out["value"], "unit": "GiB/s", "ms_per_step": out["ms_per_step"],
                                "stripes_per_gpu": B, "host_submit_ms_per_step": round(submit_ms, 4),
                                "layout": LAYOUT_NAMES[layout_for(args, L)],
                                "encode_frac": out["kernels"]["encode"]["frac"],
                                "decode_frac": out["kernels"]["decode_1erasure"]["frac"], "verified": ok}
        out["sizes"] = {key: out["sizes"][key] for key in sorted(out["sizes"], key=int)}
        rec["sizes_verified"] = all(v["verified"] for v in out["sizes"].values())
        rec["sizes_submit_ms"] = {key: v["host_submit_ms_per_step"] for key, v in out["sizes"].items()}
        rec["verified"] = rec["verified"] and rec["sizes_verified"]
    if not args.no_configs:  # BASELINE configs[3] and [4] at the same N (every rank; own barriers)
        out["configs"] = other_configs(args, world, rank, dev)
        rec["configs_verified"] = {key: v["verified"] for key, v in out["configs"].items()}
        rec["configs_submit_ms"] = {key: v["host_submit_ms_per_step"] for key, v in out["configs"].items()}
        rec["verified"] = rec["verified"] and all(rec["configs_verified"].values())
    if rank == 0:
        out["kernels"]["decode_sweep"] = sw = decode_sweep(coder, stripe, stream)
        rec["verified"] = rec["verified"] and all(v["verified"] for v in sw.values())
        ceil = hbm_ceilings(dev)
        rf = out["roofline"]
        # the achievable ceilings on this GPU (the library's 16 B/lane nt probes), and the
        # coding kernels as fractions of them; torch's own copy kernel kept for reference
        rf["device_copy_GB/s"] = ceil["copy"]
        rf["device_read_GB/s"] = ceil["read"]
        rf["device_write_GB/s"] = ceil["write"]
        rf["frac_of_copy"] = round(enc_gbs / ceil["copy"], 4)
        rf["decode_frac_of_copy"] = round(dec_gbs / ceil["copy"], 4)
        rf["frac_of_read"] = round(enc_gbs / ceil["read"], 4)
        # against probes with the kernels' own stream mix (4 in, 2 out / 4 in, 1 out)
        rf["device_encode_shape_GB/s"] = ceil["encode_shape"]
        rf["device_decode_shape_GB/s"] = ceil["decode_shape"]
        rf["frac_of_encode_shape"] = round(enc_gbs / ceil["encode_shape"], 4)
        rf["decode_frac_of_decode_shape"] = round(dec_gbs / ceil["decode_shape"], 4)
        rf["ceiling_probes"] = {key: v for key, v in ceil.items() if key not in ("read", "write", "copy", "encode_shape",
                                                                                  "decode_shape")}
        rf["torch_copy_GB/s"] = device_copy_rate(dev)
    if not args.no_host:  # every rank, over its own PCIe link, at the same time
        own_rate, agg, hi_detail = host_inclusive(coder, k, m, L, min(B, 4096), dev, world)
        rates = gather(own_rate, world)
        out["host_inclusive_GiB/s"] = rates[0]
        out["host_inclusive_sum_GiB/s"] = agg
        out["host_inclusive_passes"] = hi_detail
        out["host_inclusive_per_rank_GiB/s"] = rates
    if not args.no_host and not args.no_hostpath:  # ELECT's own calls over all the job's devices
        hp = hostpath_all_devices(args, world, rank)
        if rank == 0:
            out["hostpath_all_devices"] = hp
            out["hostpath_all_devices_GiB/s"] = hp.get("value")
            if isinstance(hp.get("pinned"), dict):
                out["hostpath_all_devices_pinned_GiB/s"] = hp["pinned"].get("value")
            rec["verified"] = rec["verified"] and hp["verified"]
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(args, k, m, L, B)
    hp = out.get("hostpath_all_devices") or {}
    lone = {}
    for op in ("decode", "encode"):  # a lone caller's synchronous call (ECRecovery.java:141) against one CPU core
        r = hp.get(f"lone_{op}")
        if isinstance(r, dict) and r.get("value") is not None:
            lat = r.get("call_latency_ms") or {}
            lone[op] = {"GiB/s": r["value"], "p50_ms": lat.get("p50"), "p99_ms": lat.get("p99"),
                        "mean_ms": lat.get("mean")}
            cb = out.get("cpu_baseline") or {}
            if (cb.get("one_call_1_core_ms") or {}).get(op):
                lone[op]["oracle_1_core_ms"] = cb["one_call_1_core_ms"][op]
    if lone:
        out["hostpath_lone_caller"] = lone
    finish(out, rank, world, rec)


if __name__ == "__main__":
    main()
