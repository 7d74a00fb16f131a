"""Where the host path's page-locked memory lands (round 6): for a
thread bound to each NUMA node in turn, the node of the pages of (a) a
hipHostMalloc block (the batcher's arenas are made that way), (b) an
elect_ec_host_alloc pool block (aligned_alloc + hsa_amd_memory_lock by the
calling thread), read with get_mempolicy(MPOL_F_NODE | MPOL_F_ADDR); and the
GPU's own node.  One JSON line.

    python tools/tune/numa_probe.py
"""
import ctypes
import glob
import json
import os
import sys
import threading

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from elect_amd import _lib  # noqa: E402

libc = ctypes.CDLL("libc.so.6", use_errno=True)
SYS_get_mempolicy = 239  # x86_64
MPOL_F_NODE, MPOL_F_ADDR = 1, 2


def page_node(addr: int) -> int:
    mode = ctypes.c_int(-1)
    rc = libc.syscall(SYS_get_mempolicy, ctypes.byref(mode), None, ctypes.c_ulong(0), ctypes.c_void_p(addr),
                      ctypes.c_ulong(MPOL_F_NODE | MPOL_F_ADDR))
    return mode.value if rc == 0 else -1


def node_cpus() -> dict:
    out = {}
    for path in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        with open(os.path.join(path, "cpulist")) as f:
            cpus = []
            for part in f.read().strip().split(","):
                lo, _, hi = part.partition("-")
                cpus += list(range(int(lo), int(hi or lo) + 1))
        out[int(path.rsplit("node", 1)[1])] = set(cpus) & os.sched_getaffinity(0)
    return out


def main():
    import torch  # (the library is bound to torch's HIP runtime in this process; torch's pinned
    # allocator makes its blocks with hipHostMalloc, as the batcher's arenas are made)
    nbytes = 64 << 20
    res = {"gpu_node": _lib.device_numa_node(0), "by_thread_node": {}}

    def probe(node, cpus, out):
        os.sched_setaffinity(0, cpus)
        t = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
        arena = sorted({page_node(t.data_ptr() + off) for off in range(0, nbytes, nbytes // 16)})
        del t
        q = _lib.host_alloc(nbytes)
        pool = sorted({page_node(q + off) for off in range(0, nbytes, nbytes // 16)})
        out[node] = {"hipHostMalloc_page_nodes": arena, "host_alloc_page_nodes": pool,
                     "host_alloc_pinned": bool(_lib.host_pinned(q, nbytes))}

    for node, cpus in node_cpus().items():
        if not cpus:
            continue
        t = threading.Thread(target=probe, args=(node, cpus, res["by_thread_node"]))
        t.start()
        t.join()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
