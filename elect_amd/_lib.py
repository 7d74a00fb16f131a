"""ctypes binding of libelect_ec.so (the C ABI in include/elect_ec.h).

There is no CPU fallback anywhere in this package: if the library is missing
this module raises at import, and without a GPU the compute entry points return
ELECT_EC_ENODEV, which is raised as ECDeviceError.
"""
from __future__ import annotations

import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ELECT_EC_LIB") or os.path.join(HERE, "libelect_ec.so")  # override: A/B builds

OK = 0
WARN_SINGULAR = 1
EINVAL = -1
ESINGULAR = -2
EDEVICE = -3
ENOMEM = -4
ENODEV = -5

DECODE_COMPAT = 0
DECODE_STRICT = 1
INPUTS_BY_UNIT = 1
OUTPUTS_BY_UNIT = 2

MAX_DATA_UNITS = 10
MAX_UNITS = 14
MAX_APPLY = 16


class ECError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{what}: {strerror(status)} ({status})" if what else strerror(status))


class ECDeviceError(ECError):
    pass


class ECSingularError(ECError):
    pass


class ECInvalidArgument(ECError, ValueError):
    pass


class Shards(ctypes.Structure):
    _fields_ = [("base", ctypes.c_void_p), ("stripe_stride", ctypes.c_size_t),
                ("shard_stride", ctypes.c_size_t)]


class ColumnT(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("stripe_stride", ctypes.c_size_t)]


class BatchT(ctypes.Structure):
    _fields_ = [("chunk_size", ctypes.c_size_t), ("num_stripes", ctypes.c_size_t), ("inp", Shards), ("out", Shards)]


_u8p = ctypes.POINTER(ctypes.c_ubyte)
_u8pp = ctypes.POINTER(ctypes.c_void_p)
_ip = ctypes.POINTER(ctypes.c_int)
_cp = ctypes.c_void_p

# (name, restype, argtypes) for every symbol include/elect_ec.h declares.
SIGNATURES = [
    ("elect_ec_version", ctypes.c_char_p, []),
    ("elect_ec_build_id", ctypes.c_char_p, []),
    ("elect_ec_strerror", ctypes.c_char_p, [ctypes.c_int]),
    ("elect_ec_device_count", ctypes.c_int, [_ip]),
    ("elect_ec_unaligned_vector_ok", ctypes.c_int, [_ip]),
    ("elect_ec_hbm_probe", ctypes.c_int, [ctypes.c_int, _cp, _cp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, _cp]),
    ("elect_ec_set_host_devices", ctypes.c_int, [_ip, ctypes.c_int]),
    ("elect_ec_device_numa_node", ctypes.c_int, [ctypes.c_int, _ip]),
    ("elect_ec_host_device_map", ctypes.c_int, [_ip, _ip, ctypes.c_int, _ip, ctypes.c_int, _ip]),
    ("elect_ec_set_batching", ctypes.c_int, [ctypes.c_int, ctypes.c_uint, ctypes.c_size_t]),
    ("elect_ec_internal_pipeline_windows", ctypes.c_int, [ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                                          ctypes.POINTER(ctypes.c_size_t), _ip]),
    ("elect_ec_host_path_stats", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]),
    ("elect_ec_mix_probe", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                          ctypes.POINTER(ColumnT), _cp, ctypes.POINTER(ColumnT), ctypes.c_int,
                                          ctypes.c_int, _cp]),
    ("elect_ec_host_alloc", ctypes.c_int, [ctypes.c_size_t, ctypes.POINTER(_cp)]),
    ("elect_ec_host_free", ctypes.c_int, [_cp]),
    ("elect_ec_host_pinned", ctypes.c_int, [_cp, ctypes.c_size_t]),
    ("elect_ec_coder_create", ctypes.c_int, [ctypes.c_int, ctypes.c_int, ctypes.POINTER(_cp)]),
    ("elect_ec_coder_destroy", None, [_cp]),
    ("elect_ec_coder_num_data_units", ctypes.c_int, [_cp]),
    ("elect_ec_coder_num_parity_units", ctypes.c_int, [_cp]),
    ("elect_ec_coder_encode_matrix", ctypes.c_int, [_cp, _u8p, ctypes.c_size_t]),
    ("elect_ec_coder_gf_tables", ctypes.c_int, [_cp, _u8p, ctypes.c_size_t]),
    ("elect_ec_coder_decode_matrix", ctypes.c_int, [_cp, _ip, _ip, ctypes.c_int, ctypes.c_int, _u8p]),
    ("elect_ec_coder_invert_matrix", ctypes.c_int, [_cp, _ip, _u8p]),
    ("elect_ec_encode", ctypes.c_int, [_cp, _u8pp, _u8pp, ctypes.c_size_t]),
    ("elect_ec_encode_update", ctypes.c_int, [_cp, _u8pp, ctypes.c_int, _u8pp, ctypes.c_size_t]),
    ("elect_ec_encode_padded", ctypes.c_int, [_cp, _u8pp, ctypes.POINTER(ctypes.c_size_t), _u8pp,
                                              ctypes.c_size_t]),
    ("elect_ec_encode_hashed", ctypes.c_int, [_cp, _u8pp, _u8pp, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_int32)]),
    ("elect_ec_encode_ex", ctypes.c_int, [_cp, _u8pp, ctypes.POINTER(ctypes.c_size_t), _u8pp, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_int32)]),
    ("elect_ec_encode_update_ex", ctypes.c_int, [_cp, _u8pp, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int,
                                                 _u8pp, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32)]),
    ("elect_ec_decode", ctypes.c_int, [_cp, _u8pp, _ip, _ip, ctypes.c_int, _u8pp, ctypes.c_size_t,
                                       ctypes.c_int]),
    ("elect_ec_decode_ex", ctypes.c_int, [_cp, _u8pp, ctypes.POINTER(ctypes.c_size_t), _ip, _ip, ctypes.c_int,
                                          _u8pp, ctypes.c_size_t, ctypes.c_int]),
    ("elect_ec_encode_batch", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, Shards, _cp]),
    ("elect_ec_decode_batch", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, _ip, _ip,
                                             ctypes.c_int, Shards, ctypes.c_uint, ctypes.c_int, _cp]),
    ("elect_ec_encode_batch_padded", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, _cp,
                                                    Shards, _cp]),
    ("elect_ec_encode_batch_hashed", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, Shards,
                                                    _cp, _cp]),
    ("elect_ec_encode_update_batch", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                                    ColumnT, ColumnT, Shards, Shards, _cp]),
    ("elect_ec_encode_batch_ex", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, _cp, Shards,
                                                _cp, _cp]),
    ("elect_ec_encode_update_batch_ex", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                                       ColumnT, ColumnT, _cp, Shards, Shards, _cp, _cp]),
    ("elect_ec_decode_batch_ex", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, Shards, _cp, _ip, _ip,
                                                ctypes.c_int, Shards, ctypes.c_uint, ctypes.c_int, _cp]),
    ("elect_ec_encode_batch_tiled", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, Shards,
                                                   _cp, Shards, _cp, _cp]),
    ("elect_ec_encode_update_batch_tiled", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                                          ctypes.c_int, ColumnT, ColumnT, _cp, Shards, Shards, _cp,
                                                          _cp]),
    ("elect_ec_decode_batch_tiled", ctypes.c_int, [_cp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, Shards,
                                                   _cp, _ip, _ip, ctypes.c_int, Shards, ctypes.c_uint, ctypes.c_int,
                                                   _cp]),
    ("elect_ec_encode_batches", ctypes.c_int, [_cp, ctypes.POINTER(BatchT), ctypes.c_int, _cp]),
    ("elect_ec_decode_batches", ctypes.c_int, [_cp, ctypes.POINTER(BatchT), ctypes.c_int, _ip, _ip, ctypes.c_int,
                                               ctypes.c_uint, ctypes.c_int, _cp]),
    ("elect_ec_apply_batch", ctypes.c_int, [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_size_t,
                                            ctypes.c_size_t, ctypes.POINTER(ColumnT),
                                            ctypes.POINTER(ColumnT), _cp]),
]

# One HIP runtime per process.  PyTorch-ROCm bundles its own libamdhip64 /
# libhsa-runtime64 (torch/lib) under the same sonames as /opt/rocm's, which the
# library links.  Loaded first, the library pulls in /opt/rocm's runtime; torch,
# imported later, then loads its own copy beside it (its libraries name the
# unversioned file), and whichever of the two HSA runtimes initialises second
# finds no device: round 5 saw elect_ec_host_alloc's hipHostMalloc fail with
# "no ROCm-capable device is detected" in a test module that imported this
# module before torch.  Importing torch first (where it is installed) makes
# the library bind to torch's already-loaded runtime, as every torch-first
# process already did.  (A JVM loads only the library's own runtime; the GPU
# suite covers that path too: tools/hostpath_cbench, a C++ caller with no torch,
# runs from tests/test_gpu_cbench.py.)  ELECT_EC_NO_TORCH=1 skips the import.
# Any failure of a broken torch install is ignored here: the
# library then loads /opt/rocm's runtime, as in a JVM.
if os.environ.get("ELECT_EC_NO_TORCH") != "1":
    try:
        import torch  # noqa: F401
    except Exception:  # noqa: BLE001
        pass

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is missing: build the MI355X engine first "
                      "(python -m elect_amd.build) — there is no CPU fallback")

lib = ctypes.CDLL(LIB_PATH)
for _name, _res, _args in SIGNATURES:
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args

BUILD_ID = lib.elect_ec_build_id().decode()


def _sources_id() -> str | None:
    try:
        from .build import build_id
        return build_id()
    except OSError:  # sources not shipped beside the library
        return None


# True when the loaded library was built from the sources beside it (by content).
BUILD_CURRENT = LIB_PATH == os.path.join(HERE, "libelect_ec.so") and BUILD_ID == _sources_id()


def strerror(status: int) -> str:
    return lib.elect_ec_strerror(status).decode()


def check(status: int, what: str = "") -> int:
    """Raise for negative statuses; pass OK / WARN_SINGULAR through."""
    if status >= 0:
        return status
    if status in (ENODEV, EDEVICE, ENOMEM):
        raise ECDeviceError(status, what)
    if status == ESINGULAR:
        raise ECSingularError(status, what)
    if status == EINVAL:
        raise ECInvalidArgument(status, what)
    raise ECError(status, what)


def device_count() -> int:
    n = ctypes.c_int(0)
    lib.elect_ec_device_count(ctypes.byref(n))
    return n.value


def unaligned_vector_ok() -> bool:
    """True when misaligned device layouts run the vector kernels (elect_ec.h)."""
    ok = ctypes.c_int(0)
    check(lib.elect_ec_unaligned_vector_ok(ctypes.byref(ok)), "unaligned_vector_ok")
    return bool(ok.value)


def hbm_probe(kind: int, src: int, dst: int, nbytes: int, block: int = 256, waves_per_cu: int = 0,
              stream: int = 0) -> None:
    """Enqueue one HBM ceiling probe (elect_ec_hbm_probe): kind 0 read, 1 write, 2 copy, 3 / 4 the
    decode- / encode-shaped stream mixes (4 streams in, 1 / 2 out); | 0x100 for XCD-major order."""
    check(lib.elect_ec_hbm_probe(kind, src or None, dst, nbytes, block, waves_per_cu, stream or None), "hbm_probe")


def mix_probe(src, dst, chunk_size: int, stripes: int, lengths: int = 0, block: int = 256, waves_per_cu: int = 0,
              stream: int = 0) -> None:
    """Enqueue one stream-mix ceiling probe (elect_ec_mix_probe): src / dst are (ptr, stripe_stride) pairs,
    lengths a device address of [stripes][len(src)] uint32 content lengths or 0."""
    s = (ColumnT * len(src))(*[ColumnT(p, st) for p, st in src])
    d = (ColumnT * len(dst))(*[ColumnT(p, st) for p, st in dst])
    check(lib.elect_ec_mix_probe(len(src), len(dst), chunk_size, stripes, s, lengths or None, d, block, waves_per_cu,
                                 stream or None), "mix_probe")


def set_host_devices(devices) -> None:
    """Spread host-memory calls of different threads over these devices (round robin)."""
    devices = list(devices)
    check(lib.elect_ec_set_host_devices(int_array(devices) if devices else None, len(devices)),
          "set_host_devices")


def set_batching(enable: bool, window_us: int = 0, arena_bytes: int = 256 << 20) -> None:
    """Cross-thread batching of concurrent host-memory encodes/decodes of one shape."""
    check(lib.elect_ec_set_batching(int(enable), window_us, arena_bytes), "set_batching")


def device_numa_node(device: int) -> int:
    """NUMA node of a HIP device (elect_ec_device_numa_node; -1 unknown)."""
    n = ctypes.c_int(-1)
    check(lib.elect_ec_device_numa_node(device, ctypes.byref(n)), "device_numa_node")
    return n.value


def host_device_map(devices, device_nodes, thread_nodes) -> list:
    """The devices threads on thread_nodes would get from devices on device_nodes,
    in that order (elect_ec_host_device_map: the library's NUMA-aware choice)."""
    out = (ctypes.c_int * max(1, len(thread_nodes)))()
    check(lib.elect_ec_host_device_map(int_array(devices), int_array(device_nodes), len(devices),
                                       int_array(thread_nodes) if thread_nodes else None, len(thread_nodes), out),
          "host_device_map")
    return list(out[:len(thread_nodes)])


def pipeline_windows(length: int, steps: int, taper: bool = True) -> list:
    """Window boundaries [0, ..., length] a lone call's units of `length` bytes are pipelined over
    in at most `steps` steps (the library's plan; a test hook, not part of include/elect_ec.h)."""
    at = (ctypes.c_size_t * (steps + 1))()
    n = ctypes.c_int()
    check(lib.elect_ec_internal_pipeline_windows(length, steps, int(taper), at, ctypes.byref(n)), "pipeline_windows")
    return list(at[:n.value + 1])


def host_path_stats() -> dict:
    """The host-memory path's counters (elect_ec_host_path_stats)."""
    out = (ctypes.c_uint64 * 19)()
    lib.elect_ec_host_path_stats(out, 19)
    phases = ("lock", "fill", "queue", "issue", "device", "wake", "unlock")
    return {"zero_copy": out[0], "zero_copy_fallback": out[1], "batched": out[2], "per_thread": out[3],
            "direct": out[4], "registered": out[5], "register_fallback": out[6], "unregister_failures": out[7],
            "register_cpu_ms": round(out[8] * 1e-6, 1), "unregister_cpu_ms": round(out[9] * 1e-6, 1),
            "dispatch_issue_cpu_ms": round(out[10] * 1e-6, 1),
            # wall ms summed over calls (issue, device: over batches), and the batch count
            "phase_ms": {name: round(out[11 + i] * 1e-6, 1) for i, name in enumerate(phases)},
            "batches": out[18]}


def host_alloc(nbytes: int) -> int:
    """Address of an elect_ec_host_alloc buffer of nbytes (page-locked when a device allows)."""
    p = ctypes.c_void_p()
    check(lib.elect_ec_host_alloc(nbytes, ctypes.byref(p)), "host_alloc")
    return p.value


def host_free(addr: int) -> None:
    check(lib.elect_ec_host_free(addr), "host_free")


def host_pinned(addr: int, nbytes: int) -> bool:
    return bool(lib.elect_ec_host_pinned(addr, nbytes))


class HostBuffer:
    """An elect_ec_host_alloc buffer as a numpy uint8 array (what a JVM would wrap in a
    direct ByteBuffer); freed on close(), or by garbage collection once neither the
    HostBuffer nor its .array is referenced (the array keeps its owner alive, so a
    kept array never outlives its memory: ADVICE r4)."""

    def __init__(self, nbytes: int):
        import numpy as np
        self.addr = host_alloc(nbytes)
        self.nbytes = nbytes
        buf = (ctypes.c_ubyte * nbytes).from_address(self.addr)
        buf._owner = self  # array -> buf -> self: the memory stays allocated while the array lives
        self.array = np.ctypeslib.as_array(buf)

    def close(self) -> None:
        if self.addr:
            self.array = None
            host_free(self.addr)
            self.addr = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def ptr_array(addrs) -> ctypes.Array:
    return (ctypes.c_void_p * max(1, len(addrs)))(*addrs)


def int_array(xs) -> ctypes.Array:
    return (ctypes.c_int * max(1, len(xs)))(*[int(x) for x in xs])
