"""ctypes wrapper over oracle/libec_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module.  PARITY UNPINNED: see ec_oracle.h.  Every function here forwards to the C
restatement whose header cites the reference (EC/erasure_coder.c) line it follows.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libec_oracle.so")
_lib = None

u8p = ctypes.POINTER(ctypes.c_ubyte)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_gf_mul.restype = ctypes.c_ubyte
        L.oracle_gf_mul.argtypes = [ctypes.c_ubyte, ctypes.c_ubyte]
        L.oracle_gf_inv.restype = ctypes.c_ubyte
        L.oracle_gf_inv.argtypes = [ctypes.c_ubyte]
        L.oracle_gf_exp_table.restype = u8p
        L.oracle_gf_log_table.restype = u8p
        L.oracle_gf_gen_cauchy1_matrix.argtypes = [u8p, ctypes.c_int, ctypes.c_int]
        L.oracle_ec_init_tables.argtypes = [ctypes.c_int, ctypes.c_int, u8p, u8p]
        L.oracle_ec_encode_data.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, u8p,
                                            ctypes.POINTER(u8p), ctypes.POINTER(u8p)]
        L.oracle_gf_invert_matrix.argtypes = [u8p, u8p, ctypes.c_int]
        L.oracle_gf_invert_matrix.restype = ctypes.c_int
        L.oracle_encoder_init.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        L.oracle_encode.argtypes = [ctypes.c_void_p, ctypes.POINTER(u8p), ctypes.POINTER(u8p),
                                    ctypes.c_int]
        L.oracle_encode_update.argtypes = [ctypes.c_void_p, ctypes.POINTER(u8p), ctypes.c_int,
                                           ctypes.POINTER(u8p), ctypes.c_int]
        L.oracle_decode_matrix.argtypes = [ctypes.c_int, ctypes.c_int, u8p,
                                           ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_int), ctypes.c_int,
                                           ctypes.c_int, u8p]
        L.oracle_decode_matrix.restype = ctypes.c_int
        L.oracle_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(u8p),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                    ctypes.c_int, ctypes.POINTER(u8p), ctypes.c_int,
                                    ctypes.c_int]
        L.oracle_decode.restype = ctypes.c_int
        L.oracle_simd_best.restype = ctypes.c_int
        L.oracle_simd_name.restype = ctypes.c_char_p
        L.oracle_simd_name.argtypes = [ctypes.c_int]
        L.oracle_ec_encode_data_simd.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                                 ctypes.c_int, u8p, ctypes.POINTER(u8p),
                                                 ctypes.POINTER(u8p)]
        L.oracle_batch_apply.restype = ctypes.c_double
        L.oracle_batch_apply.argtypes = [ctypes.c_int, ctypes.c_int, u8p, ctypes.c_int,
                                         ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_int64), ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]
        L.oracle_java_bytebuffer_hashcode.restype = ctypes.c_int32
        L.oracle_java_bytebuffer_hashcode.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_fill_splitmix.argtypes = [ctypes.c_uint64, u8p, ctypes.c_size_t]
        _lib = L
    return _lib


# sizeof(oracle_encoder) = 2 ints + 140 + 4480 bytes (no padding beyond int alignment)
_ENC_BYTES = 8 + 14 * 10 + 14 * 10 * 32 + 8


def _p(a: np.ndarray):
    return a.ctypes.data_as(u8p)


def _ptrs(arrs):
    return (u8p * len(arrs))(*[_p(a) for a in arrs])


def _ints(xs):
    return (ctypes.c_int * max(1, len(xs)))(*xs)


def gf_mul(a: int, b: int) -> int:
    return lib().oracle_gf_mul(a, b)


def gf_inv(a: int) -> int:
    return lib().oracle_gf_inv(a)


def exp_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().oracle_gf_exp_table(), shape=(256,)).copy()


def log_table() -> np.ndarray:
    return np.ctypeslib.as_array(lib().oracle_gf_log_table(), shape=(256,)).copy()


def cauchy_matrix(k: int, m: int) -> np.ndarray:
    a = np.zeros((k + m) * k, np.uint8)
    lib().oracle_gf_gen_cauchy1_matrix(_p(a), k + m, k)
    return a.reshape(k + m, k)


def init_tables(coef: np.ndarray) -> np.ndarray:
    coef = np.ascontiguousarray(coef, np.uint8)
    rows, k = coef.shape
    t = np.zeros(rows * k * 32, np.uint8)
    lib().oracle_ec_init_tables(k, rows, _p(coef), _p(t))
    return t


def invert_matrix(mat: np.ndarray):
    n = mat.shape[0]
    a = np.ascontiguousarray(mat, np.uint8).copy()
    out = np.zeros((n, n), np.uint8)
    rc = lib().oracle_gf_invert_matrix(_p(a), _p(out), n)
    return rc, out


def apply(coef: np.ndarray, src) -> list:
    """ec_encode_data (scalar base restatement): rows x k coefficients over k sources."""
    coef = np.ascontiguousarray(coef, np.uint8)
    rows, k = coef.shape
    src = [np.ascontiguousarray(s, np.uint8) for s in src]
    n = len(src[0]) if src else 0
    dst = [np.empty(n, np.uint8) for _ in range(rows)]
    t = init_tables(coef)
    lib().oracle_ec_encode_data(n, k, rows, _p(t), _ptrs(src), _ptrs(dst))
    return dst


def apply_simd(coef: np.ndarray, src, level: int | None = None) -> list:
    coef = np.ascontiguousarray(coef, np.uint8)
    rows, k = coef.shape
    src = [np.ascontiguousarray(s, np.uint8) for s in src]
    n = len(src[0]) if src else 0
    dst = [np.empty(n, np.uint8) for _ in range(rows)]
    t = init_tables(coef)
    if level is None:
        level = simd_best()
    lib().oracle_ec_encode_data_simd(level, n, k, rows, _p(t), _ptrs(src), _ptrs(dst))
    return dst


class Encoder:
    """ELECT initEncoder/encode/encodeUpdate (EC/erasure_coder.c:49-142), restated."""

    def __init__(self, k: int, m: int):
        self.k, self.m = k, m
        self._buf = ctypes.create_string_buffer(_ENC_BYTES)
        if lib().oracle_encoder_init(self._buf, k, m) != 0:
            raise ValueError(f"bad (k,m)=({k},{m})")

    def encode(self, data) -> list:
        data = [np.ascontiguousarray(d, np.uint8) for d in data]
        n = len(data[0])
        par = [np.empty(n, np.uint8) for _ in range(self.m)]
        lib().oracle_encode(self._buf, _ptrs(data), _ptrs(par), n)
        return par

    def encode_update(self, old_new_parity, target: int) -> list:
        ins = [np.ascontiguousarray(d, np.uint8) for d in old_new_parity]
        n = len(ins[0])
        out = [np.empty(n, np.uint8) for _ in range(self.m)]
        lib().oracle_encode_update(self._buf, _ptrs(ins), target, _ptrs(out), n)
        return out


def decode_matrix(k: int, m: int, decode_indexes, erased, strict: bool = False):
    em = cauchy_matrix(k, m).reshape(-1).copy()
    out = np.zeros(max(1, len(erased)) * k, np.uint8)
    rc = lib().oracle_decode_matrix(k, m, _p(em), _ints(decode_indexes), _ints(erased),
                                    len(erased), int(strict), _p(out))
    return rc, out[: len(erased) * k].reshape(len(erased), k)


def decode(k: int, m: int, inputs, decode_indexes, erased, strict: bool = False):
    ins = [np.ascontiguousarray(d, np.uint8) for d in inputs]
    n = len(ins[0])
    outs = [np.empty(n, np.uint8) for _ in range(len(erased))]
    rc = lib().oracle_decode(k, m, _ptrs(ins), _ints(decode_indexes), _ints(erased),
                             len(erased), _ptrs(outs), n, int(strict))
    return rc, outs


def simd_best() -> int:
    return lib().oracle_simd_best()


def simd_name(level: int) -> str:
    return lib().oracle_simd_name(level).decode()


def batch_apply(coef: np.ndarray, src: np.ndarray, src_stripe: int, src_col_off, dst: np.ndarray,
                dst_stripe: int, dst_row_off, length: int, stripes: int, threads: int,
                level: int | None = None) -> float:
    """Threaded strided batch (CPU baseline).  Returns wall seconds."""
    coef = np.ascontiguousarray(coef, np.uint8)
    rows, k = coef.shape
    if level is None:
        level = simd_best()
    so = (ctypes.c_int64 * k)(*[int(x) for x in src_col_off])
    do = (ctypes.c_int64 * rows)(*[int(x) for x in dst_row_off])
    return lib().oracle_batch_apply(level, threads, _p(coef), rows, k, length, stripes,
                                    src.ctypes.data, src_stripe, so, dst.ctypes.data,
                                    dst_stripe, do)


def splitmix_bytes(seed: int, n: int) -> np.ndarray:
    out = np.empty(n, np.uint8)
    lib().oracle_fill_splitmix(ctypes.c_uint64(seed), _p(out), n)
    return out


def fill_splitmix(seed: int, out: np.ndarray) -> None:
    """Fill a contiguous uint8 array in place with the splitmix64 stream."""
    assert out.dtype == np.uint8 and out.flags.c_contiguous
    lib().oracle_fill_splitmix(ctypes.c_uint64(seed), _p(out.reshape(-1)), out.size)


def java_hashcode(b) -> int:
    """java.nio.ByteBuffer.hashCode() of the bytes b (JDK loop; ECMessageVerbHandler.java:328)."""
    b = np.ascontiguousarray(b, np.uint8)
    return int(lib().oracle_java_bytebuffer_hashcode(_p(b) if b.size else None, b.size))


def zero_fill(content, code_length: int) -> np.ndarray:
    """ELECT's SSTable buffer: allocateDirect(codeLength).put(content).put(zeros)
    (ECMessageVerbHandler.java:292-310, ECParityUpdateVerbHandler.java:643-663)."""
    out = np.zeros(code_length, np.uint8)
    content = np.asarray(content, np.uint8)
    out[: content.size] = content
    return out
