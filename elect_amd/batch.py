"""Device-resident batched API over torch tensors (PyTorch is only the
allocator and stream provider here; every byte is coded by libelect_ec.so).

Layout convention: a batch is a uint8 tensor shaped [stripes, shards, L] (any
strides on the first two dims, contiguous last dim) on a HIP device.  A shard
row s,i starts at data_ptr + s*stride(0) + i*stride(1).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import ColumnT, Shards, check, int_array, lib
from .coder import RSCoder


def _shards(t: torch.Tensor) -> Shards:
    if t.dtype != torch.uint8 or t.dim() != 3 or t.stride(2) != 1:
        raise ValueError("expected a uint8 [stripes, shards, L] tensor with a contiguous last dim")
    if t.device.type != "cuda":
        raise ValueError("device-resident API needs a HIP (cuda) tensor")
    return Shards(t.data_ptr(), t.stride(0), t.stride(1))


def _column(t: torch.Tensor) -> ColumnT:
    if t.dtype != torch.uint8 or t.dim() != 2 or t.stride(1) != 1 or t.device.type != "cuda":
        raise ValueError("expected a uint8 [stripes, L] HIP tensor with a contiguous last dim")
    return ColumnT(t.data_ptr(), t.stride(0))


def _rows(name: str, t: torch.Tensor, B: int, L: int, need: int) -> None:
    """t must be [B, >= need, L]: the C ABI addresses it from its strides alone, so a
    tensor of another shape would be read or written out of bounds on the device."""
    if t.dim() != 3 or t.shape[0] != B or t.shape[2] != L or t.shape[1] < need:
        raise ValueError(f"{name}: expected [{B}, >={need}, {L}], got {tuple(t.shape)}")


def _encode_shapes(coder, data, parity):
    """data must be [B, k, L] and parity [B, >= m, L] (see _rows); returns B, L."""
    if data.dim() != 3 or data.shape[1] != coder.k:
        raise ValueError(f"data: expected a [stripes, {coder.k}, L] tensor, got {tuple(data.shape)}")
    B, _, L = data.shape
    _rows("parity", parity, B, L, coder.m)
    return B, L


def _decode_shapes(coder, inputs, decode_indexes, erased, outputs, inputs_by_unit, outputs_by_unit):
    if len(decode_indexes) != coder.k:
        raise ValueError("decode_indexes needs exactly k entries")
    if inputs.dim() != 3:
        raise ValueError(f"inputs: expected a [stripes, units, L] tensor, got {tuple(inputs.shape)}")
    B, _, L = inputs.shape
    _rows("inputs", inputs, B, L, max(decode_indexes) + 1 if inputs_by_unit else coder.k)
    _rows("outputs", outputs, B, L, max(erased) + 1 if outputs_by_unit and len(erased) else len(erased))
    return B, L


def _stream(stream) -> int:
    if stream is None:
        stream = torch.cuda.current_stream()
    return stream.cuda_stream


def encode_batch(coder: RSCoder, data: torch.Tensor, parity: torch.Tensor, stream=None) -> None:
    """parity[s, r] = XOR_j E[k+r][j] * data[s, j] for every stripe s (stream ordered)."""
    B, k, L = data.shape
    if k != coder.k or parity.shape[0] != B or parity.shape[1] != coder.m or parity.shape[2] != L:
        raise ValueError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)}")
    check(lib.elect_ec_encode_batch(coder.handle, L, B, _shards(data), _shards(parity), _stream(stream)),
          "encode_batch")


def encode_batch_hashed(coder: RSCoder, data: torch.Tensor, parity: torch.Tensor, hashes: torch.Tensor,
                        stream=None) -> None:
    """encode_batch that also writes every parity unit's java.nio.ByteBuffer.hashCode()
    into hashes (int32 device tensor [B, m])."""
    B, L = _encode_shapes(coder, data, parity)
    if hashes.shape != (B, coder.m) or hashes.dtype != torch.int32 or not hashes.is_contiguous():
        raise ValueError("hashes must be a contiguous int32 [B, m] tensor")
    check(lib.elect_ec_encode_batch_hashed(coder.handle, L, B, _shards(data), _shards(parity), hashes.data_ptr(),
                                           _stream(stream)), "encode_batch_hashed")


def encode_batch_padded(coder: RSCoder, data: torch.Tensor, lengths: torch.Tensor, parity: torch.Tensor,
                        stream=None) -> None:
    """encode_batch where data[s, j] holds only lengths[s, j] valid bytes (int32/uint32
    device tensor [B, k]); the rest reads as zero and is never loaded."""
    B, L = _encode_shapes(coder, data, parity)
    k = coder.k
    if lengths.shape != (B, k) or lengths.dtype not in (torch.int32, torch.uint32) or \
            not lengths.is_contiguous() or lengths.device != data.device:
        raise ValueError("lengths must be a contiguous int32 [B, k] tensor on the data's device")
    check(lib.elect_ec_encode_batch_padded(coder.handle, L, B, _shards(data), lengths.data_ptr(),
                                           _shards(parity), _stream(stream)), "encode_batch_padded")


def decode_batch(coder: RSCoder, inputs: torch.Tensor, decode_indexes, erased, outputs: torch.Tensor,
                 mode: int = _lib.DECODE_COMPAT, inputs_by_unit: bool = False,
                 outputs_by_unit: bool = False, stream=None) -> int:
    """Reconstruct `erased` units of every stripe from k survivors.

    inputs: [B, k, L] survivors in decode_indexes order, or (inputs_by_unit)
    a [B, k+m, L] stripe tensor read at rows decode_indexes.  outputs: [B, e, L],
    or (outputs_by_unit) the stripe tensor, written at rows erased."""
    B, L = _decode_shapes(coder, inputs, decode_indexes, erased, outputs, inputs_by_unit, outputs_by_unit)
    flags = (_lib.INPUTS_BY_UNIT if inputs_by_unit else 0) | (_lib.OUTPUTS_BY_UNIT if outputs_by_unit else 0)
    return check(lib.elect_ec_decode_batch(coder.handle, L, B, _shards(inputs), int_array(decode_indexes),
                                           int_array(erased), len(erased), _shards(outputs), flags, mode,
                                           _stream(stream)), "decode_batch")


def decode_batch_ex(coder: RSCoder, inputs: torch.Tensor, decode_indexes, erased, outputs: torch.Tensor,
                    lengths=None, mode: int = _lib.DECODE_COMPAT, inputs_by_unit: bool = False,
                    outputs_by_unit: bool = False, stream=None) -> int:
    """decode_batch over zero-padded survivors (ECRecovery.java:128-141): lengths[s, j] content
    bytes of survivor j (decode_indexes order; int32 device tensor [B, k], each <= L)."""
    B, L = _decode_shapes(coder, inputs, decode_indexes, erased, outputs, inputs_by_unit, outputs_by_unit)
    flags = (_lib.INPUTS_BY_UNIT if inputs_by_unit else 0) | (_lib.OUTPUTS_BY_UNIT if outputs_by_unit else 0)
    return check(lib.elect_ec_decode_batch_ex(coder.handle, L, B, _shards(inputs),
                                              _lengths(lengths, B, coder.k, inputs.device),
                                              int_array(decode_indexes), int_array(erased), len(erased),
                                              _shards(outputs), flags, mode, _stream(stream)), "decode_batch_ex")


def encode_update_batch(coder: RSCoder, target: int, old: torch.Tensor, new: torch.Tensor,
                        parity_in: torch.Tensor, parity_out: torch.Tensor, stream=None) -> None:
    """parity_out[s, r] = parity_in[s, r] ^ E[k+r][target] * (old[s] ^ new[s]); in place allowed."""
    B, L = _update_shapes(coder, old, new, parity_in, parity_out)
    check(lib.elect_ec_encode_update_batch(coder.handle, L, B, target, _column(old), _column(new),
                                           _shards(parity_in), _shards(parity_out), _stream(stream)),
          "encode_update_batch")


def _update_shapes(coder, old, new, parity_in, parity_out):
    if old.dim() != 2 or new.shape != old.shape:
        raise ValueError(f"old/new: expected two [stripes, L] tensors, got {tuple(old.shape)} {tuple(new.shape)}")
    B, L = old.shape
    _rows("parity_in", parity_in, B, L, coder.m)
    _rows("parity_out", parity_out, B, L, coder.m)
    return B, L


def _lengths(lengths, B: int, n: int, device) -> int:
    if lengths is None:
        return None
    if lengths.shape != (B, n) or lengths.dtype not in (torch.int32, torch.uint32) or \
            not lengths.is_contiguous() or lengths.device != device:
        raise ValueError(f"lengths must be a contiguous int32 [{B}, {n}] tensor on the data's device")
    return lengths.data_ptr()


def _hashes(hashes, B: int, m: int, device) -> int:
    if hashes is None:
        return None
    if hashes.shape != (B, m) or hashes.dtype != torch.int32 or not hashes.is_contiguous() or \
            hashes.device != device:
        raise ValueError(f"hashes must be a contiguous int32 [{B}, {m}] tensor on the data's device")
    return hashes.data_ptr()


def encode_batch_ex(coder: RSCoder, data: torch.Tensor, parity: torch.Tensor, lengths=None, hashes=None,
                    stream=None) -> None:
    """ELECT's coding-node encode step in one launch (ECMessageVerbHandler.java:283-329):
    data[s, j] holds lengths[s, j] content bytes (None: all full; the rest reads as zero),
    and hashes[s, r] (None: not wanted) receives parity[s, r]'s ByteBuffer.hashCode()."""
    B, k, L = data.shape
    if k != coder.k or parity.shape != (B, coder.m, L):
        raise ValueError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)}")
    check(lib.elect_ec_encode_batch_ex(coder.handle, L, B, _shards(data), _lengths(lengths, B, k, data.device),
                                       _shards(parity), _hashes(hashes, B, coder.m, data.device), _stream(stream)),
          "encode_batch_ex")


def encode_update_batch_ex(coder: RSCoder, target: int, old: torch.Tensor, new: torch.Tensor,
                           parity_in: torch.Tensor, parity_out: torch.Tensor, lengths=None, hashes=None,
                           stream=None) -> None:
    """ELECT's parity-update step in one launch (ECParityUpdateVerbHandler.java:634-699):
    old[s] / new[s] hold lengths[s, 0] / lengths[s, 1] content bytes (None: full), the
    new parity goes to parity_out (may be parity_in) and its hashCode() to hashes[s, r]."""
    B, L = _update_shapes(coder, old, new, parity_in, parity_out)
    check(lib.elect_ec_encode_update_batch_ex(coder.handle, L, B, target, _column(old), _column(new),
                                              _lengths(lengths, B, 2, old.device), _shards(parity_in),
                                              _shards(parity_out), _hashes(hashes, B, coder.m, old.device),
                                              _stream(stream)),
          "encode_update_batch_ex")


def _tiles_of(chunk_size: int, tile: int, rows: int) -> int:
    """Stripes in a tiled batch whose coding view has `rows` tile rows."""
    if tile <= 0:
        raise ValueError(f"a tiled view needs a positive tile length, got {tile}")
    t = max(1, -(-chunk_size // tile))
    if rows % t:
        raise ValueError(f"a tiled view needs a multiple of {t} tile rows (ceil({chunk_size}/{tile})), got {rows}")
    return rows // t


def encode_batch_tiled(coder: RSCoder, data: torch.Tensor, parity: torch.Tensor, chunk_size: int, lengths=None,
                       hashes=None, stream=None) -> None:
    """encode_batch_ex over tiled units: data [B*T, k, tile] / parity [B*T, m, tile] views
    where stripe s's unit j is tiles s*T .. s*T+T-1 of column j (T = ceil(chunk_size/tile));
    lengths [B, k] and hashes [B, m] are per stripe (include/elect_ec.h, tiled units)."""
    rows, k, tile = data.shape
    B = _tiles_of(chunk_size, tile, rows)
    if k != coder.k or parity.shape != (rows, coder.m, tile):
        raise ValueError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)}")
    check(lib.elect_ec_encode_batch_tiled(coder.handle, chunk_size, tile, B, _shards(data),
                                          _lengths(lengths, B, k, data.device), _shards(parity),
                                          _hashes(hashes, B, coder.m, data.device), _stream(stream)),
          "encode_batch_tiled")


def encode_update_batch_tiled(coder: RSCoder, target: int, old: torch.Tensor, new: torch.Tensor,
                              parity_in: torch.Tensor, parity_out: torch.Tensor, chunk_size: int, lengths=None,
                              hashes=None, stream=None) -> None:
    """encode_update_batch_ex over tiled units: old/new [B*T, tile], parity [B*T, m, tile]."""
    rows, tile = _update_shapes(coder, old, new, parity_in, parity_out)
    B = _tiles_of(chunk_size, tile, rows)
    check(lib.elect_ec_encode_update_batch_tiled(coder.handle, chunk_size, tile, B, target, _column(old), _column(new),
                                                 _lengths(lengths, B, 2, old.device), _shards(parity_in),
                                                 _shards(parity_out), _hashes(hashes, B, coder.m, old.device),
                                                 _stream(stream)),
          "encode_update_batch_tiled")


def decode_batch_tiled(coder: RSCoder, inputs: torch.Tensor, decode_indexes, erased, outputs: torch.Tensor,
                       chunk_size: int, lengths=None, mode: int = _lib.DECODE_COMPAT, inputs_by_unit: bool = False,
                       outputs_by_unit: bool = False, stream=None) -> int:
    """decode_batch_ex over tiled units: inputs [B*T, k or k+m, tile], outputs [B*T, e or k+m, tile]."""
    rows, tile = _decode_shapes(coder, inputs, decode_indexes, erased, outputs, inputs_by_unit, outputs_by_unit)
    B = _tiles_of(chunk_size, tile, rows)
    flags = (_lib.INPUTS_BY_UNIT if inputs_by_unit else 0) | (_lib.OUTPUTS_BY_UNIT if outputs_by_unit else 0)
    return check(lib.elect_ec_decode_batch_tiled(coder.handle, chunk_size, tile, B, _shards(inputs),
                                                 _lengths(lengths, B, coder.k, inputs.device),
                                                 int_array(decode_indexes), int_array(erased), len(erased),
                                                 _shards(outputs), flags, mode, _stream(stream)),
                 "decode_batch_tiled")


def encode_batches(coder: RSCoder, pairs, stream=None) -> None:
    """encode_batch over several (data [B_i, k, L_i], parity [B_i, m, L_i]) pairs of different
    chunk sizes in as few launches as possible (elect_ec_encode_batches)."""
    arr = (_lib.BatchT * max(1, len(pairs)))()
    for i, (data, parity) in enumerate(pairs):
        B, k, L = data.shape
        if k != coder.k or parity.shape != (B, coder.m, L):
            raise ValueError(f"shape mismatch: data {tuple(data.shape)} parity {tuple(parity.shape)}")
        arr[i] = _lib.BatchT(L, B, _shards(data), _shards(parity))
    check(lib.elect_ec_encode_batches(coder.handle, arr, len(pairs), _stream(stream)), "encode_batches")


def decode_batches(coder: RSCoder, pairs, decode_indexes, erased, mode: int = _lib.DECODE_COMPAT,
                   inputs_by_unit: bool = False, outputs_by_unit: bool = False, stream=None) -> int:
    """decode_batch over several (inputs, outputs) pairs with one erasure pattern (elect_ec_decode_batches)."""
    if len(decode_indexes) != coder.k:
        raise ValueError("decode_indexes needs exactly k entries")
    arr = (_lib.BatchT * max(1, len(pairs)))()
    for i, (inputs, outputs) in enumerate(pairs):
        B, L = _decode_shapes(coder, inputs, decode_indexes, erased, outputs, inputs_by_unit, outputs_by_unit)
        arr[i] = _lib.BatchT(L, B, _shards(inputs), _shards(outputs))
    flags = (_lib.INPUTS_BY_UNIT if inputs_by_unit else 0) | (_lib.OUTPUTS_BY_UNIT if outputs_by_unit else 0)
    return check(lib.elect_ec_decode_batches(coder.handle, arr, len(pairs), int_array(decode_indexes),
                                             int_array(erased), len(erased), flags, mode, _stream(stream)),
                 "decode_batches")


def apply_batch(coef: np.ndarray, src, dst, stream=None) -> None:
    """dst[r] = XOR_j coef[r, j] * src[j] over [B, L] column tensors."""
    coef = np.ascontiguousarray(coef, np.uint8)
    rows, cols = coef.shape
    if len(src) != cols or len(dst) != rows:
        raise ValueError(f"apply_batch: {cols} source and {rows} output columns expected, got {len(src)} / {len(dst)}")
    B, L = src[0].shape
    if any(t.dim() != 2 or tuple(t.shape) != (B, L) for t in list(src) + list(dst)):
        raise ValueError(f"apply_batch: every column must be [{B}, {L}]")
    s = (ColumnT * cols)(*[_column(t) for t in src])
    d = (ColumnT * rows)(*[_column(t) for t in dst])
    check(lib.elect_ec_apply_batch(coef.ctypes.data_as(_lib._u8p), rows, cols, L, B, s, d, _stream(stream)),
          "apply_batch")


def partition_by_bytes(sizes, world: int, rank: int):
    """Contiguous block of work items for `rank` so that every rank gets about
    the same number of bytes (stripes are independent: no exchange step).
    sizes: bytes per item, in order.  Returns (begin, end)."""
    sizes = np.asarray(sizes, dtype=np.int64)
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad world/rank")
    if sizes.size == 0:
        return 0, 0
    cum = np.concatenate([[0], np.cumsum(sizes)])
    total = cum[-1]
    bounds = []
    for r in range(world + 1):
        target = total * r / world
        i = int(np.searchsorted(cum, target, side="left"))
        if 0 < i <= sizes.size and target - cum[i - 1] < cum[i] - target:
            i -= 1  # nearer boundary: ranks differ by at most one stripe's bytes
        bounds.append(i)
    bounds[0], bounds[-1] = 0, sizes.size
    for i in range(1, world + 1):
        bounds[i] = max(bounds[i], bounds[i - 1])
    return bounds[rank], bounds[rank + 1]
