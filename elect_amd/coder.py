"""Python mirror of ELECT's Java coder API (org.apache.cassandra.io.erasurecode)
over the MI355X C ABI.

The reference toolchain (JDK) is absent from this image, so the host side above
the C ABI is mirrored here with the same class names, argument meaning, checks
and exceptions as the Java it stands for:

  ErasureCoderOptions      JEC/ErasureCoderOptions.java
  ErasureCoder             JEC/ErasureCoder.java
  ErasureEncoder           JEC/ErasureEncoder.java:38-71   (encode, encodeUpdate)
  ErasureDecoder           JEC/ErasureDecoder.java:30-39   (decode)
  NativeRSEncoder          JEC/NativeRSEncoder.java        (initImpl/encodeImpl/encodeUpdateImpl/destroyImpl)
  NativeRSDecoder          JEC/NativeRSDecoder.java        (initImpl/decodeImpl/destroyImpl)
  ByteBufferEncodingState  JEC/ByteBufferEncodingState.java:34-72
  ByteBufferDecodingState  JEC/ByteBufferDecodingState.java:36-123
  CoderUtil                JEC/CoderUtil.java
  ByteBuffer               java.nio.ByteBuffer (the subset the coder path uses)

JEC/ = src/elect/src/java/org/apache/cassandra/io/erasurecode.  What the JNI glue
(EC/jni_common.c, EC/NativeRS{En,De}coder.c) did — pointer extraction, count
checks, the native call — is done here through ctypes; the arithmetic runs in
libelect_ec.so's HIP kernels.  RSCoder is the Pythonic handle underneath.
"""
from __future__ import annotations

import threading

import numpy as np

from . import _lib
from ._lib import check, int_array, lib, ptr_array


# ---------------------------------------------------------------------------
# exceptions (org.apache.cassandra.exceptions.ErasureCodeException, java.io.IOException,
# java.lang.InternalError as thrown by EC/jni_common.c:72, 96)
# ---------------------------------------------------------------------------
class ErasureCodeException(RuntimeError):
    pass


class IOException(IOError):
    pass


class InternalError(RuntimeError):
    pass


class NullPointerException(RuntimeError):
    """java.lang.NullPointerException where the Java code dereferences a null
    buffer before its own null check (JEC/ByteBufferDecodingState.java:56-59)."""


# ---------------------------------------------------------------------------
# java.nio.ByteBuffer subset
# ---------------------------------------------------------------------------
class ByteBuffer:
    """Minimal ByteBuffer: a uint8 numpy array with position/limit.  Direct
    buffers are the ones the JNI path addresses (EC/jni_common.c:79)."""

    def __init__(self, array: np.ndarray, direct: bool):
        if array.dtype != np.uint8 or array.ndim != 1 or not array.flags.c_contiguous:
            raise ValueError("ByteBuffer needs a contiguous 1-D uint8 array")
        self._a = array
        self._pos = 0
        self._lim = array.size
        self._direct = direct

    @staticmethod
    def allocateDirect(capacity: int) -> "ByteBuffer":
        return ByteBuffer(np.zeros(capacity, np.uint8), True)

    @staticmethod
    def allocate(capacity: int) -> "ByteBuffer":
        return ByteBuffer(np.zeros(capacity, np.uint8), False)

    @staticmethod
    def wrap(array) -> "ByteBuffer":
        return ByteBuffer(np.ascontiguousarray(np.frombuffer(bytes(array), np.uint8)
                                               if isinstance(array, (bytes, bytearray)) else array,
                                               dtype=np.uint8), False)

    @staticmethod
    def direct_from(array: np.ndarray) -> "ByteBuffer":
        """A direct buffer over existing memory (no copy)."""
        return ByteBuffer(array, True)

    def capacity(self) -> int:
        return self._a.size

    def position(self, new_position: int | None = None):
        if new_position is None:
            return self._pos
        if not 0 <= new_position <= self._lim:
            raise ValueError("position out of range")
        self._pos = new_position
        return self

    def limit(self, new_limit: int | None = None):
        if new_limit is None:
            return self._lim
        if not 0 <= new_limit <= self._a.size:
            raise ValueError("limit out of range")
        self._lim = new_limit
        self._pos = min(self._pos, new_limit)
        return self

    def remaining(self) -> int:
        return self._lim - self._pos

    def rewind(self) -> "ByteBuffer":
        self._pos = 0
        return self

    def flip(self) -> "ByteBuffer":
        self._lim = self._pos
        self._pos = 0
        return self

    def clear(self) -> "ByteBuffer":
        self._pos = 0
        self._lim = self._a.size
        return self

    def isDirect(self) -> bool:
        return self._direct

    def hasArray(self) -> bool:
        return not self._direct

    def arrayOffset(self) -> int:
        return 0

    def array(self) -> np.ndarray:
        return self._a

    def put(self, src) -> "ByteBuffer":
        if isinstance(src, ByteBuffer):
            data = src._a[src._pos:src._lim]
            src._pos = src._lim
        else:
            data = np.frombuffer(bytes(src), np.uint8) if isinstance(src, (bytes, bytearray)) \
                else np.asarray(src, dtype=np.uint8).reshape(-1)
        if data.size > self.remaining():
            raise OverflowError("BufferOverflowException")
        self._a[self._pos:self._pos + data.size] = data
        self._pos += data.size
        return self

    def view(self) -> np.ndarray:
        """The remaining bytes, position..limit (no copy)."""
        return self._a[self._pos:self._lim]

    def address(self) -> int:
        """GetDirectBufferAddress + position, as EC/jni_common.c:79-81 computes."""
        return self._a.ctypes.data + self._pos

    def compareTo(self, other: "ByteBuffer") -> int:
        a = self.view().view(np.int8)
        b = other.view().view(np.int8)
        n = min(a.size, b.size)
        diff = np.nonzero(a[:n] != b[:n])[0]
        if diff.size:
            i = int(diff[0])
            return -1 if a[i] < b[i] else 1
        return (a.size > b.size) - (a.size < b.size)

    def hashCode(self) -> int:
        """java.nio.ByteBuffer.hashCode: h = 1; for i = limit-1 .. position: h = 31*h + b[i]
        over signed bytes, as int32 (ELECT names parity by it,
        ECMessageVerbHandler.java:326-329).  Closed form: 31^n + sum b[i]*31^i mod 2^32."""
        return java_bytebuffer_hash(self.view())


def java_bytebuffer_hash(b: np.ndarray) -> int:
    """Closed form of java.nio.ByteBuffer.hashCode over the bytes b (signed), int32."""
    b = np.ascontiguousarray(b, np.uint8)
    n = b.size
    with np.errstate(over="ignore"):
        pw = np.empty(n + 1, np.uint32)
        pw[0] = 1
        if n:
            pw[1:] = 31
            pw = np.cumprod(pw, dtype=np.uint32)
        sb = b.view(np.int8).astype(np.int64).astype(np.uint32)
        h = (np.sum(sb * pw[:n], dtype=np.uint32) + pw[n]).astype(np.uint32)
    h = int(h)
    return h - (1 << 32) if h >= 1 << 31 else h


# ---------------------------------------------------------------------------
# Pythonic handle over elect_ec_coder
# ---------------------------------------------------------------------------
class RSCoder:
    """An immutable RS(k+m, k) coder (elect_ec_coder_create, include/elect_ec.h)."""

    def __init__(self, k: int, m: int):
        h = _lib.ctypes.c_void_p()
        check(lib.elect_ec_coder_create(k, m, _lib.ctypes.byref(h)), f"create RS({k + m},{k})")
        self.k, self.m = k, m
        self._h = h

    @property
    def handle(self):
        if self._h is None:
            raise IOException("coder closed")
        return self._h

    def close(self):
        if self._h is not None:
            lib.elect_ec_coder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def encode_matrix(self) -> np.ndarray:
        out = np.zeros((self.k + self.m) * self.k, np.uint8)
        check(lib.elect_ec_coder_encode_matrix(self.handle, out.ctypes.data_as(_lib._u8p), out.size))
        return out.reshape(self.k + self.m, self.k)

    def gf_tables(self) -> np.ndarray:
        out = np.zeros(self.m * self.k * 32, np.uint8)
        check(lib.elect_ec_coder_gf_tables(self.handle, out.ctypes.data_as(_lib._u8p), out.size))
        return out

    def decode_matrix(self, decode_indexes, erased, mode: int = _lib.DECODE_COMPAT):
        """(status, num_erased x k matrix); status may be WARN_SINGULAR in compat mode."""
        out = np.zeros(max(1, len(erased)) * self.k, np.uint8)
        st = check(lib.elect_ec_coder_decode_matrix(self.handle, int_array(decode_indexes),
                                                    int_array(erased), len(erased), mode,
                                                    out.ctypes.data_as(_lib._u8p)), "decode matrix")
        return st, out[: len(erased) * self.k].reshape(len(erased), self.k)

    def invert_matrix(self, decode_indexes):
        """(status, k x k inverse of the survivor rows); WARN_SINGULAR with the partial state."""
        out = np.zeros(self.k * self.k, np.uint8)
        st = check(lib.elect_ec_coder_invert_matrix(self.handle, int_array(decode_indexes),
                                                    out.ctypes.data_as(_lib._u8p)), "invert matrix")
        return st, out.reshape(self.k, self.k)

    # host-memory, synchronous (the JNI calling convention)
    def encode_host(self, data_addrs, parity_addrs, length: int) -> int:
        return check(lib.elect_ec_encode(self.handle, ptr_array(data_addrs), ptr_array(parity_addrs),
                                         length), "encode")

    def encode_hashed_host(self, data_addrs, parity_addrs, length: int) -> list:
        """Encode and return each parity unit's java.nio.ByteBuffer.hashCode() (fused)."""
        h = (_lib.ctypes.c_int32 * self.m)()
        check(lib.elect_ec_encode_hashed(self.handle, ptr_array(data_addrs), ptr_array(parity_addrs), length, h),
              "encode_hashed")
        return list(h)

    def encode_padded_host(self, data_addrs, data_lengths, parity_addrs, length: int) -> int:
        """Encode with implicit zero padding to `length` (None address for an all-zero unit)."""
        lens = (_lib.ctypes.c_size_t * len(data_lengths))(*[int(x) for x in data_lengths])
        addrs = [a if a is not None else 0 for a in data_addrs]
        return check(lib.elect_ec_encode_padded(self.handle, ptr_array(addrs), lens, ptr_array(parity_addrs),
                                                length), "encode_padded")

    def encode_ex_host(self, data_addrs, parity_addrs, length: int, data_lengths=None, hashed: bool = False):
        """ELECT's whole coding-node encode step (ECMessageVerbHandler.java:283-329): zero fill
        to `length` (data_lengths; None address for an empty unit), encode, and (hashed) each
        parity unit's ByteBuffer.hashCode().  Returns the hashes, or None."""
        lens = None
        if data_lengths is not None:
            lens = (_lib.ctypes.c_size_t * len(data_lengths))(*[int(x) for x in data_lengths])
        h = (_lib.ctypes.c_int32 * self.m)() if hashed else None
        addrs = [a if a is not None else 0 for a in data_addrs]
        check(lib.elect_ec_encode_ex(self.handle, ptr_array(addrs), lens, ptr_array(parity_addrs), length, h),
              "encode_ex")
        return list(h) if hashed else None

    def encode_update_ex_host(self, in_addrs, target: int, out_addrs, length: int, old_new_lengths=None,
                              hashed: bool = False):
        """ELECT's whole parity-update step (ECParityUpdateVerbHandler.java:634-699): old/new
        zero filled to `length` (old_new_lengths), P' = P ^ E[k+r][target]*(old^new), and
        (hashed) each new parity unit's ByteBuffer.hashCode().  Returns the hashes, or None."""
        lens = None
        if old_new_lengths is not None:
            lens = (_lib.ctypes.c_size_t * 2)(*[int(x) for x in old_new_lengths])
        h = (_lib.ctypes.c_int32 * self.m)() if hashed else None
        addrs = [a if a is not None else 0 for a in in_addrs]
        check(lib.elect_ec_encode_update_ex(self.handle, ptr_array(addrs), lens, target, ptr_array(out_addrs),
                                            length, h), "encode_update_ex")
        return list(h) if hashed else None

    def encode_update_host(self, in_addrs, target: int, out_addrs, length: int) -> int:
        return check(lib.elect_ec_encode_update(self.handle, ptr_array(in_addrs), target,
                                                ptr_array(out_addrs), length), "encodeUpdate")

    def decode_ex_host(self, in_addrs, decode_indexes, erased, out_addrs, length: int, input_lengths=None,
                       mode: int = _lib.DECODE_COMPAT) -> int:
        """ELECT's degraded-read decode (ECRecovery.java:128-149): survivor j holds
        input_lengths[j] content bytes (zero past them; None address for an empty one);
        `length` may be just the prefix of the rebuilt units the caller needs."""
        lens = None
        if input_lengths is not None:
            lens = (_lib.ctypes.c_size_t * len(input_lengths))(*[int(x) for x in input_lengths])
        addrs = [a if a is not None else 0 for a in in_addrs]
        return check(lib.elect_ec_decode_ex(self.handle, ptr_array(addrs), lens, int_array(decode_indexes),
                                            int_array(erased), len(erased), ptr_array(out_addrs), length, mode),
                     "decode_ex")

    def decode_host(self, in_addrs, decode_indexes, erased, out_addrs, length: int,
                    mode: int = _lib.DECODE_COMPAT) -> int:
        return check(lib.elect_ec_decode(self.handle, ptr_array(in_addrs), int_array(decode_indexes),
                                         int_array(erased), len(erased), ptr_array(out_addrs), length,
                                         mode), "decode")


# ---------------------------------------------------------------------------
# CoderUtil (JEC/CoderUtil.java)
# ---------------------------------------------------------------------------
class CoderUtil:
    @staticmethod
    def findFirstValidInput(inputs):
        for x in inputs:
            if x is not None:
                return x
        raise ErasureCodeException("Invalid inputs, all being null!")

    @staticmethod
    def checkEncodeParameters(inputs, outputs, numDataUnits: int, numParityUnits: int):
        # JEC/CoderUtil.java:49-57 (k, or m+2 for encodeUpdate)
        if len(inputs) != numDataUnits and len(inputs) != numParityUnits + 2:
            raise ErasureCodeException("Invalid inputs length for encoding!")
        if len(outputs) != numParityUnits:
            raise ErasureCodeException("Invalid outputs length for encoding!")

    @staticmethod
    def checkDecodeParameters(inputs, erasedIndexes, outputs, numDataUnits: int, numParityUnits: int):
        # JEC/CoderUtil.java:68-83
        if len(inputs) < numDataUnits:
            raise ErasureCodeException("Invalid inputs length for decoding")
        if len(erasedIndexes) != len(outputs):
            raise ErasureCodeException("erasedIndexes and outputs mismatch in length")
        if len(erasedIndexes) > numParityUnits:
            raise ErasureCodeException("Too many erased, not recoverable")

    @staticmethod
    def checkBuffers(buffers, encodeLength: int, usingDirectBuffer: bool):
        # JEC/CoderUtil.java:93-107
        for b in buffers:
            if b is None:
                raise ErasureCodeException("Invalid buffer, being null")
            if b.remaining() != encodeLength:
                raise ErasureCodeException(f"Invalid buffer, not of length {encodeLength}")
            if b.isDirect() != usingDirectBuffer:
                raise ErasureCodeException(f"Invalid buffer, isDirect should be {usingDirectBuffer}")


class ByteBufferEncodingState:
    """JEC/ByteBufferEncodingState.java:34-72."""

    def __init__(self, encoder: "ErasureEncoder", inputs, outputs, usingDirectBuffer: bool = False):
        valid = CoderUtil.findFirstValidInput(inputs)
        self.encodeLength = valid.remaining()
        self.usingDirectBuffer = True if usingDirectBuffer else valid.isDirect()
        self.encoder = encoder
        self.inputs = inputs
        self.outputs = outputs
        CoderUtil.checkEncodeParameters(inputs, outputs, encoder.getNumDataUnits(),
                                        encoder.getNumParityUnits())
        CoderUtil.checkBuffers(inputs, self.encodeLength, self.usingDirectBuffer)
        CoderUtil.checkBuffers(outputs, self.encodeLength, self.usingDirectBuffer)
        self.inputOffsets = [b.arrayOffset() + b.position() if b.hasArray() else b.position()
                             for b in inputs]
        self.outputOffsets = [b.arrayOffset() + b.position() if b.hasArray() else b.position()
                              for b in outputs]


class ByteBufferDecodingState:
    """JEC/ByteBufferDecodingState.java:36-123."""

    def __init__(self, decoder: "ErasureDecoder", inputs, decodeIndexes, erasedIndexes, outputs):
        self.decoder = decoder
        self.inputs = inputs
        self.outputs = outputs
        self.decodeIndexes = list(decodeIndexes)
        self.erasedIndexes = list(erasedIndexes)
        valid = CoderUtil.findFirstValidInput(inputs)
        self.decodeLength = valid.remaining()
        self.usingDirectBuffer = valid.isDirect()
        self.inputOffsets = [b.position() if b is not None else 0 for b in inputs]
        if any(b is None for b in outputs):
            raise NullPointerException("outputs[i].position()")
        self.outputOffsets = [b.position() for b in outputs]
        CoderUtil.checkDecodeParameters(inputs, self.erasedIndexes, outputs,
                                        decoder.getNumDataUnits(), decoder.getNumParityUnits())
        self._checkInputBuffers(inputs)
        self._checkOutputBuffers(outputs)

    def _checkInputBuffers(self, buffers):
        valid = 0
        for b in buffers:
            if b is None:
                continue
            if b.remaining() != self.decodeLength:
                raise ErasureCodeException(f"Invalid buffer, not of length {self.decodeLength}")
            if b.isDirect() != self.usingDirectBuffer:
                raise ErasureCodeException(f"Invalid buffer, isDirect should be {self.usingDirectBuffer}")
            valid += 1
        if valid < self.decoder.getNumDataUnits():
            raise ErasureCodeException("No enough valid inputs are provided, not recoverable")

    def _checkOutputBuffers(self, buffers):
        for b in buffers:
            if b is None:
                raise ErasureCodeException("Invalid buffer found, not allowing null")
            if b.remaining() != self.decodeLength:
                raise ErasureCodeException(f"Invalid buffer, not of length {self.decodeLength}")
            if b.isDirect() != self.usingDirectBuffer:
                raise ErasureCodeException(f"Invalid buffer, isDirect should be {self.usingDirectBuffer}")


# ---------------------------------------------------------------------------
# coder classes
# ---------------------------------------------------------------------------
class ErasureCoderOptions:
    """JEC/ErasureCoderOptions.java."""

    def __init__(self, numDataUnits: int, numParityUnits: int, allowVerboseDump: bool = False):
        self._k = numDataUnits
        self._m = numParityUnits
        self._verbose = allowVerboseDump

    def getNumDataUnits(self) -> int:
        return self._k

    def getNumParityUnits(self) -> int:
        return self._m

    def getNumAllUnits(self) -> int:
        return self._k + self._m

    def allowVerboseDump(self) -> bool:
        return self._verbose


class ErasureCoder:
    """JEC/ErasureCoder.java."""

    def __init__(self, coderOptions: ErasureCoderOptions):
        self._options = coderOptions

    def getNumDataUnits(self) -> int:
        return self._options.getNumDataUnits()

    def getNumParityUnits(self) -> int:
        return self._options.getNumParityUnits()

    def getNumAllUnits(self) -> int:
        return self._options.getNumAllUnits()

    def getOptions(self) -> ErasureCoderOptions:
        return self._options

    def release(self):
        pass

    def allowVerboseDump(self) -> bool:
        return self._options.allowVerboseDump()


class ErasureEncoder(ErasureCoder):
    """JEC/ErasureEncoder.java."""

    def encode(self, inputs, outputs):
        st = ByteBufferEncodingState(self, inputs, outputs, False)
        if st.encodeLength == 0:
            return
        self.doEncode(st)

    def encodeUpdate(self, targetCodingBlock, parityBuffers, targetDataIndex: int):
        st = ByteBufferEncodingState(self, targetCodingBlock, parityBuffers, False)
        if st.encodeLength == 0:
            return
        self.doEncodeUpdate(st, targetDataIndex)

    def doEncode(self, encodingState):
        raise NotImplementedError

    def doEncodeUpdate(self, encodingState, targetDataIndex: int):
        raise NotImplementedError


class ErasureDecoder(ErasureCoder):
    """JEC/ErasureDecoder.java."""

    def decode(self, inputs, decodeIndexes, erasedIndexes, outputs):
        st = ByteBufferDecodingState(self, inputs, decodeIndexes, erasedIndexes, outputs)
        if st.decodeLength == 0:
            return
        self.doDecode(st)

    def doDecode(self, decodingState):
        raise NotImplementedError


class _RWLock:
    """ReentrantReadWriteLock stand-in: many readers or one writer."""

    def __init__(self):
        self._cv = threading.Condition()
        self._readers = 0
        self._writer = False

    def acquire_read(self):
        with self._cv:
            while self._writer:
                self._cv.wait()
            self._readers += 1

    def release_read(self):
        with self._cv:
            self._readers -= 1
            self._cv.notify_all()

    def acquire_write(self):
        with self._cv:
            while self._writer or self._readers:
                self._cv.wait()
            self._writer = True

    def release_write(self):
        with self._cv:
            self._writer = False
            self._cv.notify_all()


def _addresses(buffers, offsets, expected: int, what: str):
    """getInputs/getOutputs (EC/jni_common.c:62-108): count check, then
    GetDirectBufferAddress + offset per buffer."""
    if len(buffers) != expected:
        raise InternalError(f"Invalid {what}")
    out = []
    for b, off in zip(buffers, offsets):
        if b is None:
            out.append(None)
        else:
            out.append(b.array().ctypes.data + off)
    return out


class NativeRSEncoder(ErasureEncoder):
    """JEC/NativeRSEncoder.java over elect_ec_encode / elect_ec_encode_update."""

    def __init__(self, coderOptions: ErasureCoderOptions):
        super().__init__(coderOptions)
        self._lock = _RWLock()
        self._lock.acquire_write()
        try:
            self._coder = RSCoder(coderOptions.getNumDataUnits(), coderOptions.getNumParityUnits())
            self.nativeCoder = 1
        finally:
            self._lock.release_write()
        if self.allowVerboseDump():
            print("Encode matrix:\n", self._coder.encode_matrix())

    def doEncode(self, st: ByteBufferEncodingState):
        self._lock.acquire_read()
        try:
            if self.nativeCoder == 0:
                raise IOException(f"{type(self).__name__} closed")
            k, m = self.getNumDataUnits(), self.getNumParityUnits()
            ins = _addresses(st.inputs, st.inputOffsets, k, "inputs")
            outs = _addresses(st.outputs, st.outputOffsets, m, "outputs")
            self._coder.encode_host(ins, outs, st.encodeLength)
        finally:
            self._lock.release_read()

    def doEncodeUpdate(self, st: ByteBufferEncodingState, targetDataIndex: int):
        self._lock.acquire_read()
        try:
            if self.nativeCoder == 0:
                raise IOException(f"{type(self).__name__} closed")
            m = self.getNumParityUnits()
            ins = _addresses(st.inputs, st.inputOffsets, 2 + m, "inputs")
            outs = _addresses(st.outputs, st.outputOffsets, m, "outputs")
            self._coder.encode_update_host(ins, targetDataIndex, outs, st.encodeLength)
        finally:
            self._lock.release_read()

    def release(self):
        self._lock.acquire_write()
        try:
            if self.nativeCoder:
                self._coder.close()
                self.nativeCoder = 0
        finally:
            self._lock.release_write()


class NativeRSDecoder(ErasureDecoder):
    """JEC/NativeRSDecoder.java over elect_ec_decode.  mode defaults to
    DECODE_COMPAT, bit-exact with libec.so (EC/erasure_coder.c:261-281)."""

    def __init__(self, coderOptions: ErasureCoderOptions, mode: int = _lib.DECODE_COMPAT):
        super().__init__(coderOptions)
        self._lock = _RWLock()
        self._mode = mode
        self.last_status = _lib.OK
        self._lock.acquire_write()
        try:
            self._coder = RSCoder(coderOptions.getNumDataUnits(), coderOptions.getNumParityUnits())
            self.nativeCoder = 1
        finally:
            self._lock.release_write()

    def doDecode(self, st: ByteBufferDecodingState):
        self._lock.acquire_read()
        try:
            if self.nativeCoder == 0:
                raise IOException(f"{type(self).__name__} closed")
            k = self.getNumDataUnits()
            if len(st.decodeIndexes) < k:  # EC/erasure_coder.c:167-169 reads k entries
                raise InternalError("Invalid decodeIndexes")
            ins = _addresses(st.inputs, st.inputOffsets, k, "inputs")
            if any(a is None for a in ins):
                raise InternalError("Invalid inputs")
            outs = _addresses(st.outputs, st.outputOffsets, len(st.erasedIndexes), "outputs")
            if self.allowVerboseDump():
                print("Decode matrix:\n",
                      self._coder.decode_matrix(st.decodeIndexes[:k], st.erasedIndexes, self._mode)[1])
            self.last_status = self._coder.decode_host(ins, st.decodeIndexes[:k], st.erasedIndexes,
                                                       outs, st.decodeLength, self._mode)
        finally:
            self._lock.release_read()

    def release(self):
        self._lock.acquire_write()
        try:
            if self.nativeCoder:
                self._coder.close()
                self.nativeCoder = 0
        finally:
            self._lock.release_write()
