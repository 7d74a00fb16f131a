"""CPU: the Python mirror of the Java coder API raises what the Java does, in
the same order, before any native compute (JEC/CoderUtil.java,
JEC/ByteBuffer{En,De}codingState.java, JEC/NativeRS{En,De}coder.java,
EC/jni_common.c:62-108)."""
import numpy as np
import pytest

from elect_amd.coder import (ByteBuffer, ErasureCodeException, ErasureCoderOptions, InternalError,
                             IOException, NativeRSDecoder, NativeRSEncoder, NullPointerException)


def bufs(n, size, direct=True):
    return [(ByteBuffer.allocateDirect if direct else ByteBuffer.allocate)(size) for _ in range(n)]


def test_options():
    o = ErasureCoderOptions(4, 2)
    assert (o.getNumDataUnits(), o.getNumParityUnits(), o.getNumAllUnits(), o.allowVerboseDump()) == \
        (4, 2, 6, False)


def test_encode_parameter_checks():
    enc = NativeRSEncoder(ErasureCoderOptions(4, 2))
    with pytest.raises(ErasureCodeException, match="Invalid inputs length for encoding"):
        enc.encode(bufs(3, 16), bufs(2, 16))
    with pytest.raises(ErasureCodeException, match="Invalid outputs length for encoding"):
        enc.encode(bufs(4, 16), bufs(3, 16))
    with pytest.raises(ErasureCodeException, match="Invalid buffer, not of length 16"):
        enc.encode(bufs(4, 16), bufs(1, 16) + bufs(1, 17))
    with pytest.raises(ErasureCodeException, match="isDirect should be True"):
        enc.encode(bufs(3, 16) + bufs(1, 16, direct=False), bufs(2, 16))
    with pytest.raises(ErasureCodeException, match="all being null"):
        enc.encode([None] * 4, bufs(2, 16))
    # k == m + 2 is accepted by CoderUtil (JEC/CoderUtil.java:50) for encode...
    # ...but with m + 2 != k the JNI count check rejects it (EC/jni_common.c:70-73)
    enc6 = NativeRSEncoder(ErasureCoderOptions(6, 2))
    with pytest.raises(InternalError, match="Invalid inputs"):
        enc6.encode(bufs(4, 16), bufs(2, 16))


def test_zero_length_is_a_noop():
    enc = NativeRSEncoder(ErasureCoderOptions(4, 2))
    enc.encode(bufs(4, 0), bufs(2, 0))  # JEC/ErasureEncoder.java:41-44 — returns before native
    dec = NativeRSDecoder(ErasureCoderOptions(4, 2))
    dec.decode(bufs(4, 0), [1, 2, 3, 4], [0], bufs(1, 0))


def test_decode_parameter_checks():
    dec = NativeRSDecoder(ErasureCoderOptions(4, 2))
    with pytest.raises(ErasureCodeException, match="Invalid inputs length for decoding"):
        dec.decode(bufs(3, 16), [1, 2, 3], [0], bufs(1, 16))
    with pytest.raises(ErasureCodeException, match="mismatch in length"):
        dec.decode(bufs(4, 16), [1, 2, 3, 4], [0, 5], bufs(1, 16))
    with pytest.raises(ErasureCodeException, match="Too many erased"):
        dec.decode(bufs(6, 16), [1, 2, 3, 4], [0, 5, 4], bufs(3, 16))
    with pytest.raises(ErasureCodeException, match="No enough valid inputs"):
        dec.decode(bufs(3, 16) + [None, None], [1, 2, 3, 4], [0], bufs(1, 16))
    # Java reads outputs[i].position() before checkOutputBuffers' null check
    with pytest.raises(NullPointerException):
        dec.decode(bufs(4, 16), [1, 2, 3, 4], [0], [None])


def test_release_then_use_raises_ioexception():
    enc = NativeRSEncoder(ErasureCoderOptions(4, 2))
    enc.release()
    enc.release()  # destroyImpl on a closed coder is a no-op (EC/NativeRSEncoder.c:90-94)
    with pytest.raises(IOException, match="NativeRSEncoder closed"):
        enc.encode(bufs(4, 16), bufs(2, 16))
    dec = NativeRSDecoder(ErasureCoderOptions(4, 2))
    dec.release()
    with pytest.raises(IOException, match="NativeRSDecoder closed"):
        dec.decode(bufs(4, 16), [1, 2, 3, 4], [0], bufs(1, 16))


def test_bytebuffer_semantics():
    b = ByteBuffer.allocateDirect(8)
    b.put(bytes(range(8)))
    assert b.remaining() == 0
    b.rewind()
    assert b.remaining() == 8 and b.isDirect()
    c = ByteBuffer.direct_from(np.arange(8, dtype=np.uint8))
    assert b.compareTo(c) == 0
    c.array()[3] = 0x80  # signed compare: -128 < 3
    assert b.compareTo(c) == 1
    # java.nio.ByteBuffer.hashCode over signed bytes, from the limit down
    h = 1
    for x in reversed([0, 1, 2, 3, 4, 5, 6, 7]):
        h = (31 * h + x) & 0xFFFFFFFF
    assert b.hashCode() == (h - (1 << 32) if h >= 1 << 31 else h)
    assert ByteBuffer.direct_from(np.array([0x80, 0xFF], np.uint8)).hashCode() == 31 * 31 + 31 * (-1) + (-128)
    w = ByteBuffer.wrap(b"\x01\x02")
    assert not w.isDirect() and w.hasArray()


def test_java_hash_closed_form_equals_jdk_loop():
    """The vectorised closed form used everywhere equals the JDK loop literally."""
    from elect_amd.coder import java_bytebuffer_hash
    rng = np.random.default_rng(3)
    for n in (0, 1, 2, 15, 16, 17, 100, 1031):
        b = rng.integers(0, 256, n, dtype=np.uint8)
        h = 1
        for x in b[::-1].view(np.int8):
            h = (31 * h + int(x)) & 0xFFFFFFFF
        h = h - (1 << 32) if h >= 1 << 31 else h
        assert java_bytebuffer_hash(b) == h


def test_cpp_mirror_error_behaviour():
    """include/elect_ec.hpp (C++ mirror of the Java API): same checks and exceptions."""
    import subprocess
    from tests.cpp_build import build
    r = subprocess.run([build(), "cpu"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
