"""The drop-in libec.so JNI shim (elect_amd/csrc/jni/libec_jni.c), compiled and
driven by a fake JVM (tests/jni/jni_shim_test.c) — this image has no JDK, so the
shim is built against an API-level mock of <jni.h> (tests/jni/mock/jni.h).

Covers SURVEY.md §8b: the seven exported names (JEC/NativeRSEncoder.java:97-105,
JEC/NativeRSDecoder.java:81-87), the `long nativeCoder` ownership protocol
(EC/jni_common.c:24-60), direct-buffer + offset resolution (EC/jni_common.c:62-108),
and the exceptions Java callers see.  No device needed."""
import re
import subprocess

import numpy as np

from tests.jni_build import build

OPTIONAL = {  # bound only by a Java that declares them
    # the fused coding-node steps
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeExImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeUpdateExImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_decodeExImpl",
    # page-locked coding buffers (elect_ec_host_alloc)
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_allocateDirectImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_freeDirectImpl",
}
SEVEN = {
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_initImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeUpdateImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_destroyImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_initImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_decodeImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_destroyImpl",
}


def test_shim_exports_the_seven_native_methods_and_the_optional_ones():
    lib, _ = build()
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == SEVEN | OPTIONAL


def test_shim_error_paths_under_fake_jvm():
    """Count checks, heap/null buffers, closed coders, a missing nativeCoder
    field, engine validation errors and (with no device) the loud ENODEV
    failure all surface as the Java exceptions ELECT handles; no JNI call while
    an exception is pending, no leaked int[] elements or local refs."""
    lib, drv = build()
    r = subprocess.run([drv, lib, "cpu"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failure(s), 0 JNI violation(s)" in r.stdout


def _coding_matrix(buf, n1, n2):
    """EC/dump.c:46-59 dumpCodingMatrix: n2 rows of n1 entries, ' %d' each."""
    buf = list(buf) + [0] * (n1 * n2 - len(buf))
    return "".join("".join(f" {buf[j + i * n1]}" for j in range(n1)) + "\n" for i in range(n2)) + "\n"


def _decode_lines(k, m, era, L):
    """decodeImpl's three lines, printed on every call (EC/NativeRSDecoder.c:57, 65, 68)."""
    return ("NativeRSDecoder_decodeImpl, start to process: data unit = %d, parity unit = %d, data block size = %d\n"
            % (k, m, L) +
            "NativeRSDecoder_decodeImpl, read data: target recovery data block number = %d, the first recovery "
            "request block ID = %d\n" % (len(era), era[0]) +
            "NativeRSDecoder_decodeImpl, start do decode\n")


def _decoder_block(oracle, k, m, dec, era, L):
    n = k + m
    em = oracle.cauchy_matrix(k, m).reshape(-1)
    rows = np.stack([oracle.cauchy_matrix(k, m)[i] for i in dec])
    _, inv = oracle.invert_matrix(rows)
    _, dm = oracle.decode_matrix(k, m, dec, era, False)
    return (_decode_lines(k, m, era, L) +
            "Recovering (numAllUnits = %d, numDataUnits = %d, numErased = %d)\n" % (n, k, len(era)) +
            " - ErasedIndexes = " + "".join(f" {e}" for e in era) +
            "       - DecodeIndex = " + "".join(f" {d}" for d in dec) +
            "\n\nEncodeMatrix:\n" + _coding_matrix(em, k, n) +
            "InvertMatrix:\n" + _coding_matrix(inv.reshape(-1), k, n) +
            "DecodeMatrix:\n" + _coding_matrix(dm.reshape(-1), k, n))


def _dump_cases(drv, lib, **env):
    import os
    import re
    r = subprocess.run([drv, lib, "dump"], capture_output=True, text=True, timeout=60,
                       env=dict(os.environ, **env))
    assert r.returncode == 0, r.stdout + r.stderr
    return dict(re.findall(r"=== (.*?)\n(.*?)(?==== )", r.stdout, flags=re.S))


def test_stdout_matches_libec(oracle):
    """Standard output at the JNI boundary is libec.so's, verbose or not:
    decodeImpl prints its three lines on every call (EC/NativeRSDecoder.c:57,
    65, 68) and, with allowVerboseDump() true, EC/dump.c's dumpDecoder block
    (:75-104, from processErasures, EC/erasure_coder.c:195-197) with the oracle's
    matrices: the Cauchy generator, gf_invert_matrix's (partial, when singular)
    inverse in a zeroed MMAX x KMAX array, and the compat decode rows.  encode and
    encodeUpdate print nothing, verbose or not: libec.so's only dumpEncoder call
    runs right after initCoder zeroes verbose (EC/erasure_coder.c:27, 61-63).
    ELECT_EC_JNI_QUIET=1 silences the decode lines (an opt-out; the default is
    the reference's)."""
    lib, drv = build()
    cases = _dump_cases(drv, lib)
    assert cases["encode RS(6,4)"] == ""
    assert cases["encodeUpdate RS(6,4)"] == ""
    assert cases["quiet encode RS(6,4)"] == ""
    assert cases["decode RS(6,4) {4,1,2,3} erase {0}"] == _decoder_block(oracle, 4, 2, [4, 1, 2, 3], [0], 16)
    assert cases["decode RS(6,4) singular {1,1,2,3} erase {0,5}"] == \
        _decoder_block(oracle, 4, 2, [1, 1, 2, 3], [0, 5], 16)
    assert cases["decode RS(12,8) {2..8,10} erase {9,0}"] == \
        _decoder_block(oracle, 8, 4, [2, 3, 4, 5, 6, 7, 8, 10], [9, 0], 16)
    assert cases["quiet decode RS(6,4) {4,1,2,3} erase {0}"] == _decode_lines(4, 2, [0], 16)
    silenced = _dump_cases(drv, lib, ELECT_EC_JNI_QUIET="1")
    assert silenced["quiet decode RS(6,4) {4,1,2,3} erase {0}"] == ""
    assert silenced["decode RS(6,4) {4,1,2,3} erase {0}"] == \
        _decoder_block(oracle, 4, 2, [4, 1, 2, 3], [0], 16)[len(_decode_lines(4, 2, [0], 16)):]


def test_mock_jni_table_is_the_specification_layout():
    """The mock header the shim is built against pins every slot it uses to the
    JNI specification's function-table index (compile-time asserts), so the
    tested library calls the same slots a JDK-built one does."""
    import os
    from tests.conftest import ROOT
    text = open(os.path.join(ROOT, "tests", "jni", "mock", "jni.h")).read()
    want = {"FindClass": 6, "ThrowNew": 14, "ExceptionClear": 17, "DeleteLocalRef": 23, "GetObjectClass": 31,
            "GetMethodID": 33, "CallBooleanMethod": 37, "GetFieldID": 94, "GetLongField": 101, "SetLongField": 110,
            "GetArrayLength": 171, "GetObjectArrayElement": 173, "GetIntArrayElements": 187,
            "ReleaseIntArrayElements": 195, "GetIntArrayRegion": 203, "SetIntArrayRegion": 211,
            "ExceptionCheck": 228, "NewDirectByteBuffer": 229, "GetDirectBufferAddress": 230}
    for name, idx in want.items():
        assert f"JNI_SLOT({name}, {idx});" in text, name
    shim = open(os.path.join(ROOT, "elect_amd", "csrc", "jni", "libec_jni.c")).read()
    used = set(re.findall(r"\(\*env\)->(\w+)", shim))
    assert used <= set(want), used - set(want)
