"""The drop-in libec.so JNI shim (elect_amd/csrc/jni/libec_jni.c), compiled and
driven by a fake JVM (tests/jni/jni_shim_test.c) — this image has no JDK, so the
shim is built against an API-level mock of <jni.h> (tests/jni/mock/jni.h).

Covers SURVEY.md §8b: the seven exported names (JEC/NativeRSEncoder.java:97-105,
JEC/NativeRSDecoder.java:81-87), the `long nativeCoder` ownership protocol
(EC/jni_common.c:24-60), direct-buffer + offset resolution (EC/jni_common.c:62-108),
and the exceptions Java callers see.  No device needed."""
import subprocess

from tests.jni_build import build

OPTIONAL = {  # fused coding-node steps, bound only by a Java that declares them
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeExImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSEncoder_encodeUpdateExImpl",
    "Java_org_apache_cassandra_io_erasurecode_NativeRSDecoder_decodeExImpl",
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


def test_shim_exports_the_seven_native_methods_and_the_three_optional_ones():
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
