"""Build the drop-in JNI shim (elect_amd/csrc/jni/libec_jni.c) against the mock
JNI header (tests/jni/mock/jni.h; this image has no JDK) as tests/jni/libec.so,
linked to libelect_ec.so, plus the fake-JVM driver tests/jni/jni_shim_test."""
import os
import subprocess

from tests.conftest import ROOT

JNI = os.path.join(ROOT, "tests", "jni")
SHIM_SRC = os.path.join(ROOT, "elect_amd", "csrc", "jni", "libec_jni.c")
DRIVER_SRC = os.path.join(JNI, "jni_shim_test.c")
LIB = os.path.join(JNI, "libec.so")
DRIVER = os.path.join(JNI, "jni_shim_test")


def _stale(out, deps):
    return not os.path.exists(out) or os.path.getmtime(out) < max(os.path.getmtime(d) for d in deps)


def build():
    lib_dir = os.path.join(ROOT, "elect_amd")
    engine = os.path.join(lib_dir, "libelect_ec.so")
    mock = os.path.join(JNI, "mock", "jni.h")
    hdr = os.path.join(ROOT, "include", "elect_ec.h")
    if _stale(LIB, [SHIM_SRC, mock, hdr, engine]):
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-fPIC", "-shared",
                        "-fvisibility=hidden", "-I", os.path.join(JNI, "mock"), SHIM_SRC,
                        "-L", lib_dir, "-lelect_ec", f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/opt/rocm/lib",
                        "-o", LIB], check=True)
    if _stale(DRIVER, [DRIVER_SRC, mock]):
        subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Wextra", "-Werror", "-D_GNU_SOURCE",
                        "-I", os.path.join(JNI, "mock"), DRIVER_SRC, "-ldl", "-o", DRIVER], check=True)
    return LIB, DRIVER
