"""Build tests/cpp/coder_api_test against include/elect_ec.hpp + libelect_ec.so."""
import os
import subprocess

from tests.conftest import ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "coder_api_test.cpp")
BIN = os.path.join(ROOT, "tests", "cpp", "coder_api_test")


def build() -> str:
    lib_dir = os.path.join(ROOT, "elect_amd")
    if not os.path.exists(BIN) or os.path.getmtime(BIN) < max(
            os.path.getmtime(SRC), os.path.getmtime(os.path.join(ROOT, "include", "elect_ec.hpp")),
            os.path.getmtime(os.path.join(lib_dir, "libelect_ec.so"))):
        subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"), SRC,
                        "-L", lib_dir, "-lelect_ec", f"-Wl,-rpath,{lib_dir}", "-Wl,-rpath-link,/opt/rocm/lib",
                        "-o", BIN], check=True)
    return BIN
