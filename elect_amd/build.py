"""Build recipe for libelect_ec.so (gfx950) — in-tree, so the .so travels with
the repo snapshot to the GPU box.  `python -m elect_amd.build [--force]`."""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(HERE, "libelect_ec.so")
ARCH = os.environ.get("ELECT_EC_ARCH", "gfx950")

SOURCES = ["ec_capi.cpp", "host_path.cpp", "rs_kernels.hip"]
HEADERS = ["gf256.hpp", "rs_kernels.hpp", "host_path.hpp"]


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build the MI355X engine")


def _newest(paths):
    return max(os.path.getmtime(p) for p in paths)


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS]
    deps += [os.path.join(ROOT, "include", "elect_ec.h"), os.path.abspath(__file__)]
    return _newest(deps) > os.path.getmtime(LIB)


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    common = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall",
              "-I", os.path.join(ROOT, "include")]

    def compile_one(src):
        obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
        cmd = [hipcc, *common, "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src}\n{r.stderr}")
        return obj

    with ThreadPoolExecutor(max_workers=len(SOURCES)) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
