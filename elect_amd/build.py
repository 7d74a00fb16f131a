"""Build recipe for libelect_ec.so (gfx950) — in-tree, so the .so travels with
the repo snapshot to the GPU box.  `python -m elect_amd.build [--force]`.

Freshness is by content, not mtime: the build id is a SHA-256 over the sources,
headers and compile flags.  It is compiled into the library
(elect_ec_build_id()) and written next to it (libelect_ec.so.buildid), so a
copied tree whose mtimes changed is not rebuilt needlessly, a stale library is
always rebuilt here, and at run time _lib.BUILD_CURRENT says whether the loaded
library was built from the sources beside it.
"""
from __future__ import annotations

import hashlib
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
STAMP = LIB + ".buildid"
ARCH = os.environ.get("ELECT_EC_ARCH", "gfx950")

SOURCES = ["ec_capi.cpp", "host_path.cpp", "rs_kernels.hip", "rs_inst.hip"]
HEADERS = ["gf256.hpp", "rs_kernels.hpp", "rs_impl.hpp", "host_path.hpp"]
INST_KS = range(1, 17)  # rs_inst.hip, once per source-column count (ELECT_EC_INST_K)


def units():
    """(source, object stem, extra flags) of every translation unit: rs_inst.hip
    once per K, so the kernel instances compile in parallel."""
    out = []
    for src in SOURCES:
        if src == "rs_inst.hip":
            out += [(src, f"rs_inst_k{k}", [f"-DELECT_EC_INST_K={k}"]) for k in INST_KS]
        else:
            out.append((src, os.path.splitext(src)[0], []))
    return out
FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-Wall"]
# Translation units with no device code, compiled as host C++ against the HIP runtime API.
HOST_SOURCES = {"host_path.cpp"}
HOST_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include"]


def digest_files(paths, extra: str = "") -> str:
    """SHA-256 (hex, 16 chars) over the files' bytes in the given order, plus extra."""
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def build_id() -> str:
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [os.path.join(ROOT, "include", "elect_ec.h")]
    return digest_files(deps, " ".join(FLAGS + HOST_FLAGS + sorted(HOST_SOURCES)))


def stamped_id() -> str | None:
    try:
        with open(STAMP) as f:
            return f.read().strip()
    except OSError:
        return None


def _hipcc() -> str:
    for c in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found: cannot build the MI355X engine")


def _stale() -> bool:
    return not os.path.exists(LIB) or stamped_id() != build_id()


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    hipcc = _hipcc()
    os.makedirs(BUILD, exist_ok=True)
    bid = build_id()
    common = [*FLAGS, "-I", os.path.join(ROOT, "include"), f'-DELECT_EC_BUILD_ID="{bid}"']

    def compile_one(unit):
        src, stem, extra = unit
        obj = os.path.join(BUILD, stem + ".o")
        if src in HOST_SOURCES:  # no device code: host C++ (CPU builtins such as __builtin_cpu_supports)
            cmd = [hipcc, *HOST_FLAGS, "-I", os.path.join(ROOT, "include"), f'-DELECT_EC_BUILD_ID="{bid}"',
                   *extra, "-x", "c++", "-c", os.path.join(CSRC, src), "-o", obj]
        else:
            cmd = [hipcc, *common, *extra, "-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
        if verbose:
            print(" ".join(cmd))
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"compile failed: {src} {' '.join(extra)}\n{r.stderr}")
        return obj

    jobs = max(1, min(16, os.cpu_count() or 1))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, units()))
    tmp = LIB + ".tmp"
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs, "-L/opt/rocm/lib", "-lhsa-runtime64"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{r.stderr}")
    os.replace(tmp, LIB)
    with open(STAMP, "w") as f:
        f.write(bid + "\n")
    return LIB


# The host-code sanitizer build (tools/sanitize/run.sh): its own content stamp.
SANITIZE_DIR = os.path.join(ROOT, "tools", "sanitize")
SANITIZE_BIN = os.path.join(SANITIZE_DIR, "out", "host_stress")
SANITIZE_STAMP = SANITIZE_BIN + ".buildid"


def sanitize_id() -> str:
    deps = [os.path.join(CSRC, f) for f in SOURCES + HEADERS] + [
        os.path.join(ROOT, "include", "elect_ec.h"), os.path.join(SANITIZE_DIR, "host_stress.cpp"),
        os.path.join(SANITIZE_DIR, "run.sh")]
    return digest_files(deps)


def sanitize_current() -> bool:
    try:
        with open(SANITIZE_STAMP) as f:
            return os.path.exists(SANITIZE_BIN) and f.read().strip() == sanitize_id()
    except OSError:
        return False


def build_sanitize(force: bool = False) -> str:
    """ASan+UBSan build of the host code + the stress driver (host code only)."""
    if not force and sanitize_current():
        return SANITIZE_BIN
    r = subprocess.run([os.path.join(SANITIZE_DIR, "run.sh"), "build"], capture_output=True, text=True, cwd=ROOT)
    if r.returncode != 0:
        raise RuntimeError(f"sanitizer build failed\n{r.stdout[-2000:]}{r.stderr[-4000:]}")
    with open(SANITIZE_STAMP, "w") as f:
        f.write(sanitize_id() + "\n")
    return SANITIZE_BIN


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
    if "--sanitize" in sys.argv:
        print(build_sanitize(force="--force" in sys.argv))
