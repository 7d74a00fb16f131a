import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def oracle():
    from oracle import ec_oracle
    ec_oracle.lib()
    return ec_oracle


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch.device("cuda:0")


def distinct_hip_streams(n: int, device: int = 0) -> list:
    """n new, distinct HIP streams as torch.cuda.ExternalStream objects.
    torch.cuda.Stream() hands out streams from a fixed pool (32 per priority and
    device), so 80 torch.cuda.Stream objects are at most 32 distinct streams;
    these come from hipStreamCreateWithFlags of the HIP runtime already loaded in
    the process (torch's), found through /proc/self/maps.  Never destroyed
    (test processes only)."""
    import ctypes
    import torch
    torch.cuda.init()
    path = None
    with open("/proc/self/maps") as f:
        for line in f:
            if "libamdhip64" in line:
                path = line.split()[-1]
                break
    if path is None:
        raise RuntimeError("no HIP runtime loaded in this process")
    hip = ctypes.CDLL(path)
    out = []
    for _ in range(n):
        s = ctypes.c_void_p()
        rc = hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1))  # hipStreamNonBlocking
        if rc != 0:
            raise RuntimeError(f"hipStreamCreateWithFlags: {rc}")
        out.append(torch.cuda.ExternalStream(s.value, device=torch.device("cuda", device)))
    return out
