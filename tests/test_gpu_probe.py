"""elect_ec_hbm_probe, the kernels behind bench.py's achievable ceilings: every
kind writes what it should (write: segment i = (i, 1, 2, 3); copy: the source;
3 / 4: the XOR of four streams, and for 4 a second stream with 1 added to each
segment's first dword), in dispatch order and XCD-major order alike (the block
order must cover every segment exactly once), and bad arguments are refused."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _u32(t):
    return t.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("xcd", [False, True])
@pytest.mark.parametrize("block", [64, 256])
def test_probe_kinds_write_what_they_should(dev, xcd, block):
    from elect_amd import _lib
    n = 16 * block * 8 * 4  # segments: a multiple of block, blocks: a multiple of 8
    flag = 0x100 if xcd else 0
    g = torch.Generator(device=dev).manual_seed(5)
    src = torch.randint(0, 128, (4 * n,), dtype=torch.uint8, device=dev, generator=g)
    sink = torch.zeros(256, dtype=torch.uint8, device=dev)
    _lib.hbm_probe(0 | flag, src.data_ptr(), sink.data_ptr(), n, block, 18)
    out = torch.zeros(2 * n, dtype=torch.uint8, device=dev)
    _lib.hbm_probe(1 | flag, 0, out.data_ptr(), n, block, 0)
    w = _u32(out[:n]).reshape(-1, 4)
    assert (w[:, 0] == np.arange(n // 16, dtype=np.uint32)).all() and (w[:, 1:] == [1, 2, 3]).all()
    out.zero_()
    _lib.hbm_probe(2 | flag, src.data_ptr(), out.data_ptr(), n, block, 0)
    assert torch.equal(out[:n], src[:n])
    x = src.view(4, n)
    want = x[0] ^ x[1] ^ x[2] ^ x[3]
    out.zero_()
    _lib.hbm_probe(3 | flag, src.data_ptr(), out.data_ptr(), n, block, 18)
    assert torch.equal(out[:n], want) and not bool(out[n:].any())
    out.zero_()
    _lib.hbm_probe(4 | flag, src.data_ptr(), out.data_ptr(), n, block, 0)
    assert torch.equal(out[:n], want)
    second = _u32(out[n:]).reshape(-1, 4).copy()
    base = _u32(want).reshape(-1, 4).copy()
    base[:, 0] += 1
    assert (second == base).all()
    torch.cuda.synchronize()
    assert not bool(sink.any())


def test_probe_refuses_bad_arguments(dev):
    from elect_amd import _lib
    buf = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    p = buf.data_ptr()
    for kind, n, block in ((5, 4096, 256), (0, 4100, 256), (0, 4096, 96),
                           (0x100, 16 * 256 * 3, 256)):  # XCD-major needs a block count that is a multiple of 8
        with pytest.raises(RuntimeError):
            _lib.hbm_probe(kind, p, p, n, block, 0)
