"""The XOR-circulant (Cauchy-structured) encode kernel, gf_apply_x16c
(rs_impl.hpp gf_combine_cauchy4): launches whose 4-row coefficient blocks are
XOR-circulant in every 4-column group (M[a][4g+c] == M[0][4g+(a^c)], which
ISA-L's Cauchy generator gives for k % 4 == 0, EC/erasure_coder.c:43) apply 9
multiplications per group instead of 16.  Checked against the CPU oracle:

- ELECT's own RS(12,8) and RS(8,4) / RS(16,12) parity (4-row Cauchy blocks),
  whole-wave stripes so the structured kernel is the one launched;
- random XOR-circulant matrices (any coefficients with the structure, not only
  Cauchy ones), and a matrix that breaks the structure in one byte (general
  kernel), at the same shapes;
- the structured form off (ELECT_EC_CAUCHY=0) gives the same bytes."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _circulant(rng, k):
    coef = np.zeros((4, k), np.uint8)
    for g in range(k // 4):
        h = rng.integers(1, 256, 4)
        for a in range(4):
            for c in range(4):
                coef[a, 4 * g + c] = h[a ^ c]
    return coef


def _apply_check(dev, oracle, coef, B, L, seed):
    from elect_amd.batch import apply_batch
    rows, cols = coef.shape
    rng = np.random.default_rng(seed)
    data = rng.integers(0, 256, (cols, B, L), dtype=np.uint8)
    src = [torch.from_numpy(data[j]).to(dev) for j in range(cols)]
    dst = [torch.empty((B, L), dtype=torch.uint8, device=dev) for _ in range(rows)]
    apply_batch(coef, src, dst)
    got = [d.cpu().numpy() for d in dst]
    for s in (0, B // 2, B - 1):
        want = oracle.apply(coef, [data[j, s] for j in range(cols)])
        for r in range(rows):
            assert np.array_equal(got[r][s], want[r]), (s, r)


@pytest.mark.parametrize("k", [4, 8, 12])
def test_cauchy_parity_rows(dev, oracle, k):
    coef = oracle.cauchy_matrix(k, 4)[k:]  # the 4 parity rows of ISA-L's generator
    assert all(coef[a, 4 * g + c] == coef[0, 4 * g + (a ^ c)]
               for g in range(k // 4) for a in range(4) for c in range(4))
    _apply_check(dev, oracle, coef, 64, 65536, seed=k)
    _apply_check(dev, oracle, coef, 3, 1 << 20, seed=k + 1)


@pytest.mark.parametrize("k", [4, 8])
def test_random_circulant_and_a_broken_one(dev, oracle, k):
    rng = np.random.default_rng(40 + k)
    coef = _circulant(rng, k)
    _apply_check(dev, oracle, coef, 48, 65536, seed=7)
    broken = coef.copy()
    broken[2, 1] ^= 0x5A  # no longer circulant: the general kernel
    _apply_check(dev, oracle, broken, 48, 65536, seed=8)


SCRIPT = r"""
import sys, hashlib
import numpy as np, torch
sys.path.insert(0, ROOT)
from elect_amd.batch import encode_batch
from elect_amd.coder import RSCoder
k, m, B, L = 8, 4, 96, 65536
st = torch.from_numpy(np.random.default_rng(3).integers(0, 256, (B, k + m, L), dtype=np.uint8)).cuda()
encode_batch(RSCoder(k, m), st[:, :k], st[:, k:])
print(hashlib.sha256(st[:, k:].cpu().numpy().tobytes()).hexdigest())
"""


def test_structured_form_equals_general_form():
    out = []
    for on in ("1", "0"):
        env = dict(os.environ, ELECT_EC_CAUCHY=on)
        r = subprocess.run([sys.executable, "-c", SCRIPT.replace("ROOT", repr(ROOT))], capture_output=True, text=True,
                           timeout=240, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-2000:]
        out.append(r.stdout.strip().splitlines()[-1])
    assert out[0] == out[1] and len(out[0]) == 64
