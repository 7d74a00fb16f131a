"""The N>1 path through the product: two rank processes share the box's one GPU
(ELECT_BENCH_SHARE_GPU=1), each codes its byte-balanced block of a mixed-size
stripe batch with the HIP kernels (elect_amd.dist.shard + batch.encode_batch /
decode_batch), the ranks exchange only host records over gloo, and the union of
their parity equals the oracle's, stripe by stripe."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    rng = np.random.default_rng(78)
    lens = [1024] * 24 + [4096] * 8 + [65536] * 3 + [4404020 // 64, 17]
    return [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(4)] for L in lens]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank), ELECT_BENCH_SHARE_GPU="1")
    import torch

    from elect_amd import dist
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    try:
        w, r, local = dist.setup("cuda")
        dev = torch.device("cuda", local)
        stripes = _batch()
        b, e = dist.shard([4 * len(s[0]) for s in stripes], w, r)
        coder = RSCoder(4, 2)
        mine = {}
        for i in range(b, e):
            L = len(stripes[i][0])
            st = torch.zeros((1, 6, L), dtype=torch.uint8, device=dev)
            st[0, :4] = torch.from_numpy(np.stack(stripes[i])).to(dev)
            encode_batch(coder, st[:, :4], st[:, 4:])
            out = torch.empty((1, 1, L), dtype=torch.uint8, device=dev)
            decode_batch(coder, st, [4, 1, 2, 3], [0], out, inputs_by_unit=True)
            h = st.cpu().numpy()[0]
            mine[i] = ([h[4].tobytes(), h[5].tobytes()], bool(np.array_equal(out.cpu().numpy()[0, 0], h[0])))
        dist.barrier(w)
        recs = dist.gather((b, e, mine), w)
        if r == 0:
            q.put(recs)
        dist.teardown(w)
    except Exception as ex:  # noqa: BLE001
        q.put(repr(ex))
        raise


def test_two_ranks_share_gpu_product_path(oracle):
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    recs = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert not isinstance(recs, str), recs
    ranges = sorted((b, e) for b, e, _ in recs)
    assert ranges[0][0] == 0 and ranges[0][1] == ranges[1][0] and ranges[1][1] == len(_batch())
    assert ranges[0][1] > 0 and ranges[1][1] > ranges[1][0]  # both ranks coded something
    enc = oracle.Encoder(4, 2)
    union = {}
    for _, _, mine in recs:
        union.update(mine)
    for i, s in enumerate(_batch()):
        par, dec_ok = union[i]
        assert par == [p.tobytes() for p in enc.encode(s)], i
        assert dec_ok, i
