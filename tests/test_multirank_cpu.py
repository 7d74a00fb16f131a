"""CPU, world_size 2 over gloo: the N>1 path.  Each rank takes its byte-balanced
block of a mixed-size stripe batch (elect_amd.dist.shard), codes it (here with
the oracle as the stand-in for the device kernel: this test is about the
partition and the timing handshake, which are the same code bench.py runs),
and rank 0 checks that the union of the ranks' outputs equals the one-rank
result, with no data exchanged on the coding path."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from tests.conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch():
    rng = np.random.default_rng(77)
    lens = [1024] * 40 + [4096] * 10 + [65536] * 2 + [1000, 17]
    return [[rng.integers(0, 256, L, dtype=np.uint8) for _ in range(4)] for L in lens]


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    import torch.distributed as tdist

    from elect_amd import dist
    from oracle import ec_oracle
    w, r, _ = dist.setup("cpu")
    assert (w, r) == (world, rank)
    stripes = _batch()
    b, e = dist.shard([4 * len(s[0]) for s in stripes], w, r)
    enc = ec_oracle.Encoder(4, 2)
    mine = {i: [p.tobytes() for p in enc.encode(stripes[i])] for i in range(b, e)}
    dist.barrier(w)
    t = dist.max_over_ranks(float(rank + 1), w, "cpu")
    gathered = [None] * w
    tdist.all_gather_object(gathered, (b, e, mine))
    if rank == 0:
        q.put((t, gathered))
    dist.teardown(w)


def test_two_rank_partition_and_handshake():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    t, gathered = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert t == 2.0  # max over ranks
    ranges = sorted((b, e) for b, e, _ in gathered)
    assert ranges[0][0] == 0 and ranges[-1][1] == len(_batch()) and ranges[0][1] == ranges[1][0]
    sizes = [4 * len(s[0]) for s in _batch()]
    per_rank = [sum(sizes[b:e]) for b, e in ranges]
    assert max(per_rank) - min(per_rank) <= max(sizes)  # byte-balanced within one stripe
    from oracle import ec_oracle
    enc = ec_oracle.Encoder(4, 2)
    union = {}
    for _, _, mine in gathered:
        union.update(mine)
    for i, s in enumerate(_batch()):
        assert union[i] == [p.tobytes() for p in enc.encode(s)]
