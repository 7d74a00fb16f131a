"""CPU: the C ABI library loads, exports every symbol include/elect_ec.h
declares, and its host-side coder logic (generator matrix, ISA-L table layout,
decode-matrix construction incl. ELECT's compat quirk and singular handling)
matches the oracle and the golden fixtures.  No compute call needs a GPU here;
the one that runs checks that the product fails loudly without one."""
import ctypes
import itertools
import json
import os
import re

import numpy as np
import pytest

from tests.conftest import ROOT, gpu_available

HEADER = os.path.join(ROOT, "include", "elect_ec.h")


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(elect_ec_\w+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from elect_amd import _lib
    declared = header_functions()
    assert len(declared) >= 17
    for name in declared:
        assert hasattr(_lib.lib, name), f"{name} missing from libelect_ec.so"
    bound = {n for n, _, _ in _lib.SIGNATURES if not n.startswith("elect_ec_internal_")}  # (test hooks)
    assert bound == set(declared), "ctypes bindings out of sync with the header"


def test_library_links_hip_and_has_gfx950_code():
    import subprocess
    lib = os.path.join(ROOT, "elect_amd", "libelect_ec.so")
    deps = subprocess.run(["ldd", lib], capture_output=True, text=True).stdout
    assert "amdhip64" in deps
    blob = open(lib, "rb").read()
    assert b"gfx950" in blob


def test_version_and_strerror():
    from elect_amd import _lib
    assert b"gfx950" in _lib.lib.elect_ec_version()
    for st in (0, 1, -1, -2, -3, -4, -5):
        assert _lib.strerror(st) != "unknown status"


def test_library_built_from_these_sources():
    """The in-tree library's compiled-in build id is the content hash of the
    sources beside it (elect_amd/build.py): what ships to the GPU box is what
    the tree says, whatever the file mtimes."""
    from elect_amd import _lib, build
    assert _lib.BUILD_ID == build.build_id() == build.stamped_id()
    assert _lib.BUILD_CURRENT


@pytest.mark.parametrize("k,m", [(4, 2), (8, 4), (1, 1), (10, 4), (2, 12), (3, 2)])
def test_encode_matrix_and_tables_match_oracle(oracle, k, m):
    from elect_amd.coder import RSCoder
    c = RSCoder(k, m)
    assert np.array_equal(c.encode_matrix(), oracle.cauchy_matrix(k, m))
    assert np.array_equal(c.gf_tables(), oracle.init_tables(oracle.cauchy_matrix(k, m)[k:]))


@pytest.mark.parametrize("k,m", [(4, 2), (3, 2), (8, 4), (6, 3)])
def test_decode_matrix_all_patterns_match_oracle(oracle, k, m):
    from elect_amd.coder import RSCoder
    c = RSCoder(k, m)
    rng = np.random.default_rng(k + m)
    pats = [list(e) for n in range(1, m + 1) for e in itertools.combinations(range(k + m), n)]
    for erased in pats:
        surv = [i for i in range(k + m) if i not in erased][:k]
        for order in (surv, [int(x) for x in rng.permutation(surv)]):
            for mode in (0, 1):
                st, mat = c.decode_matrix(order, erased, mode)
                rc, want = oracle.decode_matrix(k, m, order, erased, bool(mode))
                assert st == rc == 0
                assert np.array_equal(mat, want), (erased, order, mode)


def test_decode_matrix_golden():
    from elect_amd.coder import RSCoder
    from elect_amd import _lib
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "decode.json")))
    coders = {}
    for case in g["cases"]:
        key = (case["k"], case["m"])
        c = coders.setdefault(key, RSCoder(*key))
        mode = _lib.DECODE_STRICT if case["mode"] == "strict" else _lib.DECODE_COMPAT
        if case["status"] != 0 and mode == _lib.DECODE_STRICT:
            with pytest.raises(_lib.ECSingularError):
                c.decode_matrix(case["decode_indexes"], case["erased"], mode)
            continue
        st, mat = c.decode_matrix(case["decode_indexes"], case["erased"], mode)
        expect_st = _lib.WARN_SINGULAR if case["status"] != 0 else _lib.OK
        assert st == expect_st
        assert mat.tobytes().hex() == case["matrix"], case


def test_singular_compat_reproduces_partial_inverse(oracle):
    """A duplicated survivor makes the k x k matrix singular; libec.so ignores
    gf_invert_matrix's failure (EC/erasure_coder.c:257) and keeps going."""
    from elect_amd.coder import RSCoder
    from elect_amd import _lib
    c = RSCoder(4, 2)
    for surv in ([1, 1, 2, 3], [4, 4, 5, 0], [0, 1, 2, 2]):
        for erased in ([0], [3], [0, 5], [5, 0]):
            st, mat = c.decode_matrix(surv, erased, _lib.DECODE_COMPAT)
            rc, want = oracle.decode_matrix(4, 2, surv, erased, False)
            assert st == _lib.WARN_SINGULAR and rc == -1
            assert np.array_equal(mat, want)


def test_invalid_arguments():
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    for k, m in ((0, 2), (11, 2), (4, 0), (10, 5), (-1, 1)):
        with pytest.raises(_lib.ECInvalidArgument):
            RSCoder(k, m)
    c = RSCoder(4, 2)
    with pytest.raises(_lib.ECInvalidArgument):
        c.decode_matrix([1, 2, 3, 4], [0, 5, 1], 0)  # more erasures than m (JEC/CoderUtil.java:79-82)
    with pytest.raises(_lib.ECInvalidArgument):
        c.decode_matrix([1, 2, 3, 6], [0], 0)  # unit index out of range
    with pytest.raises(_lib.ECInvalidArgument):
        c.decode_matrix([1, 2, 3, 4], [0], 7)  # bad mode
    h = ctypes.c_void_p()
    assert _lib.lib.elect_ec_coder_create(4, 2, None) == _lib.EINVAL
    assert _lib.lib.elect_ec_coder_create(4, 2, ctypes.byref(h)) == _lib.OK
    assert _lib.lib.elect_ec_coder_num_data_units(h) == 4
    assert _lib.lib.elect_ec_coder_num_parity_units(h) == 2
    buf = (ctypes.c_ubyte * 8)()
    assert _lib.lib.elect_ec_coder_encode_matrix(h, buf, 8) == _lib.EINVAL  # too small
    _lib.lib.elect_ec_coder_destroy(h)


@pytest.mark.skipif(gpu_available(), reason="checks the no-device path")
def test_no_device_fails_loudly():
    """There is no CPU fallback: without a GPU, compute calls return ENODEV."""
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    assert _lib.device_count() == 0
    c = RSCoder(4, 2)
    d = [np.zeros(64, np.uint8) for _ in range(4)]
    p = [np.zeros(64, np.uint8) for _ in range(2)]
    with pytest.raises(_lib.ECDeviceError):
        c.encode_host([a.ctypes.data for a in d], [a.ctypes.data for a in p], 64)
    # zero-length is a no-op before any device work (JEC/ErasureEncoder.java:41-44)
    assert c.encode_host([a.ctypes.data for a in d], [a.ctypes.data for a in p], 0) == 0
    with pytest.raises(_lib.ECDeviceError):
        _lib.unaligned_vector_ok()


def test_flow_entry_points_validate_before_device_work():
    """encode_ex / encode_update_ex / decode_ex: argument errors and the no-op cases need no device."""
    from elect_amd import _lib
    from elect_amd.coder import RSCoder
    c = RSCoder(4, 2)
    d = [np.zeros(64, np.uint8) for _ in range(6)]
    p = [np.zeros(64, np.uint8) for _ in range(2)]
    ins = [a.ctypes.data for a in d]
    outs = [a.ctypes.data for a in p]
    with pytest.raises(_lib.ECInvalidArgument):  # target data index out of range
        c.encode_update_ex_host(ins, 4, outs, 64, old_new_lengths=[64, 64])
    with pytest.raises(_lib.ECInvalidArgument):  # fused hash needs 2 + m <= 10
        RSCoder(4, 9).encode_update_ex_host(ins + [0] * 5, 0, outs + [0] * 7, 64, hashed=True)
    # hashCode() of an empty buffer is 1 (no device work)
    assert c.encode_ex_host(ins[:4], outs, 0, hashed=True) == [1, 1]
    assert c.encode_update_ex_host(ins, 0, outs, 0, hashed=True) == [1, 1]
    out = [p[0].ctypes.data]
    with pytest.raises(_lib.ECInvalidArgument):  # more erasures than m (JEC/CoderUtil.java:79-82)
        c.decode_ex_host(ins[1:5], [1, 2, 3, 4], [0, 5, 1], out * 3, 64, input_lengths=[64] * 4)
    with pytest.raises(_lib.ECInvalidArgument):  # survivor index out of range
        c.decode_ex_host(ins[1:5], [1, 2, 3, 9], [0], out, 64, input_lengths=[64] * 4)
    # a zero-length decode is a no-op before any device work (JEC/ErasureDecoder.java:36-38)
    assert c.decode_ex_host(ins[1:5], [1, 2, 3, 4], [0], out, 0, input_lengths=[5, 0, 0, 7]) == 0
    if not gpu_available():
        with pytest.raises(_lib.ECDeviceError):
            c.decode_ex_host(ins[1:5], [1, 2, 3, 4], [0], out, 64, input_lengths=[64, 10, 0, 64])
        with pytest.raises(_lib.ECDeviceError):
            c.encode_ex_host(ins[:4], outs, 64, data_lengths=[64, 3, 0, 64], hashed=True)
        with pytest.raises(_lib.ECDeviceError):
            c.encode_update_ex_host(ins, 1, outs, 64, old_new_lengths=[10, 64], hashed=True)


def test_partition_by_bytes():
    from elect_amd.batch import partition_by_bytes
    sizes = [1024] * 1000 + [4096] * 250 + [1 << 20] * 1
    for world in (1, 2, 3, 4, 8):
        parts = [partition_by_bytes(sizes, world, r) for r in range(world)]
        assert parts[0][0] == 0 and parts[-1][1] == len(sizes)
        for a, b in zip(parts, parts[1:]):
            assert a[1] == b[0]
    sizes = [65536] * 4096
    for world in (1, 2, 4, 8):
        for r in range(world):
            b, e = partition_by_bytes(sizes, world, r)
            assert e - b == 4096 // world


def test_device_api_rejects_mismatched_shapes():
    """The device-resident wrappers check every tensor's shape before the C ABI
    sees its strides: an output with another stripe count or chunk length (a
    tiled coding view decoded into a [B, 1, L] buffer, say) would otherwise be
    written out of bounds on the device.  Raised before any device call."""
    import torch
    from elect_amd.batch import apply_batch, decode_batch, decode_batches, encode_update_batch
    from elect_amd.coder import RSCoder
    import numpy as np
    c = RSCoder(4, 2)
    st = torch.zeros((16, 6, 64), dtype=torch.uint8)
    with pytest.raises(ValueError, match="outputs"):
        decode_batch(c, st, [1, 2, 3, 4], [0], torch.zeros((1, 1, 1024), dtype=torch.uint8), inputs_by_unit=True)
    with pytest.raises(ValueError, match="outputs"):
        decode_batch(c, st, [1, 2, 3, 4], [0, 5], st[:, :3], outputs_by_unit=True, inputs_by_unit=True)
    with pytest.raises(ValueError, match="inputs"):
        decode_batch(c, st[:, :3], [0, 1, 2, 3], [4], torch.zeros((16, 1, 64), dtype=torch.uint8))
    with pytest.raises(ValueError, match="outputs"):
        decode_batches(c, [(st, torch.zeros((16, 1, 32), dtype=torch.uint8))], [1, 2, 3, 4], [0], inputs_by_unit=True)
    with pytest.raises(ValueError, match="parity_out"):
        encode_update_batch(c, 0, st[:, 0], st[:, 1], st[:, 4:], torch.zeros((8, 2, 64), dtype=torch.uint8))
    with pytest.raises(ValueError, match="apply_batch"):
        apply_batch(np.ones((1, 2), np.uint8), [st[:, 0], st[:2, 1]], [st[:, 4]])
    # the hashed and padded encodes: parity with fewer stripes, rows or bytes, data of another k
    from elect_amd.batch import encode_batch_hashed, encode_batch_padded, encode_batch_tiled
    h = torch.zeros((16, 2), dtype=torch.int32)
    lens = torch.zeros((16, 4), dtype=torch.int32)
    for bad in (torch.zeros((8, 2, 64), dtype=torch.uint8), st[:, 4:5], st[:, 4:, :32]):
        with pytest.raises(ValueError, match="parity"):
            encode_batch_hashed(c, st[:, :4], bad, h)
        with pytest.raises(ValueError, match="parity"):
            encode_batch_padded(c, st[:, :4], lens, bad)
    with pytest.raises(ValueError, match="data"):
        encode_batch_hashed(c, st[:, :3], st[:, 4:], h)
    with pytest.raises(ValueError, match="data"):
        encode_batch_padded(c, st[:, :5], lens, st[:, 4:])
    # a tiled view with a zero tile length: ValueError, not ZeroDivisionError
    with pytest.raises(ValueError, match="tile"):
        encode_batch_tiled(c, st[:, :4, :0], st[:, 4:, :0], 64)


def test_host_alloc_pool_semantics():
    """elect_ec_host_alloc / _free / _pinned: every allocation is usable memory
    (page-locked when a device allows, ordinary memory otherwise, which the host
    path then stages), frees are checked, and the pinned query covers exactly a
    live page-locked buffer."""
    from elect_amd import _lib
    bufs = [_lib.HostBuffer(n) for n in (1, 4096, 65536 + 3, 4404020)]
    for b in bufs:
        b.array[:] = 0xA5  # writable over its whole length
        assert int(b.array[-1]) == 0xA5
        pinned = _lib.host_pinned(b.addr, b.nbytes)
        assert pinned == (gpu_available() and _lib.device_count() > 0)
        assert not _lib.host_pinned(b.addr, b.nbytes + (1 << 16) + 1)  # past the 64 KiB size class
    addr = bufs[-1].addr
    for b in bufs:
        b.close()
    assert not _lib.host_pinned(addr, 16)  # freed (kept in the pool, not live)
    with pytest.raises(_lib.ECInvalidArgument):
        _lib.host_free(addr)  # not live any more
    x = np.zeros(64, np.uint8)
    with pytest.raises(_lib.ECInvalidArgument):
        _lib.host_free(x.ctypes.data)  # never allocated here
    assert _lib.lib.elect_ec_host_free(None) == 0
    p = ctypes.c_void_p()
    assert _lib.lib.elect_ec_host_alloc(0, ctypes.byref(p)) == _lib.EINVAL and not p.value
    # a kept .array keeps its buffer allocated after the HostBuffer itself is dropped
    import gc
    arr = _lib.HostBuffer(4096).array
    gc.collect()
    arr[:] = 7
    owner = arr.base.obj._owner if hasattr(arr.base, "obj") else None
    assert owner is not None and owner.addr and _lib.lib.elect_ec_host_free(owner.addr) == 0
    owner.addr = 0  # freed here by hand; its close() is then a no-op


def test_numa_device_map():
    """elect_ec_host_device_map: the device each calling thread gets (host_device's
    NUMA-aware round robin, host_path.cpp numa_pick), no device needed.  ELECT's
    64 coding threads on a node of 8 GPUs, 4 per socket (the GPU boxes' layout,
    profiles/r06/numa_facts.txt)."""
    from elect_amd import _lib
    devs, nodes = list(range(8)), [0, 0, 0, 0, 1, 1, 1, 1]
    threads = [t % 2 for t in range(64)]  # alternating sockets
    got = _lib.host_device_map(devs, nodes, threads)
    for t, d in enumerate(got):
        assert nodes[d] == threads[t], (t, d)  # every thread on a GPU of its own socket
    for n in (0, 1):  # least loaded within the node: each local GPU 8 threads
        mine = [d for d, x in zip(got, threads) if x == n]
        assert mine[:4] == [4 * n + i for i in range(4)]
        assert sorted(mine.count(d) for d in set(mine)) == [8, 8, 8, 8]
    # a node without a listed GPU, or an unknown node: the least loaded of the whole list
    assert _lib.host_device_map(devs, nodes, [2, 2, 2, -1, -1]) == [0, 1, 2, 3, 4]
    # devices of unknown node (sysfs without NUMA info): round robin for every thread
    assert _lib.host_device_map([3, 5, 6], [-1, -1, -1], [0, 1, 0, 1]) == [3, 5, 6, 3]
    # a subset list (ELECT_EC_DEVICES=2,5): each socket's one GPU
    assert _lib.host_device_map([2, 5], [0, 1], [1, 0, 1, 0]) == [5, 2, 5, 2]
    # uneven sockets: 1 GPU on node 0, 3 on node 1
    assert _lib.host_device_map([0, 1, 2, 3], [0, 1, 1, 1], [0, 1, 1, 1, 1, 0]) == [0, 1, 2, 3, 1, 0]
    # every thread on one socket at its first call (unbound threads can be): local GPUs first, but no GPU
    # ever more than one thread ahead of another, so the other socket's GPUs still get their share
    one_side = _lib.host_device_map(devs, nodes, [0] * 64)
    counts = [one_side.count(d) for d in devs]
    assert max(counts) - min(counts) <= 1, counts
    assert one_side[:4] == [0, 1, 2, 3]  # the first four stay on their socket
    with pytest.raises(Exception):
        _lib.host_device_map([], [], [0])
    # sockets uneven in threads (40 on node 0, 24 on node 1, arriving interleaved): balanced, and each
    # thread local whenever a least loaded GPU is on its socket: 56 of the 64 (the most possible: 8 of
    # node 0's threads must cross to even the load)
    mixed = [1 if i % 8 in (2, 5, 7) else 0 for i in range(64)]
    got = _lib.host_device_map(devs, nodes, mixed)
    counts = [got.count(d) for d in devs]
    assert max(counts) - min(counts) <= 1, counts
    assert sum(nodes[d] == x for d, x in zip(got, mixed)) == 56


def test_pipeline_windows():
    """The windows a lone call is pipelined over (host_path.cpp pipeline_windows):
    they cover [0, len) in order with no empty window, inner boundaries on 64 KiB multiples, at
    most `steps` of them; tapered 4 : ... : 4 : 2 : 1, so the last window (the scatter left after
    the last gather) is the smallest.  ELECT's codeLength in 5 steps: the plan DESIGN quotes."""
    from elect_amd import _lib
    K64 = 1 << 16
    assert _lib.pipeline_windows(4404020, 5) == [0, 1179648, 2359296, 3538944, 4128768, 4404020]
    for length in (1, 4095, K64, (1 << 20) - 7, 1 << 20, 4404020, 3 << 20, 17 << 20, (64 << 20) + 5):
        for steps in range(1, 9):
            for taper in (True, False):
                at = _lib.pipeline_windows(length, steps, taper)
                n = len(at) - 1
                assert at[0] == 0 and at[-1] == length and 1 <= n <= steps, (length, steps, taper, at)
                assert all(a < b for a, b in zip(at, at[1:])), (length, steps, taper, at)
                assert all(b % K64 == 0 for b in at[1:-1]), (length, steps, taper, at)
                w = [b - a for a, b in zip(at, at[1:])]
                if taper and n == steps >= 3 and length >= steps * (1 << 20):
                    assert w[-1] < w[-2] < w[0], (length, steps, w)
                if not taper and n == steps and length >= steps * (1 << 20):
                    assert max(w) - min(w) <= K64 * 2, (length, steps, w)  # equal up to the 64 KiB rounding
    assert _lib.pipeline_windows(0, 3) == [0, 0]
