"""bench.py's timing machinery on the GPU (round 4: the timed steps carry no
events; split_pass() times each launch in the steps right after).

- bench.Event (a device-scope-release HIP event on torch's current stream)
  measures the same interval as torch.cuda.Event;
- timed() reports the region on the GPU's clock next to the wall clock, and
  the GPU region is not longer than the wall time;
- split_pass() returns one mean per launch position, and their sum is the
  step's GPU time up to the launch gaps (no event inflates the timed steps)."""
import importlib.util
import os

import pytest
import torch

from tests.conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench():
    spec = importlib.util.spec_from_file_location("bench_timing", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _workload(dev):
    from elect_amd.batch import decode_batch, encode_batch
    from elect_amd.coder import RSCoder
    k, m, L, B = 4, 2, 65536, 2048  # a step of ~0.2 ms: the events' few us are small beside it
    coder = RSCoder(k, m)
    st = torch.empty((B, k + m, L), dtype=torch.uint8, device=dev)
    st[:, :k] = torch.randint(0, 256, (B, k, L), dtype=torch.uint8, device=dev)
    out = torch.empty((B, 1, L), dtype=torch.uint8, device=dev)
    enc = lambda: encode_batch(coder, st[:, :k], st[:, k:])  # noqa: E731
    dec = lambda: decode_batch(coder, st, [1, 2, 3, 4], [0], out, inputs_by_unit=True)  # noqa: E731
    return st, out, enc, dec


def test_device_scope_event_matches_torch_event(dev):
    bench = _bench()
    _, _, enc, _ = _workload(dev)
    enc()
    torch.cuda.synchronize()
    for scope in ("device", "system"):
        bench.event_release = scope
        a, b = bench.Event(), bench.Event()
        ta, tb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ta.record()
        a.record()
        for _ in range(10):
            enc()
        b.record()
        tb.record()
        b.synchronize()
        torch.cuda.synchronize()
        ours, theirs = a.elapsed_time(b), ta.elapsed_time(tb)
        assert ours > 0 and abs(ours - theirs) <= 0.05 * theirs + 0.02, (scope, ours, theirs)
    bench.event_release = "device"


def test_timed_and_split_pass(dev):
    bench = _bench()
    st, out, enc, dec = _workload(dev)
    steps = 20
    info = {}
    dt, submit = bench.timed(lambda: (enc(), dec()), steps, 3, 1, 0.0, info)
    wall_ms = dt / steps * 1e3
    gpu_ms = info["gpu_ms_per_step"]
    assert 0 < gpu_ms <= wall_ms * 1.02, (gpu_ms, wall_ms)
    assert submit < wall_ms  # the host issues a step faster than the GPU runs it
    means, per = bench.split_pass(lambda i: [enc, dec], steps)
    assert len(means) == 2 and len(per) == 2 and all(len(x) == steps for x in per)
    assert all(x > 0 for x in means)
    # the launches' own times add up to the event-free step, up to the launch gaps and
    # the few microseconds each event record adds around a launch (~4 us, two launches)
    assert 0.85 * gpu_ms <= sum(means) <= 1.05 * gpu_ms + 0.012, (means, gpu_ms)
    assert torch.equal(out[:, 0], st[:, 0])  # the launches coded: erase-0 decode restores unit 0
