"""bench.py's multi-rank plumbing on CPU (no GPU work): `--gpus N` started bare
starts N ranks itself, the gloo handshake (barrier, max over ranks, per-rank
records) reaches rank 0, and a launcher whose WORLD_SIZE disagrees with --gpus
is refused instead of silently reporting the wrong n_gpus."""
import json
import os
import subprocess
import sys

from tests.conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _env(**extra):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                            "MASTER_PORT")}
    env.update(extra)
    return env


def _json_line(out: str) -> dict:
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bare_gpus_n_starts_n_ranks():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "3", "--launch-check"], capture_output=True, text=True,
                       timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 3
    assert [x["rank"] for x in d["ranks"]] == [0, 1, 2]
    assert all(x["world"] == 3 for x in d["ranks"])
    assert len({x["pid"] for x in d["ranks"]}) == 3  # one process per rank
    assert d["max_over_ranks"] == 3.0
    # the headline's host-path phase: rank 0 starts a child process of its own (no
    # launcher variables: a WORLD_SIZE left in its env would make it refuse) while
    # the other ranks wait at the barrier; the child's record reaches the line
    hp = d["hostpath_child"]
    assert hp["verified"] and hp["devices"] == 3, hp
    assert hp["child"]["n_gpus"] == 1 and hp["child"]["ranks"][0]["pid"] not in {x["pid"] for x in d["ranks"]}


def test_single_rank_needs_no_launcher():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "1", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 1 and len(d["ranks"]) == 1


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--launch-check"], capture_output=True, text=True,
                       timeout=120, env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), cwd=ROOT)
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


def test_launch_command_shape():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    captured = {}

    def fake_run(cmd, *a, **k):
        captured["cmd"] = cmd

        class R:
            returncode = 0
        return R()

    import subprocess as sp
    real = sp.run
    sp.run = fake_run
    try:
        assert mod.launch_ranks(8, ["--gpus", "8", "--steps", "3"]) == 0
    finally:
        sp.run = real
    cmd = captured["cmd"]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--master-addr=127.0.0.1" in cmd and "--nnodes=1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod2", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_hostpath_child_command_and_env():
    """The host path the headline line measures over the job's devices: ELECT's
    64 callers (concurrent_ec) on ELECT's codeLength, batching on, devices 0..N-1;
    the child's environment carries no launcher rank variables."""
    mod = _bench_module()
    cmd = mod.hostpath_child_cmd(8)
    a = dict(zip(cmd[2::2], cmd[3::2]))
    assert a["--config"] == "hostpath" and a["--threads"] == "64" and a["--host-devices"] == "8"
    assert a["--host-chunk"] == "4404020" and a["--batch"] == "1"
    old = dict(os.environ)
    try:
        os.environ.update(WORLD_SIZE="8", RANK="3", LOCAL_RANK="3", MASTER_ADDR="127.0.0.1", MASTER_PORT="1",
                          TORCHELASTIC_RUN_ID="x")
        env = mod.child_env()
    finally:
        os.environ.clear()
        os.environ.update(old)
    assert not {"WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID"} & set(env)
    assert env.get("PATH") == os.environ.get("PATH")


def test_hostpath_child_timeout_is_a_record_not_a_crash():
    """A host-path child that outlives its limit becomes an unverified record on
    rank 0 (the line still prints, and fails), not an exception that would leave
    the other ranks waiting at the barrier; the limit sits inside the gloo timeout."""
    mod = _bench_module()
    # every child of the run together stays inside the 10-minute gloo timeout
    assert mod.HOSTPATH_TOTAL_TIMEOUT_S < 10 * 60 and mod.HOSTPATH_CHILD_TIMEOUT_S <= mod.HOSTPATH_TOTAL_TIMEOUT_S
    mod.HOSTPATH_CHILD_TIMEOUT_S = 1
    res = mod.hostpath_all_devices(None, 1, 0, child=[sys.executable, "-c", "import time; time.sleep(30)"])
    assert res["verified"] is False and "timed out" in res["error"], res
    # a spent shared deadline: the next child is not started at all
    mod.HOSTPATH_CHILD_TIMEOUT_S, mod.HOSTPATH_TOTAL_TIMEOUT_S = 280, 0
    res = mod.hostpath_all_devices(None, 1, 0, child=[sys.executable, "-c", "print('{}')"])
    assert res["verified"] is False and "timed out" in res["error"], res


def test_cpu_baseline_thread_points():
    """The CPU baseline sweeps the cgroup quota, twice it, 64 and the affinity
    mask (capped at the mask), and reports the best point, so a 16-CPU quota under
    a 256-CPU mask is not reported as a 256-thread oversubscribed run."""
    mod = _bench_module()
    assert mod.cpu_thread_points({"affinity": 256, "quota_cores": 16.0}) == [16, 32, 64, 256]
    assert mod.cpu_thread_points({"affinity": 8, "quota_cores": None}) == [8]
    assert mod.cpu_thread_points({"affinity": 8, "quota_cores": 16.0}) == [8]
    assert mod.cpu_thread_points({"affinity": 128, "quota_cores": 2.5}) == [3, 6, 64, 128]


def test_metric_names_the_chunk():
    mod = _bench_module()
    assert mod.chunk_name(65536) == "64 KiB" and mod.chunk_name(1 << 20) == "1 MiB"
    assert mod.chunk_name(1024) == "1 KiB" and mod.chunk_name(4404020) == "4404020 B"


def test_parity_rows_check_sees_every_row():
    """bench.py's verified flag covers every parity row: the timed
    decode (erase 0 from survivors 1..k) never reads parity row 1 of RS(6,4), so a
    corrupted row 1 passes it; parity_rows_verified rebuilds data 0..m-1 from the
    other data and ALL parity units and catches it.  A fake decode_batch over CPU
    tensors, built on the oracle (test infrastructure), stands in for the GPU."""
    import numpy as np
    import torch
    from oracle import ec_oracle as orc
    mod = _bench_module()
    k, m, B, L = 4, 2, 3, 96

    class Coder:
        pass
    coder = Coder()
    coder.k, coder.m = k, m
    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, (B, k, L), dtype=np.uint8)
    par = np.stack([np.stack(orc.Encoder(k, m).encode(list(data[b]))) for b in range(B)])
    st = torch.from_numpy(np.concatenate([data, par], 1))

    def fake_decode(coder, stripe, surv, erased, out, inputs_by_unit=False):
        assert inputs_by_unit
        s = stripe.numpy()
        for b in range(s.shape[0]):
            got = orc.decode(k, m, [s[b, u] for u in surv], surv, erased)[1]
            for i, g in enumerate(got):
                out[b, i] = torch.from_numpy(np.asarray(g))

    def timed_check(stripe):  # what the timed region's decode verifies
        out = torch.empty((B, 1, L), dtype=torch.uint8)
        fake_decode(coder, stripe, list(range(1, k + 1)), [0], out, inputs_by_unit=True)
        return bool(torch.equal(out[:, 0], stripe[:, 0]))

    assert mod.parity_rows_verified(coder, st, fake_decode) and timed_check(st)
    bad = st.clone()
    bad[1, k + 1, 7] ^= 0x40  # parity row 1 of stripe 1
    assert timed_check(bad)  # the timed decode alone cannot see it
    assert not mod.parity_rows_verified(coder, bad, fake_decode)
    bad = st.clone()
    bad[2, k, 0] ^= 1  # parity row 0
    assert not mod.parity_rows_verified(coder, bad, fake_decode)
