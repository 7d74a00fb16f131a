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
