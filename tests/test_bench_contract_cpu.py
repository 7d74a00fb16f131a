"""The committed bench line of the latest round (profiles/<round>/bench_final.json,
the driver's command `bench.py --gpus 1 --steps 20 --warmup 5`) keeps the
driver's JSON contract, and its numbers agree with each other:

- the contract keys and types (metric, value, unit, n_gpus, steps, warmup,
  ms_per_step, higher_is_better, scaling, vs_baseline, dtype, data, config);
- roofline: bound / achieved / peak / unit / frac / traffic, frac = achieved /
  peak, achieved = the algorithmic bytes per launch / the encode's time, traffic
  within 0.1 % of the algorithmic bytes;
- cpu_baseline: value / unit / cores / kind / sample;
- value = the step's data (encode k*L + decode k*L per stripe) / ms_per_step;
- the GPU-clock region time is not longer than the wall time, and the per-kernel
  times fit inside a step.
No device needed: this reads the committed file."""
import glob
import json
import os

from tests.conftest import ROOT


def _latest_line():
    rounds = sorted(d for d in glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]"))
                    if os.path.exists(os.path.join(d, "bench_final.json")))
    assert rounds, "no profiles/rNN/bench_final.json"
    return json.load(open(os.path.join(rounds[-1], "bench_final.json")))


def test_contract_keys_and_types():
    d = _latest_line()
    for key, typ in (("metric", str), ("value", float), ("unit", str), ("n_gpus", int), ("steps", int),
                     ("warmup", int), ("ms_per_step", float), ("higher_is_better", bool), ("scaling", str),
                     ("dtype", str), ("data", str), ("config", dict)):
        assert isinstance(d[key], typ), key
    assert d["vs_baseline"] is None  # BASELINE.md holds no published number for this metric
    assert d["n_gpus"] == 1 and d["steps"] == 20 and d["warmup"] == 5  # the driver's command
    assert d["higher_is_better"] is True and d["scaling"] == "weak" and d["verified"] is True
    assert "workload" in d["config"] and d["dtype"] == "u8"


def test_roofline_is_self_consistent():
    d = _latest_line()
    rf = d["roofline"]
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in rf, key
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and rf["peak"] == 8000.0
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    enc = d["kernels"]["encode"]
    assert abs(rf["algorithmic_bytes_per_launch"] / (enc["ms"] * 1e-3) / 1e9 - rf["achieved"]) / rf["achieved"] < 2e-3
    assert abs(rf["traffic"] / rf["algorithmic_bytes_per_launch"] - 1) < 1e-3  # PMC bytes: no wasted re-reads


def test_cpu_baseline_fields():
    cb = _latest_line()["cpu_baseline"]
    for key in ("value", "unit", "cores", "kind", "sample"):
        assert key in cb, key
    assert cb["kind"] in ("port", "reference") and cb["value"] > 0 and cb["cores"] >= 1


def test_value_matches_the_step_time():
    d = _latest_line()
    c = d["config"]
    data = 2 * c["stripes_per_gpu"] * c["k"] * c["chunk_bytes"]  # encode k*L + decode k*L per stripe
    assert abs(data / (d["ms_per_step"] * 1e-3) / (1 << 30) - d["value"]) / d["value"] < 2e-3
    assert d["gpu_ms_per_step"] <= d["ms_per_step"] * 1.001
    k = d["kernels"]
    assert k["encode"]["ms"] + k["decode_1erasure"]["ms"] <= d["ms_per_step"] * 1.02
