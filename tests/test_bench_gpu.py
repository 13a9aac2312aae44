"""bench.py end to end on one GPU: the JSON line the driver reads (its keys, the roofline and
CPU-baseline blocks), and the HIP-graph step option.  Short runs (a few steps), in a child process
as the driver starts it."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def test_bench_line_contract():
    d = _bench("--steps", "3", "--warmup", "1", "--cpu-seconds", "0.3", "--no-oja")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "build_id"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["dtype"] == "f32"
    assert "workload" in d["config"] and d["config"]["step_launch"] == "eager"
    roof = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in roof, k
    assert roof["bound"] in ("hbm", "mfma") and 0 < roof["frac"] < 1
    assert abs(roof["frac"] - roof["achieved"] / roof["peak"]) < 1e-3
    cpu = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cpu, k
    assert cpu["value"] > 0 and cpu["kind"] in ("port", "reference")


def test_bench_graph_step_option():
    d = _bench("--steps", "4", "--warmup", "3", "--no-cpu-baseline", "--no-oja", "--no-kernel-profile",
               "--graph", "on")
    assert d["config"]["step_launch"].startswith("hip_graph")
    assert d["value"] > 0 and d["final_loss"] == d["final_loss"]     # finite (not NaN)
