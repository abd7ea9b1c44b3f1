"""bench.py's output contract on a small workload (GPU): one JSON line with the driver's keys, the
roofline and cpu_baseline objects, and a Gram–Schmidt block — run as the driver runs it (a child
process), so a broken bench shows up in the GPU suite and not only at round end."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_json_contract(gpu):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--E", "2000", "--steps", "2", "--warmup", "1",
                        "--cpu-E", "64", "--cpu-budget", "1.0"], capture_output=True, text=True, timeout=240,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["dtype"] == "f64"
    assert d["unit"] == "GB/s" and d["higher_is_better"] is True and d["scaling"] == "strong"
    assert 0 < d["value"] < 8000.0 and d["ms_per_step"] > 0
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["peak"] == 8000.0 and r["unit"] == "GB/s"
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["unit"] == "GB/s"
    assert d["ritz_top8_rel_err"] < 1e-10
    assert d["gram_schmidt"]["gs_ms_per_factorisation"] <= d["ms_per_step"]
