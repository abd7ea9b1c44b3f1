"""The N > 1 bench line is as complete as the N = 1 line: ``bench.py --dry-line``
runs the real line assembly (``bench_line``) and the real finish (every rank leaves the gloo
group, then rank 0 times the CPU lines and prints) over fabricated measurements, at world sizes
1, 2, 4 and 8 through bench.py's own launcher.  Every line must carry the same keys — roofline,
cpu_baseline (with its host, full-size and estimate fields), phases, all-reduce statistics,
devices and distinct_devices — and the CPU lines must be timed on rank 0 at every world size."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _port(k: int) -> str:
    w = os.environ.get("PYTEST_XDIST_WORKER", "gw0")
    return str(23000 + 40 * int(w[2:] or 0) + k)


def _line(world: int, port_k: int) -> dict:
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(MASTER_PORT=_port(port_k), OMP_NUM_THREADS="2")
    p = subprocess.run([sys.executable, BENCH, "--gpus", str(world), "--dry-line", "--E", "64", "--m", "8",
                        "--cpu-E", "8", "--cpu-E-1core", "8", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout   # ONE line, from rank 0
    return json.loads(lines[0])


def _keys(d: dict, prefix=""):
    out = set()
    for k, v in d.items():
        out.add(prefix + k)
        if isinstance(v, dict) and k in ("roofline", "gram_schmidt", "cpu_baseline", "cpu_baseline_1core",
                                         "cpu_optimised", "config"):
            out |= _keys(v, prefix + k + ".")
    return out


@pytest.fixture(scope="module")
def lines():
    return {w: _line(w, i) for i, w in enumerate((1, 2, 4, 8))}


def test_every_world_size_carries_the_one_gpu_fields(lines):
    ref = _keys(lines[1])
    for w in (2, 4, 8):
        assert _keys(lines[w]) == ref, (w, _keys(lines[w]) ^ ref)
    for w, d in lines.items():
        assert d["n_gpus"] == w and d["world"] == w and len(d["devices"]) == w
        assert "distinct_devices" in d and d["phases"] and d["roofline"]["kernel"] == "dcgs2_update"
        gs = d["gram_schmidt"]
        assert gs["allreduces_per_factorisation"] == (0 if w == 1 else 8)
        assert gs["allreduce_ms_per_factorisation_max_over_ranks"] >= gs["allreduce_ms_per_factorisation_min_over_ranks"]
        assert d["dry_line"].startswith("fabricated")


def test_cpu_lines_timed_at_every_world_size(lines):
    for w, d in lines.items():
        for key in ("cpu_baseline", "cpu_baseline_1core", "cpu_optimised"):
            c = d[key]
            assert c is not None and c["value"] > 0 and c["seconds_per_factorisation_measured"] is True, (w, key)
            assert c["gpu_ms_per_factorisation"] == d["ms_per_step"]
            # E=64 is not BASELINE's workload: no full-size measurement applies, so the ratio is an
            # estimate and the measured-only fields are null
            assert c["full_size_run"] is None and c["seconds_per_factorisation_N1e8"] is None
            assert c["time_to_solution_ratio_cpu_over_gpu"] is None and c["time_to_solution_ratio_estimate"] > 0
        assert d["cpu_baseline"]["cores"] == d["cpu_baseline"]["host"]["threads"] == 2
        assert d["cpu_baseline_1core"]["cores"] == 1
        assert "1.7x" in d["cpu_baseline"]["sample"]


def test_measured_full_size_run_leads(tmp_path, monkeypatch):
    """With a full-size measurement for the same algorithm and thread count, the seconds at N=1e8
    and the CPU/GPU ratio are the measured ones; the sample's N-scaling is kept beside them."""
    import bench

    c = {"seconds_scaled_from_sample_N1e8": 600.0}
    full = bench.cpu_full_size_run(44176, 128, 2000.0, "mgs2", 16)
    assert full is not None and full["threads"] == 16
    bench.lead_with_measured(c, full, 2000.0)
    s = full["seconds_per_factorisation"]
    assert c["seconds_per_factorisation_N1e8"] == s and c["time_to_solution_ratio_cpu_over_gpu"] == round(s / 2.0, 1)
    assert c["sample_scaled_over_measured"] == round(600.0 / s, 3)
    assert "measured at full size" in c["seconds_per_factorisation_N1e8_source"]
    # another thread count: the measurement does not apply
    assert bench.cpu_full_size_run(44176, 128, 2000.0, "mgs2", 1) is None


def test_shard_traffic_lookup(tmp_path, monkeypatch):
    """A rank's PMC traffic comes from a profile of its own shard size (traffic_E<E>.json)."""
    import bench

    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / "traffic_latest.json").write_text(json.dumps({"kernel_family": "dcgs2_update", "E": 44176, "m": 128,
                                                          "hbm_bytes_per_launch": 5.4e10, "tag": "a"}))
    (prof / "traffic_E5522.json").write_text(json.dumps({"kernel_family": "dcgs2_update", "E": 5522, "m": 128,
                                                         "hbm_bytes_per_launch": 6.7e9, "tag": "b"}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    assert bench.find_traffic("dcgs2_update", 44176, 128)[0] == 5.4e10
    t, src = bench.find_traffic("dcgs2_update", 5522, 128)
    assert t == 6.7e9 and src["file"] == os.path.join("profiles", "traffic_E5522.json") and src["E_shard"] == 5522
    assert bench.find_traffic("dcgs2_update", 11044, 128) == (None, None)
    assert bench.find_traffic("block_dot2", 5522, 128) == (None, None)


def test_driver_launcher_two_ranks_one_line():
    """The driver's own launcher (``python -m torch.distributed.run --nnodes=1 --nproc-per-node 2
    --master-addr 127.0.0.1 --master-port P bench.py --gpus 2 ...``): the ranks leave the group, rank 0
    prints ONE complete line, and torch.distributed.run's agent reports success.  (torch.distributed.run
    also parses long options after the script name by prefix, so ``--m`` would be taken for its own.)"""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(OMP_NUM_THREADS="2", NKV_BACKEND="gloo")
    p = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", _port(9), BENCH, "--gpus", "2", "--dry-line",
                        "--E", "64", "--cpu-E", "8", "--cpu-E-1core", "8", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["world"] == 2 and d["cpu_baseline"]["value"] > 0 and d["roofline"]["kernel"] == "dcgs2_update"
