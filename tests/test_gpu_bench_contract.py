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


def _gbs_fields(d, path=""):
    """Every (path, value) of a GB/s-valued field: keys naming gbs / gbps, the top-level value and
    roofline.achieved (unit GB/s)."""
    if isinstance(d, dict):
        for k, v in d.items():
            p = f"{path}.{k}"
            if isinstance(v, (dict, list)):
                yield from _gbs_fields(v, p)
            elif ("gbs" in k or "gbps" in k) and (v is None or isinstance(v, (int, float))):
                yield p, v
        if d.get("unit") == "GB/s":
            for k in ("value", "achieved"):
                if isinstance(d.get(k), (int, float)):
                    yield f"{path}.{k}", d[k]
    elif isinstance(d, list):
        for i, v in enumerate(d):
            yield from _gbs_fields(v, f"{path}[{i}]")


def _one_byte_model(d, check_peak=False):
    """One byte model per line: every GB/s figure is executed bytes / measured time; SURVEY 8(d)'s
    4-pass model appears only as the dimensionless survey_model_time_ratio.  ``check_peak``: no GB/s
    field above roofline.peak (at BASELINE size, where no vector fits the 256 MiB Infinity Cache)."""
    gbs = list(_gbs_fields(d))
    assert len(gbs) >= 8, gbs
    if check_peak:
        for path, v in gbs:
            assert v is None or v <= d["roofline"]["peak"], (path, v)
    assert d["survey_model_time_ratio"] > 0 and d["gram_schmidt"]["survey_model_time_ratio"] > 0
    for k in ("effective_gbs_survey_model", "survey_headline_gbs", "last_step_survey_gbs",
              "gpu_effective_gbs_same_model"):
        assert k not in json.dumps(d), k


def test_bench_full_size_no_gbs_field_above_peak(gpu):
    """The driver's workload (config 3, N=100,014,464, m=128), one timed step: no GB/s field of the
    line exceeds the 8 TB/s peak, the roofline fraction is the dominant kernel's."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "1", "--no-cpu",
                        "--no-ks"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    d = json.loads(lines[0])
    assert d["config"]["N"] == 100_014_464 and d["config"]["m"] == 128
    _one_byte_model(d, check_peak=True)
    assert d["roofline"]["infinity_cache"] is None and 0.5 < d["roofline"]["frac"] < 1.0
    assert d["survey_model_time_ratio"] > 1.0   # faster than a 4-pass CGS2 could be at roofline


def test_bench_json_contract(gpu):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--E", "2000", "--steps", "2", "--warmup", "1",
                        "--cpu-E", "64", "--cpu-E-1core", "8"],
                       capture_output=True, text=True, timeout=240,
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
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and cb["unit"].startswith("GB/s")
    assert cb["cores"] == cb["host"]["threads"] and cb["seconds_scaled_from_sample_N1e8"] > 0
    # E=2000 is not BASELINE's workload: no full-size CPU measurement applies, the ratio is an estimate
    assert cb["seconds_per_factorisation_N1e8"] is None and cb["time_to_solution_ratio_estimate"] > 1
    _one_byte_model(d)
    assert d["world"] == 1 and d["gram_schmidt"]["allreduce_ms_per_factorisation"] == 0
    assert len(d["devices"]) == 1 and d["devices"][0]["pci"] and d["distinct_devices"] is True
    assert d["devices"][0]["name"]   # the marketing name, or the ISA name where libdrm has none
    ks = d["krylov_schur_leg"]   # k_dim=m=128, schur_tgt=4: converges in the first factorisation
    assert ks["k_dim"] == 128 and ks["schur_tgt"] == 4 and ks["converged"] >= 4 and ks["top4_rel_err_vs_exact"] < 1e-10
    kr = d["krylov_schur_restart_leg"]   # a clustered spectrum: real 128-column restarts
    assert kr["schur_cnt"] >= 1 and kr["converged"] >= 4 and kr["top4_rel_err_vs_exact"] < 1e-10
    for leg in (ks, kr):
        assert leg["relatively_converged"] >= 4 and leg["ritz_rel_err_vs_exact"] < 1e-10
    assert d["ritz_top8_rel_err"] < 1e-10
    assert d["gram_schmidt"]["gs_ms_per_factorisation"] <= d["ms_per_step"]


def test_bench_plain_command_two_gloo_ranks_one_gpu(gpu):
    """``python bench.py --gpus 2`` (no torchrun) spawns two ranks; with NKV_BACKEND=gloo both share
    the one GPU of this box.  One JSON line with n_gpus 2, and the same Ritz values as one rank."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["NKV_BACKEND"] = "gloo"
    common = ["--E", "2000", "--m", "48", "--steps", "1", "--warmup", "1", "--no-cpu", "--no-restart", "--no-ks"]
    outs = {}
    for n in (1, 2):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *common],
                           capture_output=True, text=True, timeout=300, cwd=ROOT, env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        outs[n] = json.loads(lines[0])
    d2 = outs[2]
    assert d2["n_gpus"] == 2 and d2["world"] == 2 and d2["backend"] == "gloo"
    # both ranks drove the one GPU: the line says so (an 8-GPU RCCL line must say true)
    assert len(d2["devices"]) == 2 and d2["distinct_devices"] is False
    g = d2["gram_schmidt"]
    assert g["allreduces_per_factorisation"] >= 48 and g["allreduce_ms_per_factorisation_max_over_ranks"] > 0
    assert g["gs_ms_per_factorisation_min_over_ranks"] <= g["gs_ms_per_factorisation_max_over_ranks"]
    assert abs(d2["ritz_top8_rel_err"] - outs[1]["ritz_top8_rel_err"]) < 1e-12
    assert d2["ritz_converged"] == outs[1]["ritz_converged"]


def test_bench_two_ranks_with_restart_and_krylov_schur_legs(gpu):
    """The driver's multi-GPU line runs the WHOLE bench on every rank, the restart and both
    Krylov–Schur legs included (outside the timed region).  Two gloo ranks sharing this box's GPU
    against one rank, small E: the legs complete on both ranks and make the same discrete choices
    (restart count, mstart and converged-count histories), with the same converged values."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["NKV_BACKEND"] = "gloo"
    common = ["--E", "400", "--m", "48", "--steps", "1", "--warmup", "1", "--no-cpu"]
    outs = {}
    for n in (1, 2):
        p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *common],
                           capture_output=True, text=True, timeout=400, cwd=ROOT, env=env)
        assert p.returncode == 0, p.stderr[-3000:]
        lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, p.stdout
        outs[n] = json.loads(lines[0])
    d1, d2 = outs[1], outs[2]
    assert d2["world"] == 2
    for leg in ("krylov_schur_leg", "krylov_schur_restart_leg"):
        a, b = d1[leg], d2[leg]
        assert a is not None and b is not None
        for key in ("schur_cnt", "mstart_history", "cnt_history", "converged", "relatively_converged"):
            assert a[key] == b[key], (leg, key, a[key], b[key])
        assert b["top4_rel_err_vs_exact"] < 1e-10
    assert d2["krylov_schur_restart_leg"]["schur_cnt"] >= 1
    assert d1["restart"]["mstart"] == d2["restart"]["mstart"]
    assert d2["restart"]["rotate_kept_ms"] > 0 and d2["restart"]["rotate_full_ms"] > 0
    assert 0 < d2["restart"]["rotate_kept_steady_frac_hbm"] < 1
    assert d2["restart"]["rotate_wide_kept"] >= 17 and 0 < d2["restart"]["rotate_wide_frac_hbm"] < 1
