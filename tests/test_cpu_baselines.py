"""The timed CPU comparison lines of bench.py: the optimised blocked CGS2
(oracle/cpu_cgs2.c) must build the same Hessenberg column as the reference-order MGS2 restatement
(rounding only) — otherwise its GB/s would be for different work.  Likewise the -Ofast build of the
restatement (oracle/liboracle_prod.so) that cpu_baseline times."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import oracle as orc  # noqa: E402

from nekstab_next_amd import synthetic as syn  # noqa: E402
from nekstab_next_amd.layout import box3d_layout  # noqa: E402


def test_cpu_cgs2_matches_mgs2_hessenberg():
    lay = box3d_layout(8)
    L = orc.OLayout(lay.n_v, lay.n_p, lay.n_wf, False, lay.ldim)
    w = syn.mass_weights(lay)
    d, _ = syn.laplacian_shift_invert(lay)
    dref = syn.to_reference_order(lay, d)
    c = ctypes.byref(L.c)
    m = 12
    Hs = []
    steps = (orc.lib().orc_update_hessenberg, orc.cgs2_lib().cpu_cgs2_update_hessenberg,
             orc.prod_lib().orc_update_hessenberg)  # the -Ofast build bench.py times
    for step in steps:
        orc.cgs2_lib().cpu_cgs2_set_threads(4)
        Q = np.zeros((m + 1, L.len))
        Q[0] = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
        H = np.zeros((m + 1, m))
        f, wrk = L.zeros(), L.zeros()
        for j in range(1, m + 1):
            orc.lib().orc_op_diag(c, dref, Q[j - 1], f, 0.0)
            col = np.zeros(j + 1)
            step(c, w, col, f, Q[:j], j, wrk)
            Q[j] = f
            H[: j + 1, j - 1] = col
        Hs.append(H)
    for H in Hs[1:]:
        np.testing.assert_allclose(H, Hs[0], rtol=0, atol=1e-12 * np.abs(Hs[0]).max())


def test_bench_cpu_baseline_leg_small():
    """bench.py's cpu_baseline leg on a tiny sample (CPU only): the reported object keeps the
    contract's keys and names the build it timed."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    import bench

    for variant in ("mgs2", "cgs2"):
        r = bench.cpu_baseline(8, 6, 2, variant=variant, fit_js=(1, 3, 6))
        assert {"value", "unit", "cores", "kind", "sample"} <= set(r)
        assert r["unit"].startswith("GB/s") and r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
        assert "one complete m=6 factorisation" in r["sample"] and "warm-up" in r["sample"]
    assert "-Ofast" in bench.cpu_baseline(8, 4, 1)["sample"]


def test_bench_cpu_baseline_measures_one_factorisation():
    """bench.cpu_baseline times one complete m-step factorisation (measured, not
    extrapolated from single steps), reports its value in the bytes the timed algorithm executes (the
    GPU value's basis), seconds to solution scaled to N=1e8, and the round-3 fit
    (steps js only) with its error against the measured total."""
    import bench

    r = bench.cpu_baseline(16, 16, 2, fit_js=(1, 4, 8, 16))
    assert r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
    assert r["seconds_per_factorisation_measured"] is True
    assert "reference MGS2" in r["executed_bytes_model"] and "executes" in r["unit"]
    assert sorted(r["step_seconds"]) == [1, 4, 8, 16]
    assert sum(r["step_seconds"].values()) < r["seconds_per_factorisation_sample"]
    fc = r["fit_check"]
    assert fc["js"] == [1, 4, 8, 16] and fc["fitted_total_s"] > 0
    assert -1.0 < fc["rel_err_vs_measured"] < 10.0
    lay_N = box3d_layout(16).N
    assert abs(r["seconds_scaled_from_sample_N1e8"] / r["seconds_per_factorisation_sample"]
               - bench.N_HEADLINE / lay_N) < 0.05 * bench.N_HEADLINE / lay_N
    o = bench.cpu_baseline(16, 16, 2, variant="cgs2")
    assert o["value"] > 0 and "4-pass CGS2" in o["executed_bytes_model"]


def test_host_threads_respects_cpu_share(monkeypatch):
    import bench

    monkeypatch.setenv("OMP_NUM_THREADS", "3")
    h = bench.host_threads()
    assert h["threads"] == min(3, h["affinity_cpus"]) and h["nproc"] >= 1
    monkeypatch.delenv("OMP_NUM_THREADS")
    h = bench.host_threads()
    assert 1 <= h["threads"] <= h["affinity_cpus"]


def test_reference_byte_model_is_about_20jN():
    import bench

    N, N_w, n_v = 100_014_464, 90_472_448, 22_618_112
    per_col = (bench.reference_step_bytes(N, N_w, n_v, 101) - bench.reference_step_bytes(N, N_w, n_v, 100)) / 8
    assert 18 * N < per_col < 21 * N


def test_full_size_cpu_run_is_the_committed_measurement():
    """The full-size CPU factorisation (profiles/cpu_full_size_latest.json, measured on the GPU box's
    host at BASELINE's E=44,176) is read by bench.py only for that workload, and
    the bounded sample's N-scaling stays within 40 % of it."""
    import json

    import bench

    fj = json.load(open(os.path.join(bench.ROOT, "profiles", "cpu_full_size_latest.json")))
    r = fj["runs"][0]
    assert r["E"] == 44176 and fj["m"] == 128 and r["seconds_per_factorisation_N1e8"] == \
        r["seconds_per_factorisation_sample"]
    assert fj["tag"] and fj["head"]
    f = bench.cpu_full_size_run(44176, 128, 2000.0)
    assert f["seconds_per_factorisation"] == r["seconds_per_factorisation_sample"]
    assert f["time_to_solution_ratio_cpu_over_gpu"] == round(f["seconds_per_factorisation"] / 2.0, 1)
    assert bench.cpu_full_size_run(5522, 128, 2000.0) is None and bench.cpu_full_size_run(44176, 64, 1.0) is None
    # the r05e bench's bounded sample (N=4.5e6, scaled x22) against the full-size measurement
    b = json.loads(open(os.path.join(bench.ROOT, "profiles", "r05e_bench_n1.json")).read().strip().splitlines()[-1])
    scaled = b["cpu_baseline"]["seconds_per_factorisation_N1e8"]
    assert 0.7 < f["seconds_per_factorisation"] / scaled < 1.4
