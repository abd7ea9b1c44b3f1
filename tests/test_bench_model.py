"""bench.py's byte models (CPU): the executed-bytes model of each mode against the SURVEY.md §8(d)
4-pass CGS2 model, and the kernel-family bookkeeping the roofline line relies on."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_byte_models_order():
    N, N_w, n_v, m = 100_014_464, 90_472_448, 22_618_112, 128
    survey = bench.survey_model_bytes(N, N_w, n_v, m)
    cgs2 = bench.executed_bytes(N, N_w, n_v, m, "cgs2")
    dcgs2 = bench.executed_bytes(N, N_w, n_v, m, "dcgs2")
    ref = sum(bench.reference_step_bytes(N, N_w, n_v, j) for j in range(1, m + 1))
    assert dcgs2 < cgs2 < survey < ref
    # 4 -> 3 -> 2 reads of the basis per step (the basis dominates at m = 128); the reference's MGS2
    # with its per-column copies ~20 jN
    assert 0.70 < cgs2 / survey < 0.80
    assert 0.62 < dcgs2 / cgs2 < 0.72
    assert 4.5 < ref / survey < 5.5
    for mode in ("mgs2", "mgs2-icwy", "dcgs2-native", "cgs2-native"):
        assert bench.executed_bytes(N, N_w, n_v, m, mode) > 0


def test_survey_model_matches_worked_total():
    # config 3, m=128 -> sum_j B(j) = 26.03 TB (+ 3N per step for the matvec)
    N, N_w, n_v, m = 100_014_464, 90_472_448, 22_618_112, 128
    tot = bench.survey_model_bytes(N, N_w, n_v, m) - m * 8.0 * 3 * N
    assert abs(tot / 1e12 - 26.03) < 0.01


def test_lagged_mode_byte_model():
    """``bench.py --mode mgs2-lagged`` has a byte model — the DCGS2 kernels' bytes (the
    same two-vector dot and dual update per step) plus the weights of its closing fused norm — and
    its native twin moves the same bytes."""
    import bench

    N, N_w, n_v, m = 100_014_464, 90_472_448, 22_618_112, 128
    d = bench.executed_bytes(N, N_w, n_v, m, "dcgs2")
    lg = bench.executed_bytes(N, N_w, n_v, m, "mgs2-lagged")
    assert lg == d + 8.0 * n_v
    assert bench.executed_bytes(N, N_w, n_v, m, "mgs2-lagged-native") == lg
