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
        r = bench.cpu_baseline(8, 6, 2, 5.0, variant=variant)
        assert {"value", "unit", "cores", "kind", "sample"} <= set(r)
        assert r["unit"] == "GB/s" and r["kind"] == "port" and r["cores"] == 2 and r["value"] > 0
        assert "steps j=1..6 of m=6" in r["sample"]
    assert "-Ofast" in bench.cpu_baseline(8, 4, 1, 5.0)["sample"]
