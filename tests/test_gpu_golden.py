"""GPU parity against the committed golden fixtures (tests/golden/, see make_golden.py) — the HIP
path only, no oracle in the process.  The fixtures are the oracle's runs with its dense steps on
Intel MKL (the LAPACK the reference's build links, bin/mks:32-44); the product's host path runs
SciPy's OpenBLAS, so every restart decision below is taken by a different LAPACK than the one that
made the fixture.

Gates: restart counts, mstart and converged-count sequences identical; Ritz values
in the comparison set (converged + top-8 by modulus) within 1e-10 relative; the first
factorisation's Hessenberg matrix within 1e-12·max|H| (1e-11 for the 3e8-graded config-3 spectrum);
GMRES inner residual history within 1e-8 relative.  Config 2 runs on the reference's own data: the
seed is the cylinder base flow ``examples/cylinder/BF_1cyl0.f00001`` (U, V, P) on the real mesh."""
import os

import numpy as np
import pytest

from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.arnoldi import HessenbergDev, arnoldi_factorization
from nekstab_next_amd.config import GmresConfig, KrylovSchurConfig
from nekstab_next_amd.gmres import ts_gmres
from nekstab_next_amd.krylov_schur import krylov_schur, prepare_seed
from nekstab_next_amd.layout import NekLayout, box3d_layout, cylinder_layout
from nekstab_next_amd.operators import DiagOperator, Rot2Operator, ShiftedOperator
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name):
    return np.load(os.path.join(G, name))


def _compare_ks(res, z, tol=1e-10):
    assert "Math Kernel Library" in str(z["lapack"])
    assert res.schur_cnt == int(z["schur_cnt"])
    assert res.mstart_history == z["mstart"].tolist()
    assert res.cnt_history == z["cnt"].tolist()
    if "selected" in z:   # the kept eigenvalues of every restart equal MKL's selection
        assert len(res.selected_history) == z["selected"].shape[0]
        for got, want in zip(res.selected_history, z["selected"]):
            assert int(np.count_nonzero(got)) == int(np.count_nonzero(want))
    vals = z["vals"]
    sel = sorted(set(np.nonzero(z["residual"] < 1e-6)[0].tolist()) | set(range(min(8, len(vals)))))
    pool = list(res.vals)
    for i in sel:   # nearest match (order may differ inside a conjugate pair)
        j = int(np.argmin([abs(vals[i] - y) for y in pool]))
        assert abs(pool.pop(j) - vals[i]) <= tol * abs(vals[i]), (i, vals[i])


def _first_factorisation(ctx, op, seed, k, mode):
    Q = ctx.basis(k + 1)
    prepare_seed(seed, Q[0])
    Hd = HessenbergDev(ctx, k)
    arnoldi_factorization(ctx, op, Q, Hd, 1, k, mode=mode)
    return Hd.download()


@pytest.mark.parametrize("mode", ["dcgs2", "cgs2", "mgs2"])
def test_golden_config1(gpu, mode):
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1136)
    z = _load("ks_config1.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=32)
    d, exact = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    H = _first_factorisation(ctx, op, seed, 16, mode)
    assert np.max(np.abs(H - z["H_first"])) <= 1e-12 * np.max(np.abs(z["H_first"]))
    res = krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=16, schur_tgt=5, mode=mode))
    _compare_ks(res, z)
    np.testing.assert_allclose(np.sort(res.vals[res.residual < 1e-6].real)[::-1], exact, atol=1e-9)


@pytest.mark.parametrize("mode", ["dcgs2"])
@pytest.mark.parametrize("k", [16, 64])
def test_golden_config2_reference_base_flow_seed(gpu, mode, k):
    """Real cylinder mesh (E=1996, N=175,648), seed = the reference's base flow BF_1cyl0.f00001,
    rotation-scaling operator with three dominant conjugate pairs; k=16 restarts twice."""
    lay = cylinder_layout(1996)
    z = _load(f"ks_config2_bf_k{k}.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=80)
    c, s, dr, exact = syn.rot2_operator(lay)
    op = Rot2Operator(ctx, c, s, dr)
    seed = ctx.vector().from_packed(syn.from_reference_order(lay, _load("bf_1cyl0_seed.npz")["seed_ref"]))
    H = _first_factorisation(ctx, op, seed, k, mode)
    assert np.max(np.abs(H - z["H_first"])) <= 1e-12 * np.max(np.abs(z["H_first"]))
    res = krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=k, schur_tgt=2, mode=mode))
    _compare_ks(res, z)
    for v in res.vals[res.residual < 1e-6]:
        assert np.min(np.abs(exact - v)) < 1e-8


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_golden_config3_graded_spectrum(gpu, mode):
    lay = box3d_layout(40)
    z = _load("ks_config3_arnoldi.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=48)
    d, exact = syn.laplacian_shift_invert(lay)
    op = DiagOperator(ctx, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    H = _first_factorisation(ctx, op, seed, 40, mode)
    assert np.max(np.abs(H - z["H"])) <= 1e-11 * np.max(np.abs(z["H"]))
    res = krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=40, schur_tgt=0, mode=mode))
    _compare_ks(res, dict(z, schur_cnt=0, mstart=np.array([], dtype=np.int64), cnt=np.array(res.cnt_history)))
    np.testing.assert_allclose(res.vals[:6].real, exact[:6], rtol=1e-10)


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_golden_restart_m128(gpu, mode):
    """BASELINE's m = 128 with a real restart (config 3's layout at E=128, N=289,792; the clustered
    time-stepper-like spectrum, schur_tgt=4): one condensation keeping 25 columns (the >16-column
    MFMA rotation), then 19 converged.  MKL's restart trajectory and selection reproduced on
    OpenBLAS, comparison-set Ritz values 1e-10, converged values equal the exact cluster 1e-10."""
    lay = box3d_layout(128)
    z = _load("ks_restart_m128.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=136)
    d, exact = syn.clustered_spectrum(lay)
    seed = ctx.vector()
    seed.fill_hash(11)
    res = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=128, schur_tgt=4, mode=mode))
    assert int(z["schur_cnt"]) == 1 and z["mstart"].tolist() == [26]
    _compare_ks(res, z)
    for v in res.vals[res.residual < 1e-6]:
        assert np.min(np.abs(exact - v)) <= 1e-10


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_golden_config3_k32(gpu, mode):
    """Config 3's operator family at E=128 (N=289,792), Krylov–Schur k_dim=32, schur_tgt=4: the MKL
    trajectory (10 converged in the first factorisation) and Ritz values 1e-10; top 4 = exact."""
    lay = box3d_layout(128)
    z = _load("ks_config3_k32.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=40)
    d, exact = syn.laplacian_shift_invert(lay)
    seed = ctx.vector()
    seed.fill_hash(11)
    res = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=32, schur_tgt=4, mode=mode))
    _compare_ks(res, z)
    np.testing.assert_allclose(res.vals[:4].real, exact[:4], rtol=1e-10)


def test_golden_config4_gmres(gpu):
    lay = cylinder_layout(1996)
    z = _load("gmres_config4.npz")
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=210)
    d, _ = syn.diag_spectrum(lay)
    op = ShiftedOperator(DiagOperator(ctx, d), -1.0)
    rhs = ctx.vector()
    rhs.fill_hash(3)
    sol = ctx.vector()
    info = ts_gmres(ctx, op, rhs, sol, GmresConfig(k_dim=200, maxiter=10, tol=1e-9))
    assert info.converged
    assert len(info.inner_residuals) == len(z["inner"]) and len(info.outer_residuals) == len(z["outer"])
    np.testing.assert_allclose(info.inner_residuals[:20], z["inner"][:20], rtol=1e-8)
    assert "Math Kernel Library" in str(z["lapack"])   # dgels on MKL (oracle) vs OpenBLAS (product)
    got = syn.to_reference_order(lay, sol.to_packed())
    np.testing.assert_allclose(got[:256], z["sol_head"], rtol=1e-9, atol=1e-12)


def test_golden_wavemaker_reference_base_flow(gpu, tmp_path):
    """The product's wave_maker file chain against the frozen oracle output: the four mode parts
    (the direct mode's real part is the reference's cylinder base flow BF_1cyl0, the rest hashed)
    written as dRe/dIm<session>0.f00001 and aRe/aIm<session>0.f00002, read back, bi-orthogonalised
    and combined on the device — to 1e-12 of the field's maximum."""
    from nekstab_next_amd import fld
    from nekstab_next_amd.sensitivity import velocity_layout, wave_maker

    z = _load("wavemaker_cyl.npz")
    vlay = velocity_layout(cylinder_layout(1996))
    w = syn.mass_weights(vlay)
    ctx = NekContext(vlay, weights=w, max_cols=4)
    nvel = vlay.ldim * vlay.n_v
    bf = _load("bf_1cyl0_seed.npz")["seed_ref"]
    parts = [np.concatenate([bf[:nvel], [0.0]])]
    for s_ in (41, 42, 43):
        parts.append(syn.to_reference_order(vlay, syn.hash_vector(vlay, s_)))
    parts[1] = 0.3 * parts[1]
    for (prefix, num), ref in zip((("dRe", 1), ("dIm", 1), ("aRe", 2), ("aIm", 2)), parts):
        f = fld.fld_from_vector(vlay, syn.from_reference_order(vlay, ref), time=float(num), istep=num)
        fld.write_fld(str(tmp_path / fld.fld_name(prefix, "cyl", 0, num)), f)
    res = wave_maker(ctx, str(tmp_path), session="cyl")
    wm = z["wavemaker"]
    assert np.max(np.abs(res["wavemaker"] - wm)) <= 1e-12 * np.max(np.abs(wm))
    d, di, a, ai = res["vectors"]
    re = ctx.dot(a, d, False) + ctx.dot(ai, di, False)
    assert abs(re - z["ad_after"][0]) < 1e-12
