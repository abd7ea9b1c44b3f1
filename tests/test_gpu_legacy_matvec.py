"""The legacy ``matvec(f, q)`` dispatcher (core/matvec.f90:56-146) against the oracle's restatement
(oracle.legacy_matvec) on the same operators and inputs: every ``uparam(1)`` family, the time slot
included (k_sub2 / k_cmult carry it; the UPO period row of mode 2.1 writes it).  Gate: max |diff|
<= 1e-13 * max |ref| per vector (floating point; the GPU's axpy may contract to FMA).

Then Newton for a periodic orbit end to end: ts_gmres on the mode-2.1 bordered map with the time
slot inside k_dot (uparam(1)==2.1, krylov_subspace.f90:52-54), residual histories against the
oracle's ts_gmres on the oracle's map (1e-8 relative), solution and period correction to 1e-10
relative (W-norm with time)."""
import ctypes

import numpy as np
import pytest

import oracle as orc
from helpers import olayout, oracle_rot2_matvec
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.config import GmresConfig
from nekstab_next_amd.gmres import ts_gmres
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.operators import DiagOperator, LegacyMatvec, Rot2Operator
from nekstab_next_amd.vector import NekContext

LAYOUTS = {
    "2d": NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300),
    "3d_scalar": NekLayout(ldim=3, lx1=5, lx2=3, nelgv=37, n_scalars=1),
}
MODES = [3.1, 3.11, 3.2, 3.3, 4.1, 2.0, 2.01, 2.1]   # 3.11 / 2.01: with the finite-difference map


def _vec(ctx, lay, seed, time, scale=1.0):
    p = syn.hash_vector(lay, seed) * scale
    p[lay.time_offset] = time
    return ctx.vector().from_packed(p), syn.to_reference_order(lay, p)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(LAYOUTS))
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("time_in_dot", [False, True])
def test_dispatch_vs_oracle(gpu, name, mode, time_in_dot):
    lay = LAYOUTS[name]
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=8, time_in_dot=time_in_dot)
    L = olayout(lay, time_in_dot=time_in_dot)
    c, s, dr, _ = syn.rot2_operator(lay)
    op = Rot2Operator(ctx, c, s, dr)
    fwd, adj = oracle_rot2_matvec(lay, c, s, dr), oracle_rot2_matvec(lay, c, s, dr, transpose=True)
    # 3.11 / 2.01: the finite-difference forward map (iffindiff) — a distinct operator so the dispatch shows
    d, _ = syn.diag_spectrum(lay)
    use_fd = mode in (3.11, 2.01)
    fd_op = DiagOperator(ctx, d, time_scale=0.5) if use_fd else None
    dref = syn.to_reference_order(lay, d)
    fd = (lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.5)) if use_fd else None
    bfc, bfc_r = _vec(ctx, lay, 21, 0.9, 0.3)   # nonzero time: must be ignored (compute_bvec :610)
    bic, bic_r = _vec(ctx, lay, 22, -0.4, 0.2)
    A = LegacyMatvec(mode, op, fd_op=fd_op, b_fc=bfc, b_ic=bic)
    q, q_r = _vec(ctx, lay, 7, 0.37)
    f = ctx.vector()
    f.fill_hash(99)                              # stale contents must not leak through
    A.matvec(q, f)
    f_r = L.zeros()
    evop = orc.legacy_matvec(L, w, mode, fwd, adj, f_r, q_r.copy(), fd=fd, b_fc=bfc_r, b_ic=bic_r)
    assert A.evop == evop
    got = syn.to_reference_order(lay, f.to_packed())
    assert np.max(np.abs(got - f_r)) <= 1e-13 * np.max(np.abs(f_r)), (mode, np.max(np.abs(got - f_r)))
    if mode == 2.1:
        assert abs(got[-1]) > 1e-3        # the period row is live
    elif int(mode) == 2:
        assert got[-1] == 0.0
    # q is read-only for every map
    np.testing.assert_array_equal(syn.to_reference_order(lay, q.to_packed()), q_r)


def test_modes_that_select_nothing_are_refused():
    """matvec.f90:110-143 dispatches 2.x, [3.0, 3.4) and 4.x; anything else leaves f untouched there
    and is refused here — before any device work."""
    for mode in (1.0, 3.4, 3.5, 5.0, 0.0):
        with pytest.raises(ValueError):
            LegacyMatvec(mode, op=None)
    with pytest.raises(ValueError):
        LegacyMatvec(2.1, op=None)           # the period row needs b_fc and b_ic


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["dcgs2", "mgs2"])
def test_upo_newton_gmres_vs_oracle(gpu, mode):
    """One Newton correction for a periodic orbit (uparam(1)=2.1): ts_gmres on the bordered map
    [Phi' - I, b_fc; <b_ic, .>_W, 0] with time inside k_dot, k_dim=8 so the outer loop restarts."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=16, time_in_dot=True)
    L = olayout(lay, time_in_dot=True)
    d, _ = syn.diag_spectrum(lay)
    dref = syn.to_reference_order(lay, d)
    bfc, bfc_r = _vec(ctx, lay, 31, 0.0, 0.5)
    bic, bic_r = _vec(ctx, lay, 32, 0.0, 0.5)
    A = LegacyMatvec(2.1, DiagOperator(ctx, d), b_fc=bfc, b_ic=bic)
    rhs, rhs_r = _vec(ctx, lay, 3, 0.25)
    sol = ctx.vector()
    info = ts_gmres(ctx, A, rhs, sol, GmresConfig(k_dim=8, maxiter=12, tol=1e-12, mode=mode))

    fwd = lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.0)  # noqa: E731
    mv = lambda x, y: orc.legacy_matvec(L, w, 2.1, fwd, None, y, x, b_fc=bfc_r, b_ic=bic_r)  # noqa: E731
    sref, hist = orc.ts_gmres(L, w, mv, rhs_r, maxiter=12, ksize=8, tol=1e-12)
    assert len(info.outer_residuals) == len(hist["outer"]) >= 2
    assert len(info.inner_residuals) == len(hist["inner"])
    np.testing.assert_allclose(info.inner_residuals, hist["inner"], rtol=1e-8)
    np.testing.assert_allclose(info.outer_residuals, hist["outer"], rtol=1e-8)
    got = syn.to_reference_order(lay, sol.to_packed())
    diff = got - sref
    scale = max(1.0, np.sqrt(orc.k_dot(L, w, sref, sref)))   # D - I is nearly singular: ||sol|| >> 1
    assert np.sqrt(orc.k_dot(L, w, diff, diff)) < 1e-10 * scale
    assert abs(sref[-1]) > 1e-6                 # the period correction is part of the solution


@pytest.mark.gpu
def test_transient_growth_map_krylov_schur_vs_oracle_and_svds(gpu):
    """uparam(1) = 3.3: the in-tree Krylov–Schur on transient_growth_map (adjoint∘forward,
    matvec.f90:478-495; evop 'p') against the oracle's Krylov–Schur on its restatement of the same
    map (trajectory and Ritz values 1e-10), and against the LightKrylov-style svds of the forward map
    (transient_growth_analysis, linear_stab.f90:82-119): the leading eigenvalues are sigma^2 (1e-10)."""
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur, prepare_seed
    from nekstab_next_amd.lightkrylov import svds
    from nekstab_next_amd.operators import RankTwoPerturbed
    from helpers import match_ritz, oracle_rank2_matvec, ritz_compare_set

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=200)
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=40)
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    hv = [0.05 * syn.hash_vector(lay, s5) for s5 in (21, 22, 23, 24)]
    vs = [ctx.vector().from_packed(v) for v in hv]
    A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=2.0)
    P = LegacyMatvec(3.3, A)
    assert P.evop == "p"
    seed = ctx.vector()
    seed.fill_hash(11)
    cfg = KrylovSchurConfig(k_dim=24, schur_tgt=3)
    res = krylov_schur(ctx, P, seed, cfg)
    fwd = oracle_rank2_matvec(lay, d, *hv, 2.0, w)
    adj = oracle_rank2_matvec(lay, d, *hv, 2.0, w, transpose=True)
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
    ref = orc.krylov_schur(L, w, lambda x, y: orc.legacy_matvec(L, w, 3.3, fwd, adj, y, x), q1, 24, 3)
    assert res.schur_cnt == ref["schur_cnt"] and res.mstart_history == ref["mstart"]
    sel = ritz_compare_set(ref["vals"], ref["residual"], cfg.eigen_tol)
    got = match_ritz(ref["vals"][sel], res.vals)
    assert np.max(np.abs(got - ref["vals"][sel]) / np.abs(ref["vals"][sel])) <= 1e-10
    # the same gains from the bidiagonalisation of A
    U, V = ctx.basis(25), ctx.basis(25)
    prepare_seed(seed, V[0])
    sv = svds(ctx, A, U, V, nev=3, tolerance=1e-10)
    conv = np.sort(res.vals[res.residual < 1e-8].real)[::-1][:3]
    np.testing.assert_allclose(conv, np.sort(sv.sigma ** 2)[::-1][:3], rtol=1e-10)
