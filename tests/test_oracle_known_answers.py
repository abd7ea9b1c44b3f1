"""Pin the CPU oracle to closed-form known answers (CPU only).

The reference ships no tests or golden vectors for this path and cannot be built here (DESIGN.md
§Oracle), so the oracle's restatement is checked against synthetic operators whose spectra /
solutions are exact, and against the one recorded run of the real reference (SURVEY.md §8(c),
"Verified runs" (2): k_dim=16, schur_tgt=5, diag(0.99..0.89, bulk): 2 Schur condensations with
9 eigenvalues selected each, 6 converged, residuals 3e-11..3e-9).
"""

import numpy as np
import pytest

import oracle as orc
from helpers import olayout, oracle_diag_matvec, oracle_rot2_matvec
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout, box3d_layout, cylinder_layout


def _setup(lay, seed=11):
    L = olayout(lay)
    w = syn.mass_weights(lay)
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, seed)))
    return L, w, q1


def test_config1_krylov_schur_matches_reference_probe():
    """Config 1 geometry (2-D lx1=6, E=1136, N=99,968), k_dim=16, schur_tgt=5."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1136)
    assert lay.N == 99968 and lay.N_w == 81792
    L, w, q1 = _setup(lay)
    d, exact = syn.diag_spectrum(lay)
    r = orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 16, 5)
    assert r["schur_cnt"] == 2 and r["mstart"] == [10, 10]  # 9 selected per condensation
    assert r["converged"] == 6
    conv = r["residual"] < 1e-6
    assert np.all(r["residual"][conv] < 1e-7)
    np.testing.assert_allclose(np.sort(r["vals"][conv].real)[::-1], exact, rtol=0, atol=1e-9)
    assert np.all(np.abs(r["vals"][conv].imag) == 0)


def test_config1_plain_arnoldi_m16():
    """schur_tgt <= 0: one 16-step Arnoldi; leading Ritz value approaches 0.99 (probe (1))."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1136)
    L, w, q1 = _setup(lay)
    d, exact = syn.diag_spectrum(lay)
    r = orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 16, 0)
    assert r["schur_cnt"] == 0
    assert abs(r["vals"][0].real - 0.99) < 5e-3
    # Arnoldi relation residual: H(k+1,k) > 0 and columns orthonormal
    Q = r["Q"]
    G = np.array([[orc.k_dot(L, w, Q[a], Q[b]) for b in range(17)] for a in range(17)])
    assert np.max(np.abs(G - np.eye(17))) < 1e-13


def test_config2_rot2_conjugate_pairs():
    """Rotation-scaling operator: exact eigenvalues r e^{±i theta} (conjugate-pair handling in eig
    and select_eigenvalues), k_dim=24, schur_tgt=2 as 1cyl.usr:15."""
    lay = cylinder_layout(400)
    L, w, q1 = _setup(lay, seed=5)
    c, s, dr, exact = syn.rot2_operator(lay)
    r = orc.krylov_schur(L, w, oracle_rot2_matvec(lay, c, s, dr), q1, 24, 2)
    conv = r["residual"] < 1e-6
    assert conv.sum() >= 2
    for v in r["vals"][conv]:
        assert np.min(np.abs(exact - v)) < 1e-8
    # the leading pair 0.99 e^{±0.35 i} is found as a conjugate pair with conjugate eigenvectors
    lead = r["vals"][:2]
    assert abs(lead[0] - np.conj(lead[1])) < 1e-12 and abs(abs(lead[0]) - 0.99) < 1e-9


def test_config3_shift_invert_laplacian_reduced():
    lay = box3d_layout(40)
    L, w, q1 = _setup(lay)
    d, exact = syn.laplacian_shift_invert(lay)
    r = orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 40, 0)
    top = r["vals"][:6]
    np.testing.assert_allclose(top.real, exact[:6], rtol=1e-11)
    # exact mu values are the diagonal itself
    dd = syn.to_reference_order(lay, d)[: L.n - L.np]
    assert np.all(np.isin(exact[:6], dd))


def test_config4_gmres_exact_solution():
    """J = D - I (newton_linearized_map returns Phi'(q) - q); ts_gmres solves J x = rhs; exact
    x = rhs ./ (d - 1) on every stored row (pressure included)."""
    lay = cylinder_layout(60)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    d, _ = syn.diag_spectrum(lay)
    dref = syn.to_reference_order(lay, d)
    J = dref - 1.0
    rhs = syn.to_reference_order(lay, syn.hash_vector(lay, 3))

    def mv(x, y):
        y[:] = J * x
        y[-1] = 0.0

    sol, hist = orc.ts_gmres(L, w, mv, rhs, maxiter=20, ksize=40, tol=1e-20)
    exact = rhs[:-1] / J[:-1]
    # weighted fields converge in the W-norm; pressure (unweighted, invisible to the dot) follows
    nw = L.nwf * L.nv
    assert np.max(np.abs(sol[:nw] - exact[:nw])) < 1e-8
    assert hist["outer"][-1] < 1e-16


def test_config5_biorthogonalize_property():
    """After biorthogonalize, <adjoint, direct>_W = 1 + 0i and the direct mode has unit norm."""
    lay = box3d_layout(6)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    vs = [syn.to_reference_order(lay, syn.hash_vector(lay, s)) for s in (1, 2, 3, 4)]
    dRe, dIm, aRe, aIm = orc.biorthogonalize(L, w, *vs)
    ip = lambda p, q: orc.k_dot(L, w, p, q)  # noqa: E731
    re = ip(aRe, dRe) + ip(aIm, dIm)
    im = ip(aRe, dIm) - ip(aIm, dRe)
    assert abs(re - 1.0) < 1e-12 and abs(im) < 1e-12


@pytest.mark.parametrize("ldim", [2, 3])
def test_wave_maker_closed_form(ldim):
    """wave_maker (sensitivity.f90:3-77) in closed form: bi-orthogonalisation scales the direct mode
    d by 1/||d||_W and the adjoint mode a by 1/conj(<a, d/||d||>_W), so the pointwise product is
    wm = |d| |a| / |<a, d>_W| (|.| the pointwise complex velocity modulus, <a, d> = (aRe.dRe +
    aIm.dIm) + i (aRe.dIm - aIm.dRe)).  Hence wm does not change when either mode is multiplied
    by a complex constant."""
    lay = NekLayout(ldim=ldim, lx1=6, lx2=4, nelgv=9, n_scalars=0, ifpo=False)
    L = orc.OLayout(lay.n_v, 0, ldim, False, ldim)
    w = syn.mass_weights(lay)
    vs = [syn.to_reference_order(lay, syn.hash_vector(lay, s)) for s in (5, 6, 7, 8)]
    wm, _ = orc.wave_maker(L, w, *vs)
    nv = lay.n_v
    ww = np.tile(w[:nv] if w.size >= nv else w, ldim)[: ldim * nv]
    ip = lambda p, q: float(np.sum(p[: ldim * nv] * ww * q[: ldim * nv]))  # noqa: E731
    dRe, dIm, aRe, aIm = vs
    ad = complex(ip(aRe, dRe) + ip(aIm, dIm), ip(aRe, dIm) - ip(aIm, dRe))
    mod = lambda re, im: np.sqrt(sum(re[c * nv:(c + 1) * nv] ** 2 + im[c * nv:(c + 1) * nv] ** 2  # noqa: E731
                                     for c in range(ldim)))
    closed = mod(dRe, dIm) * mod(aRe, aIm) / abs(ad)
    np.testing.assert_allclose(wm, closed, rtol=1e-12)
    # a complex multiple of either mode leaves the wave-maker unchanged
    c1, c2 = 2.5 - 0.7j, -0.3 + 1.9j
    d2 = (c1.real * dRe - c1.imag * dIm, c1.real * dIm + c1.imag * dRe)
    a2 = (c2.real * aRe - c2.imag * aIm, c2.real * aIm + c2.imag * aRe)
    wm2, _ = orc.wave_maker(L, w, *d2, *a2)
    np.testing.assert_allclose(wm2, wm, rtol=1e-12)


def test_glsc3_is_sequential_sum():
    rng = np.random.default_rng(0)
    a, b, m = (rng.standard_normal(1000) for _ in range(3))
    ref = 0.0
    for i in range(1000):
        ref = ref + a[i] * b[i] * m[i]
    assert orc.lib().orc_glsc3(a, b, m, 1000) == ref


def test_k_dot_time_component():
    L = orc.OLayout(100, 20, 2, time_in_dot=True)
    w = np.ones(100)
    p, q = L.zeros(), L.zeros()
    p[-1], q[-1] = 2.0, 3.0
    assert orc.k_dot(L, w, p, q) == 6.0
    L2 = orc.OLayout(100, 20, 2, time_in_dot=False)
    assert orc.k_dot(L2, w, p, q) == 0.0
    assert orc.real_dot(L2, w, p, q) == 6.0  # real_dot always includes time (nek_vectors.f90:106)


def test_legacy_matvec_closed_forms():
    """oracle.legacy_matvec (matvec.f90:56-146) on a diagonal map D (self-adjoint) in closed form:
    3.x -> D q, 3.3 -> D^2 q, 4.x -> q - D q (time: q%time - 0), 2.0 -> D q - q with time 0, 2.1 ->
    D q - q + b_fc q%time with time = <b_ic, q>_W (the time of b_ic ignored, compute_bvec :610)."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=40)
    L = olayout(lay, time_in_dot=True)
    w = syn.mass_weights(lay)
    d = syn.to_reference_order(lay, syn.diag_spectrum(lay)[0])
    mv = oracle_diag_matvec(L, d)
    rng = np.random.default_rng(0)
    q = rng.standard_normal(L.len)
    bfc, bic = rng.standard_normal(L.len), rng.standard_normal(L.len)
    n = L.n
    for mode, evop, fields, time in (
            (3.1, "d", d[:n] * q[:n], 0.0),
            (3.2, "a", d[:n] * q[:n], 0.0),
            (3.3, "p", d[:n] * d[:n] * q[:n], 0.0),
            (4.1, None, q[:n] - d[:n] * q[:n], q[-1]),
            (2.0, "n", d[:n] * q[:n] - q[:n], 0.0),
            (2.1, "n", d[:n] * q[:n] - q[:n] + bfc[:n] * q[-1], None)):
        f = np.full(L.len, 7.0)
        assert orc.legacy_matvec(L, w, mode, mv, mv, f, q.copy(), b_fc=bfc, b_ic=bic) == evop
        np.testing.assert_allclose(f[:n], fields, rtol=0, atol=1e-15)
        if time is None:
            wf = np.concatenate([np.tile(w, L.nwf), np.zeros(L.np)])
            time = float(np.sum(wf * bic[:n] * q[:n]))
        assert abs(f[-1] - time) <= 1e-12 * max(1.0, abs(time))
    with pytest.raises(ValueError):
        orc.legacy_matvec(L, w, 3.4, mv, mv, np.zeros(L.len), q)


def test_steady_force_sensitivity_closed_form():
    """oracle.ts_steady_force_sensitivity (sensitivity.f90:273-346) with a diagonal adjoint map D and
    no recast: GMRES on q - D q, so the solution is the forcing / (1 - d) on the velocity (other
    fields 0), to 1e-10 after its 10 restarts."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=40)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    d = 0.5 * syn.to_reference_order(lay, syn.diag_spectrum(lay)[0])
    rhs = syn.to_reference_order(lay, syn.hash_vector(lay, 5))
    nvel = lay.ldim * lay.n_v
    rhs[nvel:] = 0.0
    sol, hist, alpha = orc.ts_steady_force_sensitivity(L, w, oracle_diag_matvec(L, d), rhs, 20, 1e-24)
    exact = np.zeros_like(rhs)
    exact[:nvel] = rhs[:nvel] / (1.0 - d[:nvel])
    assert np.max(np.abs(sol[:-1] - exact[:-1])) <= 1e-10 * np.max(np.abs(exact))
    assert hist["outer"][-1] < 1e-20


def test_newton_krylov_closed_form():
    """oracle.newton_krylov (newton_krylov.f90:1-166) on the pointwise quadratic fixed point
    q = d q + c + eps q^2: from q = 0 Newton reaches, at every point, the root of
    eps q^2 + (d - 1) q + c = 0 nearest 0, quadratically, to 1e-12 in the W-norm (GMRES minimises
    the k_dot norm, which leaves pressure out)."""
    import ctypes

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=30)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    eps = 0.3
    d = 0.5 * syn.to_reference_order(lay, syn.diag_spectrum(lay)[0])
    c = 0.05 * syn.to_reference_order(lay, syn.hash_vector(lay, 8))
    live = np.ones(L.len)
    live[-1] = 0.0

    def onl(x, y):
        y[:] = (d * x + c + eps * x * x - x) * live

    def olin(x0):
        g = (d + 2.0 * eps * x0) * live
        return lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), g, x, y, 0.0)

    q, r, _ = orc.newton_krylov(L, w, onl, olin, L.zeros(), 1e-24, 10, 20)
    b = d - 1.0
    root = 2.0 * c / (-b + np.sqrt(b * b - 4.0 * eps * c))   # the root through q = 0 as c -> 0 (stable form)
    # GMRES minimises in the W-norm of k_dot (weighted fields only): gate the weighted velocity error
    nvel = lay.ldim * lay.n_v
    err = q[:nvel] - root[:nvel]
    assert np.sqrt(np.sum(np.tile(w, lay.ldim) * err * err)) <= 1e-12
    assert r[-1] < 1e-24 and r[2] < 1e-5 * r[1]
