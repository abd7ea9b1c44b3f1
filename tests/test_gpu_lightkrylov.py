"""LightKrylov-compatible surface (eigs / svds / gmres / get_vec / axpby_linop) on the device.
LightKrylov itself is not in the container (parity unpinned); these tests pin the restated
algorithms to exact answers: dense W-weighted SVD / eigen-decomposition of small operators and the
exact solution of a diagonal system."""
import numpy as np
import pytest

from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.krylov_schur import prepare_seed
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.lightkrylov import AxpbyLinop, IdentityLinop, eigs, get_vec, gmres, svds
from nekstab_next_amd.operators import DiagOperator, RankTwoPerturbed
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu

LAY = NekLayout(ldim=2, lx1=4, lx2=2, nelgv=40, ifpo=False)  # no pressure: W is invertible


def _setup():
    w = syn.mass_weights(LAY)
    ctx = NekContext(LAY, weights=w, max_cols=64)
    d, _ = syn.diag_spectrum(LAY)
    vh = [syn.hash_vector(LAY, s) * 0.05 for s in (31, 32, 33, 34)]
    vs = [ctx.vector().from_packed(v) for v in vh]
    A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=3.0)
    return ctx, w, d, vh, A


def _dense(ctx, A, w):
    """Dense matrix of A on the live weighted dofs, by applying it to unit vectors."""
    n = LAY.N_w
    idx = [f * LAY.sv + i for f in range(LAY.n_wf) for i in range(LAY.n_v)]
    M = np.zeros((n, n))
    x, y = ctx.vector(), ctx.vector()
    for c, r in enumerate(idx):
        e = np.zeros(LAY.ld)
        e[r] = 1.0
        x.from_packed(e)
        A.matvec(x, y)
        M[:, c] = y.to_packed()[idx]
    W = np.tile(w, LAY.n_wf)
    return M, W, idx


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_svds_matches_dense_weighted_svd(gpu, mode):
    ctx, w, d, vh, A = _setup()
    M, W, idx = _dense(ctx, A, w)
    s_exact = np.linalg.svd(np.sqrt(W)[:, None] * M / np.sqrt(W)[None, :], compute_uv=False)
    k = 40
    U, V = ctx.basis(k + 1), ctx.basis(k + 1)
    seed = ctx.vector()
    seed.fill_hash(7)
    prepare_seed(seed, V[0])
    r = svds(ctx, A, U, V, nev=3, tolerance=1e-8, mode=mode)
    conv = r.residuals < 1e-8
    assert conv.sum() >= 3 and not r.breakdown
    np.testing.assert_allclose(r.sigma[:3], s_exact[:3], rtol=1e-10)
    # singular triplet: A v = sigma u
    u, v, Av = ctx.vector(), ctx.vector(), ctx.vector()
    get_vec(u, U, r.uvecs[:, 0], k)
    get_vec(v, V, r.vvecs[:, 0], k)
    A.matvec(v, Av)
    Av.axpby(1.0, u, -r.sigma[0])
    assert np.sqrt(ctx.dot(Av, Av, False)) < 1e-9 * r.sigma[0]


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_svds_rank_deficient_breakdown(gpu, mode):
    """A rank-3 operator (three nonzero diagonal entries, W-self-adjoint, so the singular values are
    |d_i|) with k=12: the bidiagonalisation is invariant after 4 steps.  svds detects it (the
    new-direction norms alpha_j / beta_j fall below 1e-8 of their columns), redoes it in MGS2 order
    and returns the three exact singular values to 1e-10; the rest are rounding-level."""
    w = syn.mass_weights(LAY)
    ctx = NekContext(LAY, weights=w, max_cols=64)
    d = np.zeros(LAY.ld)
    exact = np.array([0.9, 0.6, 0.3])
    for i, v in enumerate(exact):
        d[7 * (i + 1)] = v
    A = DiagOperator(ctx, d)
    k = 12
    U, V = ctx.basis(k + 1), ctx.basis(k + 1)
    seed = ctx.vector()
    seed.fill_hash(7)
    prepare_seed(seed, V[0])
    r = svds(ctx, A, U, V, nev=3, tolerance=1e-8, mode=mode)
    assert r.breakdown
    np.testing.assert_allclose(r.sigma[:3], exact, rtol=1e-10)
    assert np.all(r.sigma[3:] < 1e-12)
    u, v, Av = ctx.vector(), ctx.vector(), ctx.vector()
    get_vec(u, U, r.uvecs[:, 0], k)
    get_vec(v, V, r.vvecs[:, 0], k)
    A.matvec(v, Av)
    Av.axpby(1.0, u, -r.sigma[0])
    assert np.sqrt(ctx.dot(Av, Av, False)) < 1e-9 * r.sigma[0]


@pytest.mark.parametrize("k", [1, 2, 17, 40])
def test_svds_dcgs2_equals_cgs2(gpu, k):
    """The delayed re-orthogonalisation (two reads of each basis per step) against the CGS2 path
    (three reads) on the same operator and seed: the bidiagonal projections C, D agree to
    1e-12 of their size, both bases are W-orthonormal to 1e-12, the relations A V_k = U_k C and
    A^T U_k = V_{k+1} D hold to 1e-12, and sigma / singular vectors agree to 1e-10."""
    ctx, w, d, vh, A = _setup()
    out = {}
    for mode in ("cgs2", "dcgs2"):
        U, V = ctx.basis(k + 1), ctx.basis(k + 1)
        seed = ctx.vector()
        seed.fill_hash(7)
        prepare_seed(seed, V[0])
        r = svds(ctx, A, U, V, nev=1, tolerance=1e-8, mode=mode)
        out[mode] = (r, U, V)
    (rc, Uc, Vc), (rd, Ud, Vd) = out["cgs2"], out["dcgs2"]
    np.testing.assert_allclose(rd.C, rc.C, rtol=0, atol=1e-12 * np.abs(rc.C).max())
    np.testing.assert_allclose(rd.sigma, rc.sigma, rtol=1e-10, atol=1e-13 * rc.sigma[0])
    for B, n in ((Ud, k), (Vd, k + 1)):
        G = np.array([[ctx.dot(B[a], B[b], False) for b in range(n)] for a in range(n)])
        assert np.abs(G - np.eye(n)).max() < 1e-12
    x, y = ctx.vector(), ctx.vector()
    for c in range(k):       # A v_c = sum_i C[i, c] u_i ;  A^T u_c = sum_i D[i, c] v_i
        A.matvec(Vd[c], x)
        get_vec(y, Ud, rd.C[:, c], k)
        x.axpby(1.0, y, -1.0)
        assert np.sqrt(ctx.dot(x, x, False)) < 1e-12 * max(1.0, np.abs(rd.C).max())
    # leading singular vectors agree up to sign
    u1, u2, v1, v2 = (ctx.vector() for _ in range(4))
    get_vec(u1, Uc, rc.uvecs[:, 0], k)
    get_vec(u2, Ud, rd.uvecs[:, 0], k)
    get_vec(v1, Vc, rc.vvecs[:, 0], k)
    get_vec(v2, Vd, rd.vvecs[:, 0], k)
    sgn = np.sign(ctx.dot(u1, u2, False))
    u1.axpby(1.0, u2, -sgn)
    v1.axpby(1.0, v2, -sgn)
    assert np.sqrt(ctx.dot(u1, u1, False)) < 1e-10 and np.sqrt(ctx.dot(v1, v1, False)) < 1e-10


def test_eigs_and_get_vec(gpu):
    ctx, w, d, vh, A = _setup()
    M, W, idx = _dense(ctx, A, w)
    lam = np.linalg.eigvals(M)
    lam = lam[np.argsort(-np.abs(lam))]
    k = 30
    X = ctx.basis(k + 1)
    seed = ctx.vector()
    seed.fill_hash(5)
    prepare_seed(seed, X[0])
    vecs, vals, res, info = eigs(ctx, A, X, nev=3, tolerance=1e-8)
    assert info == 0
    np.testing.assert_allclose(vals[:3], lam[:3], rtol=1e-10)
    xr, xi, y = ctx.vector(), ctx.vector(), ctx.vector()
    get_vec(xr, X, vecs[:, 0].real, k)
    A.matvec(xr, y)
    y.axpby(1.0, xr, -vals[0].real)  # real leading eigenvalue
    assert abs(vals[0].imag) == 0.0
    assert np.sqrt(ctx.dot(y, y, False)) < 1e-8 * np.sqrt(ctx.dot(xr, xr, False))
    # adjoint: same spectrum
    X2 = ctx.basis(k + 1)
    prepare_seed(seed, X2[0])
    _, vals_t, _, _ = eigs(ctx, A, X2, nev=3, tolerance=1e-8, transpose=True)
    np.testing.assert_allclose(vals_t[:3], lam[:3], rtol=1e-10)


def test_gmres_resolvent_composite(gpu):
    """S = Id - A (axpby_linop(Id, A, 1, -1)) solved with LightKrylov-style gmres; exact solution of
    the diagonal case is x = b / (1 - d)."""
    w = syn.mass_weights(LAY)
    ctx = NekContext(LAY, weights=w, max_cols=64)
    d, _ = syn.diag_spectrum(LAY)
    S = AxpbyLinop(IdentityLinop(), DiagOperator(ctx, d), 1.0, -1.0, False, True)
    b = ctx.vector()
    b.fill_hash(3)
    x = ctx.vector()
    info, hist = gmres(ctx, S, b, x, atol=1e-12, rtol=1e-12, kdim=30, maxiter=20)
    assert info == 0 and hist[-1] < 1e-11 * hist[0]
    bx = b.to_packed()
    got = x.to_packed()
    live = [f * LAY.sv + i for f in range(LAY.n_wf) for i in range(LAY.n_v)]
    np.testing.assert_allclose(got[live], bx[live] / (1.0 - d[live]), rtol=1e-9, atol=1e-12)


def test_drivers_linear_stability_and_transient_growth(gpu, tmp_path):
    from nekstab_next_amd import fld
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.drivers import linear_stability_analysis, transient_growth_analysis

    ctx, w, d, vh, A = _setup()
    M, W, idx = _dense(ctx, A, w)
    lam = np.linalg.eigvals(M)
    lam = lam[np.argsort(-np.abs(lam))]
    seed = ctx.vector()
    seed.fill_hash(5)
    t = 2.5
    out = linear_stability_analysis(ctx, A, seed, t, KrylovSchurConfig(k_dim=30, schur_tgt=3, maxmodes=2),
                                    outdir=str(tmp_path), session="box")
    np.testing.assert_allclose(out["eigvals"][:3], lam[:3], rtol=1e-10)
    np.testing.assert_allclose(out["eigvals_ns"][:3], np.log(lam[:3].astype(complex)) / t, rtol=1e-10)
    spec = np.loadtxt(tmp_path / "Spectrum_NSd.dat")
    np.testing.assert_allclose(spec[0, 0], np.log(abs(lam[0])) / t, rtol=1e-6)
    f = fld.read_fld(str(tmp_path / "dRebox0.f00001"))
    assert f.rdcode == "U" and f.nelgt == LAY.nelgv
    g = transient_growth_analysis(ctx, A, seed, k_dim=40, nev=2, tolerance=1e-8, outdir=str(tmp_path),
                                  session="box")
    s_exact = np.linalg.svd(np.sqrt(W)[:, None] * M / np.sqrt(W)[None, :], compute_uv=False)
    np.testing.assert_allclose(g["gain"][:2], s_exact[:2] ** 2, rtol=1e-10)
    assert (tmp_path / "pUbox0.f00001").exists() and (tmp_path / "Spectrum_Sp.dat").exists()


def test_op_cdiag_vs_numpy(gpu):
    from nekstab_next_amd.layout import pair_layout
    from nekstab_next_amd.operators import ComplexDiagOperator

    p = pair_layout(NekLayout(ldim=3, lx1=5, lx2=3, nelgv=7, n_scalars=1))
    b = p.base
    ctx = NekContext(p, weights=np.tile(syn.mass_weights(b), 2), max_cols=8)
    cr, ci, _ = syn.resolvent_diag(p, omega=0.7)
    op = ComplexDiagOperator(ctx, cr, ci)
    rng = np.random.default_rng(1)
    xr, xi = rng.standard_normal(b.ld), rng.standard_normal(b.ld)
    x = ctx.vector().from_packed(p.pack(xr, xi))
    y = ctx.vector()
    c_re, _ = p.unpack(cr)
    c_im, _ = p.unpack(ci)
    for conj in (False, True):
        (op.rmatvec if conj else op.matvec)(x, y)
        yr, yi = p.unpack(y.to_packed())
        c = c_re + 1j * (-c_im if conj else c_im)
        z = c * (xr + 1j * xi)
        for _, s, n in b.field_slices():
            np.testing.assert_allclose(yr[s: s + n], z.real[s: s + n], rtol=1e-15, atol=1e-16)
            np.testing.assert_allclose(yi[s: s + n], z.imag[s: s + n], rtol=1e-15, atol=1e-16)
        assert y.time == 0.0


def test_resolvent_analysis_singular_values(gpu, tmp_path):
    """resolvent_analysis (linear_stab.f90:120-163) on complex pair vectors: the leading gains
    sigma^2 of R = (i omega - L)^-1 for a W-normal stable L are 1/(omega^2 + gamma^2)."""
    from nekstab_next_amd.drivers import resolvent_analysis
    from nekstab_next_amd.layout import pair_layout
    from nekstab_next_amd.operators import ComplexDiagOperator

    p = pair_layout(NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300))
    ctx = NekContext(p, weights=np.tile(syn.mass_weights(p.base), 2), max_cols=48)
    cr, ci, sv = syn.resolvent_diag(p, omega=0.3)
    seed = ctx.vector()
    seed.fill_hash(17)
    out = resolvent_analysis(ctx, ComplexDiagOperator(ctx, cr, ci), seed, k_dim=40, nev=6, tolerance=1e-8,
                             outdir=str(tmp_path))
    # the cmplx dot is real (re.re + im.im), so x and i x are independent directions: every complex
    # singular value appears twice (as in nekStab's LightKrylov svds on cmplx_nek_vector)
    exact = np.repeat(sv[:3] ** 2, 2)
    np.testing.assert_allclose(out["sigma2"][:6], exact, rtol=1e-10)
    assert out["info"] == 0
    data = np.loadtxt(tmp_path / "Spectrum_Sr.dat")
    assert data.shape == (40, 2)
    np.testing.assert_allclose(data[:6, 0], exact, rtol=1e-6)
