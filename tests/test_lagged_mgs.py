"""The host algebra of ``"mgs2-lagged"`` (arnoldi.lagged_coefficients = the library's host-only
nkv_lagged_coef, callable without a GPU) on CPU: the device kernels it
drives (the two-vector multi-dot, the DCGS2 dual update, the closing block update) are emulated
in numpy with the same coefficient layout, and the factorisation is compared with the reference's
column-by-column MGS2 (krylov_decomposition.f90:155-186) in the W inner product — from the
default noise seed's unnormalised Q(1) (eigensolvers.f90:195-203), and after a Krylov–Schur
restart that rotates that non-orthonormal basis (eigensolvers.f90:421-442)."""
import numpy as np
import scipy.linalg as sla

from nekstab_next_amd.arnoldi import lagged_coefficients


def _problem(n=1500, seed=3):
    rng = np.random.default_rng(seed)
    w = rng.uniform(0.5, 1.5, n)
    lam = np.concatenate([np.linspace(1.0, 0.9, 6), rng.uniform(0.0, 0.8, n - 6)])
    u, v = rng.standard_normal(n) * 1e-2, rng.standard_normal(n) * 1e-2
    A = np.diag(lam) + np.outer(u, v)   # non-normal
    x = rng.standard_normal(n)
    x /= np.sqrt(np.sum(w * x * x))
    return A, w, A @ x                  # Q(1) = A (noise / ||noise||), NOT renormalised


def _mgs2(A, w, Q, H, c0, c1):
    for c in range(c0, c1):
        f = A @ Q[:, c]
        h = np.zeros(c + 1)
        for _ in range(2):
            for i in range(c + 1):
                a = np.sum(w * f * Q[:, i])
                f = f - a * Q[:, i]
                h[i] += a
        H[: c + 1, c] = h
        H[c + 1, c] = np.sqrt(np.sum(w * f * f))
        Q[:, c + 1] = f / H[c + 1, c]


def _lagged(A, w, Q, H, c0, c1):
    """arnoldi._lagged_factorization with numpy in place of the kernels (same coefficient layout)."""
    k1 = Q.shape[1]
    G = np.zeros((k1, k1))
    for i in range(c0):   # rows of the columns before the first matvec column, rebuilt
        G[i, : i + 1] = G[: i + 1, i] = Q[:, : i + 1].T @ (w * Q[:, i])
    for c in range(c0, c1):
        f = A @ Q[:, c]
        j = c + 1
        hv = np.concatenate([Q[:, :j].T @ (w * Q[:, c]), Q[:, :j].T @ (w * f)])
        coef = lagged_coefficients(G, H, hv, c, 1 if c == c0 else 0)
        x, rinv, yc, sc, a = coef[:c], coef[2 * c + 1], coef[2 * c + 2], coef[2 * c + 4], coef[2 * c + 5:3 * c + 5]
        qbar = (Q[:, c] * sc - Q[:, :c] @ a) * rinv
        Q[:, c] = qbar
        Q[:, c + 1] = f * (sc * rinv) - Q[:, :c] @ x - qbar * yc
    m = c1
    p = Q[:, : m + 1].T @ (w * Q[:, m])
    beta = lagged_coefficients(G, H, p, m, 2)[:m]   # H(0:m, m-1) += beta
    u = Q[:, m] - Q[:, :m] @ beta
    H[m, m - 1] = np.sqrt(np.sum(w * u * u))
    Q[:, m] = u / H[m, m - 1]


def _restart(Q, H, k, ms):
    """schur_condensation's effect on (Q, H): Schur form of H_k with the ms largest |lambda| first."""
    ev = np.sort(np.abs(np.linalg.eigvals(H[:k, :k])))[::-1]
    thr = 0.5 * (ev[ms - 1] + ev[ms])
    T, Z, sdim = sla.schur(H[:k, :k], output="real", sort=lambda re, im: np.hypot(re, im) > thr)
    b = H[k, k - 1] * Z[k - 1, :sdim]
    Q[:, :sdim] = Q[:, :k] @ Z[:, :sdim]
    Q[:, sdim] = Q[:, k]
    H[:] = 0.0
    H[:sdim, :sdim] = T[:sdim, :sdim]
    H[sdim, :sdim] = b
    return sdim


def _top_ritz(H, k, n=10):
    e = np.linalg.eigvals(H[:k, :k])
    return e[np.argsort(-np.abs(e))][:n]


def test_lagged_matches_mgs2_from_the_unnormalised_seed_and_after_a_restart():
    A, w, q1 = _problem()
    n, k = q1.size, 40
    assert abs(np.sqrt(np.sum(w * q1 * q1)) - 1.0) > 0.1   # the basis is far from orthonormal
    Qr, Hr = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Ql, Hl = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Qr[:, 0] = Ql[:, 0] = q1
    _mgs2(A, w, Qr, Hr, 0, k)
    _lagged(A, w, Ql, Hl, 0, k)
    assert np.max(np.abs(Hl - Hr)) <= 1e-12 * np.max(np.abs(Hr))
    assert np.max(np.abs(Ql - Qr)) <= 1e-11
    ms = _restart(Qr, Hr, k, 12)
    assert _restart(Ql, Hl, k, 12) == ms
    _mgs2(A, w, Qr, Hr, ms, k)
    _lagged(A, w, Ql, Hl, ms, k)
    er, el = _top_ritz(Hr, k), _top_ritz(Hl, k)
    assert np.max(np.abs(er - el) / np.abs(er)) <= 1e-12


def test_lagged_with_an_orthonormal_basis_is_mgs2():
    """A normalised seed: G stays I to rounding, and the lagged form is DCGS2's algebra."""
    A, w, q1 = _problem(seed=5)
    q1 = q1 / np.sqrt(np.sum(w * q1 * q1))
    n, k = q1.size, 30
    Qr, Hr = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Ql, Hl = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Qr[:, 0] = Ql[:, 0] = q1
    _mgs2(A, w, Qr, Hr, 0, k)
    _lagged(A, w, Ql, Hl, 0, k)
    assert np.max(np.abs(Hl - Hr)) <= 1e-12 * np.max(np.abs(Hr))
    G = Ql.T @ (w[:, None] * Ql)
    assert np.max(np.abs(G - np.eye(k + 1))) < 1e-12


def test_lagged_in_one_column_calls_matches_one_call():
    """The factorisation cut into calls of one, one, three and the remaining columns (each call
    rebuilds the Gram rows, takes the first-step stage, and finishes its last column in the closing
    pass) gives the single call's H and Q, from the unnormalised seed."""
    A, w, q1 = _problem(seed=7)
    n, k = q1.size, 20
    Q1, H1 = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Q2, H2 = np.zeros((n, k + 1)), np.zeros((k + 1, k), order="F")
    Q1[:, 0] = Q2[:, 0] = q1
    _lagged(A, w, Q1, H1, 0, k)
    for c0, c1 in ((0, 1), (1, 2), (2, 5), (5, k)):
        _lagged(A, w, Q2, H2, c0, c1)
    assert np.max(np.abs(H2 - H1)) <= 1e-12 * np.max(np.abs(H1))
    assert np.max(np.abs(Q2 - Q1)) <= 1e-11


def test_lagged_flags_a_closed_krylov_space():
    """An operator of rank 3: the fourth column has no new direction.  Either the algebra raises the
    NaN error (r^2 <= 0) or H's subdiagonal collapses where krylov_schur's breakdown test
    (breakdown_column) looks; both make krylov_schur redo the factorisation in MGS2 order."""
    from nekstab_next_amd._lib import NkvNaNError
    from nekstab_next_amd.krylov_schur import breakdown_column

    rng = np.random.default_rng(1)
    n = 200
    U = np.linalg.qr(rng.standard_normal((n, 3)))[0]
    A = U @ np.diag([0.9, 0.5, 0.2]) @ U.T
    w = np.ones(n)
    q1 = A @ rng.standard_normal(n)
    Q, H = np.zeros((n, 8)), np.zeros((8, 7), order="F")
    Q[:, 0] = q1
    try:
        _lagged(A, w, Q, H, 0, 7)
    except NkvNaNError:
        return
    assert 0 <= breakdown_column(H, 0, 7, 1e-8) <= 3


def test_lagged_coef_rejects_bad_input():
    """nkv_lagged_coef's argument checks (a status, not a crash): stage, sizes, NULL arrays."""
    from nekstab_next_amd import _lib

    lib = _lib.load()
    a = np.zeros(64)
    p = a.ctypes.data
    assert lib.nkv_lagged_coef(2, 3, p, p, 3, p, 3, p) == _lib.NKV_EINVAL
    assert lib.nkv_lagged_coef(0, 0, p, p, 1, p, 1, p) == _lib.NKV_EINVAL   # stage 0 needs a previous column
    assert lib.nkv_lagged_coef(2, 1, p, p, 2, p, 3, p) == _lib.NKV_EINVAL   # ldg < c+1
    assert lib.nkv_lagged_coef(2, 1, None, p, 3, p, 3, p) == _lib.NKV_EINVAL
    assert "lagged" in _lib.last_error()
