"""CPU check of the algebra behind svds' delayed re-orthogonalisation (nekstab_next_amd.lightkrylov
._gkl_dcgs2 / the kernel k_gkl_coef, include/nekkrylov.h "svds"), restated in numpy with the same
coefficient rule: two interleaved DCGS2 sequences, the projections of a provisional vector's image
corrected once it is finished (A v~ = r A v + U C a).  Against a plain Golub–Kahan–Lanczos with
full CGS2 re-orthogonalisation and a dense W-weighted SVD (no GPU)."""
import numpy as np
import pytest


def _ip(w):
    return lambda a, b: float(np.sum(a * w * b))


def gkl_dcgs2(A, At, w, v0, k):
    """numpy twin of _gkl_dcgs2: per pass (a, r) of the provisional column from hq, the raw
    coefficients of the other side's output from hw, and the previous column finalised."""
    ip = _ip(w)
    n = v0.size
    U, V = np.zeros((k + 1, n)), np.zeros((k + 1, n))
    C, D = np.zeros((k + 1, k)), np.zeros((k + 1, k))
    AU, AV = np.zeros((k + 1, k + 1)), np.zeros((k + 1, k + 1))
    rU, rV = np.zeros(k + 1), np.zeros(k + 1)
    V[0] = v0

    def coef(side, m, hq, hw, M, As, rs, Ao, ro):
        a = hq[:m]
        r = np.sqrt(hq[m] - a @ a)
        As[:m, m], rs[m] = a, r
        p = m - side
        out = dict(a=a, r=r)
        if hw is not None:
            b = hw[:m]
            bm = (hw[m] - a @ b) / r
            M[:m, p + 1], M[m, p + 1] = b, bm
            out.update(x=b / r, y=bm / r)
        if p >= 0:
            rho = rs[m - 1] if m > 0 else 1.0
            M[:m, p] = (M[:m, p] - M[:m, :p] @ Ao[:p, p] + rho * a) / ro[p]
            M[m, p] = rho * r / ro[p]
        return out

    def update(Q, m, c, f, out_col):
        qbar = (Q[m] - Q[:m].T @ c["a"]) / c["r"]
        Q[m] = qbar
        if f is not None:
            Q[out_col] = f / c["r"] - Q[:m].T @ c["x"] - qbar * c["y"]

    def dots(Q, m, f):
        hq = np.array([ip(Q[i], Q[m]) for i in range(m + 1)])
        hw = None if f is None else np.array([ip(Q[i], f) for i in range(m + 1)])
        return hq, hw

    U[0] = A(V[0])
    for j in range(1, k + 1):
        if j > 1:
            f = A(V[j - 1])
            m = j - 2
            update(U, m, coef(0, m, *dots(U, m, f), C, AU, rU, AV, rV), f, j - 1)
        f = At(U[j - 1])
        m = j - 1
        update(V, m, coef(1, m, *dots(V, m, f), D, AV, rV, AU, rU), f, j)
    update(U, k - 1, coef(0, k - 1, *dots(U, k - 1, None), C, AU, rU, AV, rV), None, None)
    update(V, k, coef(1, k, *dots(V, k, None), D, AV, rV, AU, rU), None, None)
    return U, V, C[:k], D


def gkl_cgs2(A, At, w, v0, k):
    ip = _ip(w)
    n = v0.size
    U, V = np.zeros((k + 1, n)), np.zeros((k + 1, n))
    C, D = np.zeros((k, k)), np.zeros((k + 1, k))
    V[0] = v0

    def orth(Q, j, f):
        h = np.zeros(j + 1)
        for _ in range(2):
            c = np.array([ip(Q[i], f) for i in range(j)])
            f = f - Q[:j].T @ c
            h[:j] += c
        h[j] = np.sqrt(ip(f, f))
        return f / h[j], h

    for j in range(1, k + 1):
        U[j - 1], C[:j, j - 1] = orth(U, j - 1, A(V[j - 1]))
        V[j], D[: j + 1, j - 1] = orth(V, j, At(U[j - 1]))
    return U, V, C, D


@pytest.mark.parametrize("k", [1, 2, 7, 24])
def test_gkl_delayed_reorth_algebra(k):
    rng = np.random.default_rng(k)
    n = 300
    w = rng.uniform(0.5, 1.5, n)
    M = rng.standard_normal((n, n)) @ np.diag(np.logspace(0, -5, n)) @ rng.standard_normal((n, n)) / 20
    A = lambda x: M @ x                   # noqa: E731
    At = lambda y: (M.T @ (w * y)) / w    # noqa: E731  (W-adjoint: <At y, x>_W = <y, A x>_W)
    v0 = rng.standard_normal(n)
    v0 /= np.sqrt(np.sum(v0 * w * v0))
    U, V, C, D = gkl_dcgs2(A, At, w, v0, k)
    Uc, Vc, Cc, Dc = gkl_cgs2(A, At, w, v0, k)
    for B, nb in ((U, k), (V, k + 1)):
        G = B[:nb] @ (w * B[:nb]).T
        assert np.abs(G - np.eye(nb)).max() < 1e-13
    AV = np.stack([A(V[c]) for c in range(k)], 1)
    assert np.abs(AV - U[:k].T @ C).max() < 1e-13 * np.abs(AV).max()
    AtU = np.stack([At(U[c]) for c in range(k)], 1)
    assert np.abs(AtU - V[: k + 1].T @ D).max() < 1e-13 * np.abs(AtU).max()
    assert np.abs(np.tril(C, -1)).max() == 0.0 and np.abs(np.tril(D, -2)).max() == 0.0
    np.testing.assert_allclose(C, Cc, rtol=0, atol=1e-12 * np.abs(Cc).max())
    np.testing.assert_allclose(D, Dc, rtol=0, atol=1e-12 * np.abs(Dc).max())
    sw = np.sqrt(w)
    s_true = np.linalg.svd(sw[:, None] * M / sw[None, :], compute_uv=False)
    s = np.linalg.svd(C, compute_uv=False)
    if k >= 24:
        np.testing.assert_allclose(s[:3], s_true[:3], rtol=1e-12)
