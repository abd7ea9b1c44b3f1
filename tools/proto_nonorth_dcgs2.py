"""Prototype (numpy, W = I): the reference's MGS2 Arnoldi on a NON-orthonormal basis (the default
noise seed, eigensolvers.f90:195-203: Q(1) = A q0 unnormalised; and what a Krylov–Schur restart
makes of it, Q(:,1:ms) <- Q(:,1:k) V) computed with TWO reads of Q per step, against the
column-by-column MGS2 of krylov_decomposition.f90:155-180 (the oracle's order).

MGS on a basis with Gram matrix G = Q^T Q (not I) is not a projection: its coefficients are
alpha = (I + L)^-1 Q^T f with L the strictly lower part of G.  The lagged form keeps, as DCGS2 does,
the newest column provisional (u = the first-pass result) and finishes it inside the next step:

  y = A u;  one multi-dot: p = Q^T u, pu = u.u, t = Q^T y, tu = u.y       (read 1)
  beta = (I+L)^-1 p;  r^2 = pu - 2 beta.p + beta^T G beta;  q = (u - Q beta) / r
  G's new row: (p - G beta) / r;  H(:, c-1) += beta, H(c, c-1) = r
  A q = (y - Q_c H_c beta) / r   (the Arnoldi relation of the finished columns)
  b = Q_c^T A q = ([t; (tu - beta.t)/r] - G_c H_c beta) / r;  alpha = (I+L_c)^-1 b
  u_next = y / r - Q_c (H_c beta / r + alpha)                              (read 2, also writes q)

With G = I it is DCGS2.  Prints max |H_lagged - H_mgs2| / max |H| for a first factorisation from an
unnormalised seed, and the top-10 Ritz values after a restart, over operators of increasing spread.

  python tools/proto_nonorth_dcgs2.py
"""
import numpy as np


def mgs2_steps(A, Q, H, c0, c1):
    """Reference order: columns c0..c1-1 (0-based step c: f = A q_c, two MGS passes over q_0..q_c)."""
    for c in range(c0, c1):
        f = A @ Q[:, c]
        h = np.zeros(c + 1)
        for _ in range(2):
            for i in range(c + 1):
                a = Q[:, i] @ f
                f = f - a * Q[:, i]
                h[i] += a
        H[: c + 1, c] = h
        H[c + 1, c] = np.linalg.norm(f)
        Q[:, c + 1] = f / H[c + 1, c]


def lagged_steps(A, Q, H, G, c0, c1):
    """The same columns with one multi-dot and one update per step.  On entry Q[:, :c0+1] and
    G[:c0+1, :c0+1] are final (q_c0 is the column the first matvec acts on).  On exit the same
    holds for c1 (a closing pass finishes the last provisional column)."""
    def lower_solve(Gc, rhs):   # (I + L) x = rhs, L = strictly lower part of Gc
        n = rhs.size
        x = np.zeros(n)
        for i in range(n):
            x[i] = rhs[i] - Gc[i, :i] @ x[:i]
        return x

    # first step (no pending second pass): f = A q_c0, one pass
    c = c0
    y = A @ Q[:, c]
    b = Q[:, : c + 1].T @ y
    alpha = lower_solve(G[: c + 1, : c + 1], b)
    u = y - Q[:, : c + 1] @ alpha
    H[: c + 1, c] = alpha
    for c in range(c0 + 1, c1 + 1):   # finish column c (u), then the first pass of A q_c
        y = A @ u if c < c1 else None
        Qp = Q[:, :c]                                   # final columns 0..c-1
        p, pu = Qp.T @ u, u @ u                         # the multi-dot (read 1)
        beta = lower_solve(G[:c, :c], p)
        r = np.sqrt(pu - 2.0 * beta @ p + beta @ G[:c, :c] @ beta)
        H[:c, c - 1] += beta
        H[c, c - 1] = r
        g = (p - G[:c, :c] @ beta) / r
        G[:c, c] = G[c, :c] = g
        G[c, c] = 1.0
        Q[:, c] = (u - Qp @ beta) / r                   # (read 2, first output)
        if c == c1:
            break
        t, tu = Qp.T @ y, u @ y
        Hc = H[: c + 1, :c]
        bq = np.concatenate([t, [(tu - beta @ t) / r]])
        b = (bq - G[: c + 1, : c + 1] @ (Hc @ beta)) / r
        alpha = lower_solve(G[: c + 1, : c + 1], b)
        u = y / r - Q[:, : c + 1] @ (Hc @ beta / r + alpha)   # (read 2, second output)
        H[: c + 1, c] = alpha


def run(n=4000, k=40, ms=12, spread=1e2, seed=0):
    rng = np.random.default_rng(seed)
    lam = np.concatenate([np.linspace(1.0, 0.9, 6), rng.uniform(0.0, 0.8, n - 6)])
    lam = lam * np.where(rng.random(n) < 0.5, 1.0, spread ** (-rng.random(n)))
    U = np.linalg.qr(rng.standard_normal((n, n)))[0] if n <= 600 else None
    A = (U * lam) @ U.T if U is not None else np.diag(lam)
    x = rng.standard_normal(n)
    q1 = A @ (x / np.linalg.norm(x))                    # the noise seed: NOT renormalised
    out = {}
    Qr, Hr = np.zeros((n, k + 1)), np.zeros((k + 1, k))
    Ql, Hl, G = np.zeros((n, k + 1)), np.zeros((k + 1, k)), np.zeros((k + 1, k + 1))
    Qr[:, 0] = Ql[:, 0] = q1
    G[0, 0] = q1 @ q1
    mgs2_steps(A, Qr, Hr, 0, k)
    lagged_steps(A, Ql, Hl, G, 0, k)
    out["first"] = np.max(np.abs(Hl - Hr)) / np.max(np.abs(Hr))
    # a restart as schur_condensation does it, on both: Schur form of H_k sorted so the largest
    # |lambda| come first, Q(:,1:ms) <- Q(:,1:k) Z, H <- [T11; b^T Z1], Q(ms+1) <- Q(k+1)
    import scipy.linalg as sla

    outs = []
    for Q, H in ((Qr, Hr), (Ql, Hl)):
        w = np.sort(np.abs(np.linalg.eigvals(H[:k, :k])))[::-1]
        thr = 0.5 * (w[ms - 1] + w[ms])
        T, Z, sdim = sla.schur(H[:k, :k], output="real", sort=lambda re, im: np.hypot(re, im) > thr)
        b = H[k, k - 1] * Z[k - 1, :sdim]
        Q[:, :sdim] = Q[:, :k] @ Z[:, :sdim]
        Q[:, sdim] = Q[:, k]
        H[:] = 0.0
        H[:sdim, :sdim] = T[:sdim, :sdim]
        H[sdim, :sdim] = b
        outs.append(sdim)
    m0 = outs[0]
    assert outs[0] == outs[1]
    G[:] = 0.0
    G[: m0 + 1, : m0 + 1] = Ql[:, : m0 + 1].T @ Ql[:, : m0 + 1]   # the lagged form's G after the rotation
    mgs2_steps(A, Qr, Hr, m0, k)
    lagged_steps(A, Ql, Hl, G, m0, k)
    # H itself depends on the Schur vectors' signs and the order inside T (scipy's schur on two
    # inputs equal to rounding may differ there), so compare the Ritz values after the restart
    er = np.linalg.eigvals(Hr[:k, :k])
    el = np.linalg.eigvals(Hl[:k, :k])
    er, el = er[np.argsort(-np.abs(er))][:10], el[np.argsort(-np.abs(el))][:10]
    out["after_restart"] = float(np.max(np.abs(er - el) / np.abs(er)))
    out["kept"] = m0
    out["r_q1"] = float(np.linalg.norm(q1))
    return out


if __name__ == "__main__":
    for n in (400, 4000):
        for spread in (1.0, 1e2, 1e4):
            o = run(n=n, spread=spread)
            print(f"n={n:5d} spread={spread:7.0e} |q1|={o['r_q1']:.3f}  first factorisation "
                  f"{o['first']:.2e}  top-10 Ritz after a restart {o['after_restart']:.2e} ({o['kept']} kept)")
