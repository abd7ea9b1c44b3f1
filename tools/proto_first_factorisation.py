"""Prototype (numpy, W = I): the reference's MGS2 Arnoldi on a basis whose first column is
unnormalised (the default noise seed: Q(1) = A q0, eigensolvers.f90:192-203), computed from ONE
multi-dot per step plus a Q'-only re-orthogonalisation, against the column-by-column MGS2 of
krylov_decomposition.f90:155-180.

With Q = [q1, Q'], r^2 = <q1, q1>, g = Q'^T q1 and Q' orthonormal (it is, in the first
factorisation: DESIGN.md §10 open directions), MGS2's coefficients follow from b = Q^T f alone:
  pass 1: a1 = b1,  B1 = b' - a1 g;   pass 2: a2 = b1 - a1 r^2 - g.B1,  B2 = -a2 g
  h = (a1 + a2, B1 + B2),  f <- f - q1 h1 - Q' h'
and the exact result is orthogonal to Q', so the rounding left by the closed form is removed by a
projection onto Q'-perp (in DCGS2 form: merged into the next step's multi-dot, two reads of Q per
step instead of the three of "mgs2-icwy").  Prints max |H_proto - H_mgs2| / max |H|.

  python tools/proto_first_factorisation.py
"""
import numpy as np


def mgs2(A, q1, m):
    n = q1.size
    Q = np.zeros((n, m + 1))
    H = np.zeros((m + 1, m))
    Q[:, 0] = q1
    for k in range(m):
        f = A @ Q[:, k]
        h = np.zeros(k + 1)
        for _ in range(2):
            for i in range(k + 1):
                a = Q[:, i] @ f
                f = f - a * Q[:, i]
                h[i] += a
        H[: k + 1, k] = h
        H[k + 1, k] = np.linalg.norm(f)
        Q[:, k + 1] = f / H[k + 1, k]
    return Q, H


def closed_form(A, q1, m):
    n = q1.size
    Q = np.zeros((n, m + 1))
    H = np.zeros((m + 1, m))
    Q[:, 0] = q1
    r2 = q1 @ q1
    for k in range(m):
        f = A @ Q[:, k]
        b = Q[:, : k + 1].T @ f                 # the step's one multi-dot
        g = Q[:, 1: k + 1].T @ q1               # Gram row of q1 (kept incrementally in practice)
        a1 = b[0]
        B1 = b[1:] - a1 * g
        a2 = b[0] - a1 * r2 - g @ B1
        B2 = -a2 * g
        h = np.concatenate([[a1 + a2], B1 + B2])
        f = f - Q[:, : k + 1] @ h               # the update (second read)
        c = Q[:, 1: k + 1].T @ f                # Q'-only correction (DCGS2: delayed into the next multi-dot)
        f = f - Q[:, 1: k + 1] @ c
        h[1:] += c
        H[: k + 1, k] = h
        H[k + 1, k] = np.linalg.norm(f)
        Q[:, k + 1] = f / H[k + 1, k]
    return Q, H


def main():
    rng = np.random.default_rng(0)
    for n, m, scale in ((400, 40, 1.0), (2000, 100, 1.0), (2000, 100, 30.0)):
        A = rng.standard_normal((n, n)) / np.sqrt(n) + np.diag(np.linspace(0.0, 1.5, n))
        q0 = rng.standard_normal(n)
        q0 /= np.linalg.norm(q0)
        q1 = scale * (A @ q0)
        _, Hm = mgs2(A, q1, m)
        Qc, Hc = closed_form(A, q1, m)
        G = Qc[:, 1:].T @ Qc[:, 1:]
        ev_m = np.sort_complex(np.linalg.eigvals(Hm[:m, :m]))
        ev_c = np.sort_complex(np.linalg.eigvals(Hc[:m, :m]))
        print(f"n={n} m={m} |q1|={np.linalg.norm(q1):.3g}: max|H_c - H_mgs2|/max|H| = "
              f"{np.abs(Hc - Hm).max() / np.abs(Hm).max():.2e}, ||Q'^T Q' - I|| = "
              f"{np.abs(G - np.eye(m)).max():.2e}, Ritz max rel diff = "
              f"{np.max(np.abs(ev_c - ev_m) / np.abs(ev_m)):.2e}")


if __name__ == "__main__":
    main()
