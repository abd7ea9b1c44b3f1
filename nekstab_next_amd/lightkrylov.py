"""LightKrylov-compatible API surface over the MI355X kernels.

nekStab's live drivers call LightKrylov (external, not vendored, unpinned — `LightKrylov_setup.sh:54`
clones `main`):

* ``eigs(A, X, eigvecs, eigvals, residuals, info, nev=schur_tgt, tolerance=eigen_tol, transpose)``
  (core/linear_stab.f90:66-67),
* ``svds(A, U, V, uvecs, vvecs, sigma, residuals, info, nev, tolerance)`` for transient growth and
  resolvent analysis (:112, :153; nekStab then squares sigma),
* ``gmres(S, b, x, info, options=gmres_opts(atol, rtol), transpose)`` with
  ``S = axpby_linop(identity_linop(), A, 1, -1, .false., .true.)`` (core/linear_operators.f90:405-416),
* ``get_vec(vec, X(1:k), coeffs)`` to build eigen/singular vectors (linear_stab.f90:362-378).

LightKrylov's own arithmetic is not in the container, so these are restatements of the published
algorithms with nekStab's call semantics — parity unpinned for this surface:
``eigs`` runs nekStab's Krylov–Schur (``krylov_schur.py``) in the caller's basis ``X``; ``svds`` is a
k-step Golub–Kahan–Lanczos bidiagonalisation with full CGS2 re-orthogonalisation of both bases (the
same block kernels; two bases resident, as BASELINE config 5); ``gmres`` is restarted GMRES stopping
on ||r|| <= rtol ||b|| + atol.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lapack
from .arnoldi import HessenbergDev, arnoldi_factorization, orthonormalize
from .config import KrylovSchurConfig
from ._lib import NkvNaNError
from .krylov_schur import _MGS2, _mgs2_of, breakdown_column, krylov_schur
from .operators import LinearOperator
from .vector import Basis, NekContext, NekVector, combine, k_add2, k_copy, k_matmul


class IdentityLinop(LinearOperator):
    def matvec(self, x: NekVector, y: NekVector) -> None:
        y.copy_from(x)

    rmatvec = matvec


class AxpbyLinop(LinearOperator):
    """S x = alpha op(A) x + beta op(B) x with op = transpose when the flag is set
    (LightKrylov ``axpby_linop(A, B, alpha, beta, transA, transB)``)."""

    def __init__(self, A: LinearOperator, B: LinearOperator, alpha: float, beta: float, transA: bool = False,
                 transB: bool = False):
        self.A, self.B, self.alpha, self.beta, self.tA, self.tB = A, B, float(alpha), float(beta), transA, transB
        self._tmp = None

    def _apply(self, x, y, flip):
        if self._tmp is None:
            self._tmp = x.ctx.vector()
        ta, tb = self.tA ^ flip, self.tB ^ flip
        (self.A.rmatvec if ta else self.A.matvec)(x, y)
        (self.B.rmatvec if tb else self.B.matvec)(x, self._tmp)
        y.axpby(self.alpha, self._tmp, self.beta)

    def matvec(self, x, y):
        self._apply(x, y, False)

    def rmatvec(self, x, y):
        self._apply(x, y, True)


def get_vec(out: NekVector, X: Basis, coeffs, k: int | None = None) -> None:
    """out = X(1:k) coeffs (real coefficients), fields only (LightKrylov ``get_vec``)."""
    c = np.asarray(coeffs, dtype=np.float64)
    k = c.shape[0] if k is None else k
    combine(out, X, torch.as_tensor(np.ascontiguousarray(c[:k])).to(out.ctx.device), k, with_time=False)


def eigs(ctx: NekContext, A: LinearOperator, X: Basis, nev: int, tolerance: float, transpose: bool = False,
         schur_del: float = 0.1, mode: str = "dcgs2"):
    """Leading eigenpairs of A (or A^T) in the caller's basis X (X[0] = prepared seed).  Returns
    (eigvecs[k,k] complex Krylov coefficients, eigvals[k], residuals[k], info)."""
    k = X.k - 1
    cfg = KrylovSchurConfig(k_dim=k, schur_tgt=nev, eigen_tol=tolerance, schur_del=schur_del, mode=mode)
    seed = ctx.vector()
    seed.copy_from(X[0])
    res = krylov_schur(ctx, A, seed, cfg, transpose=transpose, Q=X)
    info = 0 if (nev <= 0 or res.converged >= nev) else 1
    return res.vecs, res.vals, res.residual, info


@dataclass
class SvdsResult:
    sigma: np.ndarray      # singular values, decreasing
    uvecs: np.ndarray      # k x k: left singular vectors = U(1:k) uvecs(:, i)
    vvecs: np.ndarray      # k x k: right singular vectors = V(1:k) vvecs(:, i)
    residuals: np.ndarray  # beta_k |p_i(k)|
    info: int
    C: np.ndarray          # k x k upper-triangular projection A V_k = U_k C
    breakdown: bool = False  # the bidiagonalisation reached an invariant subspace and was redone in MGS2


def svds(ctx: NekContext, A: LinearOperator, U: Basis, V: Basis, nev: int, tolerance: float,
         mode: str = "cgs2", breakdown_tol: float = 1e-8) -> SvdsResult:
    """k-step Golub–Kahan–Lanczos bidiagonalisation with full re-orthogonalisation, k = len(U)-1.
    V[0] holds the prepared (normalised) seed.  A: ``matvec`` (direct) and ``rmatvec`` (adjoint).

    A rank-deficient A makes the bidiagonalisation invariant before k steps (alpha_j or beta_j is
    rounding noise).  As in ``krylov_schur`` the classical modes cannot carry on from noise, so
    after the k steps the new-direction norms are checked (``breakdown_column``, |alpha_j| or
    |beta_j| < ``breakdown_tol`` x its column, or a NaN) and the whole bidiagonalisation is redone in
    the one-projection-at-a-time MGS2 order (V[0] is never written, so it needs no snapshot)."""
    k = U.k - 1
    if V.k < k + 1:
        raise ValueError("V must have as many vectors as U")
    Cd = HessenbergDev(ctx, k)   # columns: projections of A v_j on u_1..u_j (+ norm)
    Dd = HessenbergDev(ctx, k)   # columns: projections of A^T u_j on v_1..v_{j+1}
    f = ctx.vector()
    broken = False
    while True:
        for j in range(1, k + 1):
            A.matvec(V[j - 1], f)
            orthonormalize(ctx, U, j - 1, f, U.col_ptr(j - 1), Cd.col_ptr(j - 1), mode)
            A.rmatvec(U[j - 1], f)
            orthonormalize(ctx, V, j, f, V.col_ptr(j), Dd.col_ptr(j - 1), mode)
        if mode in _MGS2:
            ctx.check_nan()
            break
        try:
            ctx.check_nan()
            nan = False
        except NkvNaNError:
            nan = True
        broken_here = (nan or breakdown_column(Cd.download(), 0, k, breakdown_tol, offset=0) >= 0
                       or breakdown_column(Dd.download(), 0, k, breakdown_tol, offset=1) >= 0)
        if ctx.comm.world > 1:   # the C/D tests are replicated; the NaN flag is per rank
            flag = torch.tensor([1.0 if broken_here else 0.0], dtype=torch.float64, device=ctx.device)
            broken_here = float(ctx.comm.allreduce_(flag).item()) > 0.0
        if not broken_here:
            break
        mode, broken = _mgs2_of(mode), True
    Ct = Cd.download()  # (k+1, k): column j-1 holds <u_i, A v_j> (i < j) and alpha_j at row j-1
    C = np.zeros((k, k))
    for j in range(k):
        C[: j + 1, j] = Ct[: j + 1, j]
    beta_k = Dd.download()[k, k - 1]
    P, s, Rt = np.linalg.svd(C)
    residuals = np.abs(beta_k * P[k - 1, :])
    info = 0 if int(np.count_nonzero(residuals < tolerance)) >= nev else 1
    return SvdsResult(sigma=s, uvecs=P, vvecs=Rt.T, residuals=residuals, info=info, C=C, breakdown=broken)


def gmres(ctx: NekContext, A: LinearOperator, b: NekVector, x: NekVector, atol: float = 1e-12,
          rtol: float = 1e-12, kdim: int = 30, maxiter: int = 10, transpose: bool = False,
          mode: str = "cgs2"):
    """Restarted GMRES from the initial guess ``x`` (updated in place); stops when
    ||b - A x||_W <= rtol ||b||_W + atol.  Returns (info, residual_history); info = 0 converged."""
    Q = ctx.basis(kdim + 1)
    Hd = HessenbergDev(ctx, kdim)
    f = ctx.vector()
    r = ctx.vector()
    apply = A.rmatvec if transpose else A.matvec
    bnorm = float(np.sqrt(ctx.dot(b, b, ctx.time_in_dot)))
    tol = rtol * bnorm + atol
    hist = []
    for _ in range(maxiter):
        apply(x, r)
        r.axpby(-1.0, b, 1.0)  # r = b - A x
        beta = float(np.sqrt(ctx.dot(r, r, ctx.time_in_dot)))
        hist.append(beta)
        if beta <= tol:
            return 0, hist
        k_copy(Q[0], r)
        Q[0].scal(1.0 / beta)
        Hd.t.zero_()
        e = np.zeros(kdim + 1)
        e[0] = beta
        H = np.zeros((kdim + 1, kdim))
        k_used = kdim
        y = None
        for k in range(1, kdim + 1):
            arnoldi_factorization(ctx, A, Q, Hd, k, k, f=f, mode=mode, transpose=transpose)
            H[: k + 1, k - 1] = Hd.t[k - 1, : k + 1].cpu().numpy()
            y = lapack.lstsq(H[: k + 1, :k], e[: k + 1])
            res = float(np.linalg.norm(e[: k + 1] - H[: k + 1, :k] @ y))
            k_used = k
            if res <= tol:
                break
        dq = ctx.vector()
        k_matmul(dq, Q, y, k_used)
        k_add2(x, dq)
    apply(x, r)
    r.axpby(-1.0, b, 1.0)
    beta = float(np.sqrt(ctx.dot(r, r, ctx.time_in_dot)))
    hist.append(beta)
    return (0 if beta <= tol else 1), hist
