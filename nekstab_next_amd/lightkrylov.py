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
k-step Golub–Kahan–Lanczos bidiagonalisation with full re-orthogonalisation of both bases (two bases
resident, as BASELINE config 5) — by default with delayed re-orthogonalisation (``"dcgs2"``: each
basis read twice per step, one all-reduce per half-step), or CGS2 (three reads); ``gmres`` is
restarted GMRES stopping on ||r|| <= rtol ||b|| + atol.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import lapack
from ._lib import NKV_TIME, NKV_X_IS_LAST
from .arnoldi import HessenbergDev, arnoldi_factorization, orthonormalize
from .config import KrylovSchurConfig
from .gmres import GivensResidual, dcgs2_cycle
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


def _gkl_dcgs2(ctx: NekContext, A: LinearOperator, U: Basis, V: Basis, k: int, Cd: HessenbergDev,
               Dd: HessenbergDev) -> None:
    """Golub–Kahan–Lanczos with delayed re-orthogonalisation (include/nekkrylov.h, nkv_gkl_coef): two
    interleaved DCGS2 sequences.  The U side's operator output is A applied to V's provisional
    vector, the V side's is A^T applied to U's; each pass over a basis finishes that basis's
    provisional column (the second projection) and projects the other side's output once (the
    first), so every vector is still projected twice, and each basis is read twice per step (a
    two-vector multi-dot and a dual update) instead of three times.  The projection coefficients
    of a provisional vector are corrected once it is finished (A ṽ = r A v + A V a, and A V = U C).
    On return U[0:k], V[0:k+1] are final and W-orthonormal, Cd/Dd hold C and D as the CGS2 path
    writes them.  V[0] (the seed) is renormalised in the first pass."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    lay, tm = ctx.layout, ctx.timer
    tf = NKV_TIME if ctx.time_in_dot else 0
    f64 = dict(dtype=torch.float64, device=ctx.device)
    ld = k + 1
    AU, AV = torch.zeros((ld, ld), **f64), torch.zeros((ld, ld), **f64)
    rU, rV = torch.zeros(ld, **f64), torch.zeros(ld, **f64)
    Cd.t.zero_()
    Dd.t.zero_()
    cp = ctx.coef.data_ptr()
    f = ctx.vector()
    sides = {0: (U, Cd, AU, rU, AV, rV), 1: (V, Dd, AV, rV, AU, rU)}

    def dual_pass(side, m, out_col):
        Q, M, As, rs, Ao, ro = sides[side]
        j = m + 1
        h = ctx.hd[: 2 * j]
        hp = h.data_ptr()
        if tm:
            tm.begin("block_dot2")
        ctx.call("nkv_block_dot2", w, Q.ptr, j, Q.col_ptr(m), f.ptr, hp, ws, tf | NKV_X_IS_LAST, st)
        if tm:
            tm.end("block_dot2", 8.0 * (m * lay.N_w + 2 * lay.N_w + lay.n_v))
        ctx.comm.allreduce_(h)
        ctx.call_nl("nkv_gkl_coef", side, m, hp, hp + 8 * j, M.t.data_ptr(), ld, As.data_ptr(), rs.data_ptr(),
                    Ao.data_ptr(), ro.data_ptr(), ld, cp, ws, st)
        if tm:
            tm.begin("dcgs2_update")
        ctx.call("nkv_dcgs2_update", w, Q.ptr, m, cp, Q.col_ptr(m), f.ptr, Q.col_ptr(out_col), None, ws, NKV_TIME, st)
        if tm:
            tm.end("dcgs2_update", 8.0 * (m * lay.N + 4 * lay.N))

    def close(side, m):
        Q, M, As, rs, Ao, ro = sides[side]
        h = ctx.hd[: m + 1]
        if tm:
            tm.begin("block_dot")
        ctx.call("nkv_block_dot", w, Q.ptr, m + 1, Q.col_ptr(m), h.data_ptr(), ws, tf, st)
        if tm:
            tm.end("block_dot", 8.0 * ((m + 1) * lay.N_w + lay.N_w + lay.n_v))
        ctx.comm.allreduce_(h)
        ctx.call_nl("nkv_gkl_coef", side, m, h.data_ptr(), None, M.t.data_ptr(), ld, As.data_ptr(), rs.data_ptr(),
                    Ao.data_ptr(), ro.data_ptr(), ld, cp, ws, st)
        if m > 0:
            if tm:
                tm.begin("block_update")
            ctx.call("nkv_block_update", w, Q.ptr, m, ctx.coef[2 * m + 5:].data_ptr(), Q.col_ptr(m), None, ws,
                     NKV_TIME, st)
            if tm:
                tm.end("block_update", 8.0 * (m * lay.N + 2 * lay.N))
        ctx.call("nkv_normalize_dev", Q.col_ptr(m), ctx.coef[2 * m + 3:].data_ptr(), None, 0, st)

    A.matvec(V[0], U[0])            # step 1, U side: the first provisional u is A v_0 itself
    for j in range(1, k + 1):
        if j > 1:
            A.matvec(V[j - 1], f)
            dual_pass(0, j - 2, j - 1)
        A.rmatvec(U[j - 1], f)
        dual_pass(1, j - 1, j)
    close(0, k - 1)
    close(1, k)


def svds(ctx: NekContext, A: LinearOperator, U: Basis, V: Basis, nev: int, tolerance: float,
         mode: str = "dcgs2", breakdown_tol: float = 1e-8) -> SvdsResult:
    """k-step Golub–Kahan–Lanczos bidiagonalisation with full re-orthogonalisation, k = len(U)-1.
    V[0] holds the prepared (normalised) seed.  A: ``matvec`` (direct) and ``rmatvec`` (adjoint).
    ``mode``: ``"dcgs2"`` (default; delayed re-orthogonalisation, two reads of each basis per step,
    see ``_gkl_dcgs2``), ``"cgs2"`` / ``"cgs2-native"`` (three reads), ``"mgs2"`` (reference order).

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
    if mode in ("dcgs2", "dcgs2-native") and (k + 1 > ctx.max_cols or ctx.hd.numel() < 2 * (k + 1)):
        raise ValueError(f"svds k={k} needs max_cols >= {k + 1}")
    while True:
        if mode in ("dcgs2", "dcgs2-native"):
            _gkl_dcgs2(ctx, A, U, V, k, Cd, Dd)
        else:
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
          mode: str = "dcgs2"):
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
        giv = GivensResidual(beta, kdim)
        if mode == "dcgs2":   # one continuous DCGS2 factorisation, the residual test per column (gmres.py)
            k_used = dcgs2_cycle(ctx, apply, Q, Hd, f, kdim, giv, lambda res: res <= tol)
            H[: k_used + 1, :k_used] = Hd.download()[: k_used + 1, :k_used]
            y = lapack.lstsq(H[: k_used + 1, :k_used], e[: k_used + 1])
            dq = ctx.vector()
            k_matmul(dq, Q, y, k_used)
            k_add2(x, dq)
            continue
        for k in range(1, kdim + 1):
            arnoldi_factorization(ctx, A, Q, Hd, k, k, f=f, mode=mode, transpose=transpose)
            H[: k + 1, k - 1] = Hd.t[k - 1, : k + 1].cpu().numpy()
            res = giv.add_column(H[: k + 1, k - 1])     # O(k) per column; y solved once below
            k_used = k
            if res <= tol:
                break
        y = lapack.lstsq(H[: k_used + 1, :k_used], e[: k_used + 1])
        dq = ctx.vector()
        k_matmul(dq, Q, y, k_used)
        k_add2(x, dq)
    apply(x, r)
    r.axpby(-1.0, b, 1.0)
    beta = float(np.sqrt(ctx.dot(r, r, ctx.time_in_dot)))
    hist.append(beta)
    return (0 if beta <= tol else 1), hist
