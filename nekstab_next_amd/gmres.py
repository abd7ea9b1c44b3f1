"""Time-stepper GMRES (the Newton–Krylov inner solver) on the device basis.

Reference: ``ts_gmres(rhs, sol, maxiter, ksize, calls)`` and ``initialize_gmres_vector``
(core/newton_krylov.f90:170-299, 303-326), Saad's restarted GMRES (alg. 6.9):

    Q(1) = rhs/||rhs||, beta = ||rhs||                                   :241-242
    do restart i = 1, maxiter
        H = 0; e = beta e_1
        do k = 1, k_dim
            arnoldi_factorization(Q, H, k, k, ksize)   (one column, MGS2)   :252
            y = lstsq(H(1:k+1,1:k), e(1:k+1))          (dgels)              :255
            beta = ||e - H y||;  exit if beta**2 < tol                      :258-269
        sol += k_matmul(Q(1:k), y)                                          :279-280
        Q(1) = -(A sol - rhs)/||.||, beta = ||A sol - rhs||                 :283-284
        exit if beta**2 < tol                                               :291-292

Differences, all documented in DESIGN.md: the orthogonalisation is the block CGS2 kernel path
(or ``mode="mgs2"``); ``Q(2:ksize+1)`` is not zeroed at each restart (every column is written by
the Arnoldi step before it is read); when the inner loop runs to k_dim without converging the
reference leaves ``k = k_dim+1`` and reads ``yvec(k_dim+1)`` out of bounds in ``k_matmul`` — here the
update uses the k_dim columns that exist.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import lapack
from .arnoldi import HessenbergDev, arnoldi_factorization
from .config import GmresConfig
from .operators import LinearOperator
from .vector import NekContext, NekVector, k_add2, k_copy, k_cmult, k_matmul, k_normalize, k_sub2


@dataclass
class GmresInfo:
    converged: bool
    restarts: int
    inner_residuals: list = field(default_factory=list)   # beta**2 per Arnoldi column (residu_arnoldi.dat)
    outer_residuals: list = field(default_factory=list)   # beta**2 per restart (residu_gmres.dat)
    y_history: list = field(default_factory=list)
    matvecs: int = 0


def initialize_gmres_vector(ctx: NekContext, op: LinearOperator, q: NekVector, rhs: NekVector,
                            f: NekVector) -> float:
    """q <- -(A q - rhs)/||A q - rhs||; returns the norm (newton_krylov.f90:303-326)."""
    op.matvec(q, f)
    k_sub2(f, rhs)
    k_cmult(f, -1.0)
    beta = k_normalize(f)
    k_copy(q, f)
    return beta


def ts_gmres(ctx: NekContext, op: LinearOperator, rhs: NekVector, sol: NekVector,
             cfg: GmresConfig | None = None) -> GmresInfo:
    """Solve A sol = rhs; ``sol`` is overwritten (starts from zero, newton_krylov.f90:234)."""
    cfg = cfg or GmresConfig()
    ks = cfg.k_dim
    Q = ctx.basis(ks + 1)
    Hd = HessenbergDev(ctx, ks)
    f = ctx.vector()
    dq = ctx.vector()
    sol.zero()
    k_copy(Q[0], rhs)
    beta = k_normalize(Q[0])
    info = GmresInfo(False, 0)
    for it in range(cfg.maxiter):
        Hd.t.zero_()
        H = np.zeros((ks + 1, ks), order="F")
        evec = np.zeros(ks + 1)
        evec[0] = beta
        yvec = np.zeros(ks)
        k_used = ks
        for k in range(1, ks + 1):
            arnoldi_factorization(ctx, op, Q, Hd, k, k, f=f, mode=cfg.mode)
            info.matvecs += 1
            H[: k + 1, k - 1] = Hd.t[k - 1, : k + 1].cpu().numpy()
            yvec[:k] = lapack.lstsq(H[: k + 1, :k], evec[: k + 1])
            beta = float(np.linalg.norm(evec[: k + 1] - H[: k + 1, :k] @ yvec[:k]))
            info.inner_residuals.append(beta ** 2)
            k_used = k
            if beta ** 2 < cfg.tol or (cfg.findiff and beta ** 2 < 1e-8):
                break
        ctx.check_nan()
        info.y_history.append(yvec[:k_used].copy())
        k_matmul(dq, Q, yvec[:k_used], k_used)
        k_add2(sol, dq)
        k_copy(Q[0], sol)
        beta = initialize_gmres_vector(ctx, op, Q[0], rhs, f)
        info.matvecs += 1
        info.outer_residuals.append(beta ** 2)
        info.restarts = it + 1
        if beta ** 2 < cfg.tol or (cfg.findiff and beta ** 2 < 1e-6):
            info.converged = True
            break
    return info
