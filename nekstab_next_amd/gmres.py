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

Orthogonalisation (``GmresConfig.mode``): ``"dcgs2-native"`` (default) / ``"dcgs2"`` (the same
sequence driven from Python, bit-identical) runs the inner Arnoldi as ONE continuous
DCGS2 factorisation (two reads of the basis per column instead of CGS2's three) with the norm of
each new provisional vector fused into the update (``_dcgs2_step(nrm2=...)``), so the residual test
of column k needs nothing from column k+1 — no lag, no extra matvec.  Column k's coefficients are
then the once-projected ones (its re-orthogonalisation correction, O(eps) relative, arrives with the
next column); the test uses them, and after the exit one closing multi-dot finalises the last
column's row of H, so ``lstsq`` (dgels) sees an Arnoldi factorisation exact to rounding, as with
CGS2.  ``"cgs2"`` / ``"mgs2"``: one finished column per step (``arnoldi_factorization(k, k)``).

Host work per inner iteration is O(k): the reference solves the whole (k+1) x k least-squares
problem with dgels at every column only to test ||e - H y|| (:255-258).  That residual is the
last entry of Q_k^T e after the Givens rotations that triangularise H (Saad alg. 6.9's own
update), so each column applies the k-1 stored rotations to the new H column, forms one more,
and reads the residual off; ``lstsq`` (dgels, the reference's call) runs once, on the final
system, so y is the reference's.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib, lapack
from .arnoldi import HessenbergDev, arnoldi_factorization
from .config import GmresConfig
from .operators import LinearOperator
from .vector import NekContext, NekVector, k_add2, k_copy, k_cmult, k_matmul, k_normalize, k_sub2


class GivensResidual:
    """||beta e_1 - H_k y_k|| of the GMRES least-squares problem, updated per Hessenberg column in
    O(k): the rotations G_i that reduce H to upper-triangular R are stored, column k gets
    G_{k-1} ... G_1 and a new rotation G_k zeroing H(k+1, k); g = G_k ... G_1 beta e_1, and the
    least-squares residual is |g_{k+1}| (Saad, Iterative Methods, 2nd ed., prop. 6.9)."""

    def __init__(self, beta: float, kmax: int):
        self.cs = np.zeros(kmax)
        self.sn = np.zeros(kmax)
        self.g = np.zeros(kmax + 1)
        self.g[0] = beta
        self.h = np.zeros(kmax + 1)
        self.k = 0
        self._f = _lib.load().nkv_givens_column   # host C (include/nekkrylov.h): O(k), no device work
        self._p = [a.ctypes.data for a in (self.h, self.cs, self.sn, self.g)]

    def add_column(self, h: np.ndarray) -> float:
        """h = H(1:k+1, k) of the next column k (0-based self.k); returns the residual norm."""
        k = self.k
        self.h[: k + 2] = h[: k + 2]
        res = self._f(k, *self._p)
        self.k = k + 1
        return float(res)


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
        giv = GivensResidual(beta, ks)
        if cfg.mode in ("dcgs2", "dcgs2-native"):
            if cfg.mode == "dcgs2":
                def stop(b):
                    info.inner_residuals.append(b ** 2)
                    return b ** 2 < cfg.tol or (cfg.findiff and b ** 2 < 1e-8)
                k_used = dcgs2_cycle(ctx, op.matvec, Q, Hd, f, ks, giv, stop)
            else:   # the same cycle as ONE library call (nkv_gmres_dcgs2), bit-identical
                tol2 = max(cfg.tol, 1e-8) if cfg.findiff else cfg.tol
                k_used, res = gmres_cycle_native(ctx, op.matvec, Q, Hd, f, ks, beta, tol2)
                info.inner_residuals.extend(float(r) ** 2 for r in res)
            info.matvecs += k_used
            H[: k_used + 1, :k_used] = Hd.download()[: k_used + 1, :k_used]
            yvec[:k_used] = lapack.lstsq(H[: k_used + 1, :k_used], evec[: k_used + 1])
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
            continue
        col = _pinned_column(ks)
        for k in range(1, ks + 1):
            arnoldi_factorization(ctx, op, Q, Hd, k, k, f=f, mode=cfg.mode)
            info.matvecs += 1
            H[: k + 1, k - 1] = _download(col, Hd.t[k - 1, : k + 1])
            beta = giv.add_column(H[: k + 1, k - 1])        # ||e - H y|| without solving for y
            info.inner_residuals.append(beta ** 2)
            k_used = k
            if beta ** 2 < cfg.tol or (cfg.findiff and beta ** 2 < 1e-8):
                break
        yvec[:k_used] = lapack.lstsq(H[: k_used + 1, :k_used], evec[: k_used + 1])   # :255, the final system
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


def _pinned_column(ks: int) -> torch.Tensor:
    """Page-locked host buffer for the per-column H download: a direct DMA, no staging copy."""
    return torch.empty(ks + 1, dtype=torch.float64, pin_memory=True)


def _download(buf: torch.Tensor, src: torch.Tensor) -> np.ndarray:
    """src (a device vector) -> host, through the pinned ``buf``; waits for the stream."""
    n = src.numel()
    buf[:n].copy_(src, non_blocking=True)
    torch.cuda.current_stream(src.device).synchronize()
    return buf[:n].numpy()


def dcgs2_cycle(ctx: NekContext, apply, Q, Hd: HessenbergDev, f: NekVector, ks: int, giv: GivensResidual,
                stop) -> int:
    """The inner loop (newton_krylov.f90:250-276) on one continuous DCGS2 factorisation
    (``apply(x, y)``: y = A x; ``stop(residual)`` after every column).  Column k:
    matvec on the provisional Q[k-1] (Q[0] normalised), one DCGS2 step with the fused norm, then the
    residual estimate from H(0:k+1, k-1) — the step's once-projected coefficients and H(k, k-1) =
    ||next u||_W.  On exit the closing multi-dot of Q[k] against Q[0:k+1] corrects H's row k and
    fills in H(k, k-1) (nkv_dcgs2_coef without a second right-hand side); Q[k] itself is not needed
    by the solution update and is left unfinished.  Returns the number of columns k."""
    from .arnoldi import _dcgs2_step

    if ks > ctx.max_cols or Q.k < ks + 1 or Hd.k < ks:   # the closing multi-dot takes ks + 1 columns
        raise ValueError(f"GMRES k_dim={ks} needs max_cols >= {ks} (context has {ctx.max_cols}), "
                         f"a basis of {ks + 1} columns and H of {ks}")
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    nrm2 = ctx.scal[5:6]
    col = _pinned_column(ks)
    k_used = ks
    for k in range(1, ks + 1):
        apply(Q[k - 1], f)
        _dcgs2_step(ctx, Q, Hd, k, f, first=(k == 1), nrm2=nrm2)
        Hd.t[k - 1, k].copy_(torch.sqrt(nrm2[0]))            # provisional H(k, k-1), on the device
        beta = giv.add_column(_download(col, Hd.t[k - 1, : k + 1]))
        k_used = k
        if stop(beta):
            break
    m = k_used   # close: H row m corrected, H(m, m-1) from the fused norm (re-orthogonalised)
    h = ctx.hd[: m + 1]
    tf = _lib.NKV_TIME if ctx.time_in_dot else 0
    ctx.call("nkv_block_dot", w, Q.ptr, m + 1, Q.col_ptr(m), h.data_ptr(), ws, tf, st)
    ctx.comm.allreduce_(h)
    ctx.call_nl("nkv_dcgs2_coef", m, h.data_ptr(), None, nrm2.data_ptr(), Hd.t.data_ptr(), Hd.k + 1,
                ctx.coef.data_ptr(), ws, st)
    return k_used


def gmres_cycle_native(ctx: NekContext, apply, Q, Hd: HessenbergDev, f: NekVector, ks: int, beta: float,
                       tol2: float):
    """``dcgs2_cycle`` as ONE library call (``nkv_gmres_dcgs2``, include/nekkrylov.h): the operator
    and the all-reduce as callbacks, the per-column residuals returned.  Returns (k, residuals)."""
    import ctypes

    from .arnoldi import _allreduce_callback, _native_scratch

    if ks > ctx.max_cols or Q.k < ks + 1 or Hd.k < ks:   # ws holds the partials of ks + 1 columns
        raise ValueError(f"GMRES k_dim={ks} needs max_cols >= {ks} (context has {ctx.max_cols})")
    scratch = _native_scratch(ctx, ks)
    base, ld8, fptr = Q.ptr, 8 * ctx.layout.ld, f.ptr
    errors = []

    def matvec(_user, x, y, _stream):
        try:
            c, r = divmod((x or 0) - base, ld8)
            if r or not 0 <= c < Q.k or y != fptr:
                raise ValueError(f"nkv_gmres_dcgs2 matvec callback: x={x}, y={y} are not a basis column and f")
            apply(Q[c], f)
            return 0
        except BaseException as e:  # noqa: BLE001 — surfaced after the call returns
            errors.append(e)
            return 1

    mv_c = _lib.MATVEC_FN(matvec)
    ar_c = _allreduce_callback(ctx, scratch, errors)
    res = np.zeros(ks)
    k_out = ctypes.c_int(0)
    rc = ctx.lib.nkv_gmres_dcgs2(ctx._Lp, ctx.w.data_ptr(), Q.ptr, int(ks), float(beta), float(tol2),
                                 Hd.t.data_ptr(), Hd.k + 1, fptr, scratch.data_ptr(), ctx.ws.data_ptr(), mv_c, None,
                                 ar_c, None, res.ctypes.data, ctypes.addressof(k_out),
                                 _lib.NKV_TIME_DOT if ctx.time_in_dot else 0, ctx.stream)
    if errors:
        raise errors[0]
    _lib.check(rc, "nkv_gmres_dcgs2")
    k = int(k_out.value)
    return k, res[:k]
