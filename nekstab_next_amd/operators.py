"""Linear operators: the matvec boundary of the Krylov path.

Reference: LightKrylov ``abstract_linop`` extended by ``exponential_prop`` with type-bound
``matvec(self, vec_in, vec_out)`` / ``rmatvec`` (core/linear_operators.f90:17-23, 39-103) and the
legacy ``matvec(f, q)`` dispatcher (core/matvec.f90:56-146).  In nekStab the operator body is a
Nek5000 time integration (out of scope here); the operators below are the synthetic, exactly
known ones SURVEY.md §8(d) defines for every BASELINE config, each a device kernel or a
composition of the library's device ops.  Any Python object with ``matvec(x, y)`` (and optionally
``rmatvec``) over :class:`~nekstab_next_amd.vector.NekVector` plugs into the solvers.
"""
from __future__ import annotations

import numpy as np
import torch

from ._lib import NKV_TIME
from .vector import NekContext, NekVector


class LinearOperator:
    """y <- A x (matvec) and y <- A^T x under the W inner product (rmatvec)."""

    def matvec(self, x: NekVector, y: NekVector) -> None:  # pragma: no cover - interface
        raise NotImplementedError

    def rmatvec(self, x: NekVector, y: NekVector) -> None:  # pragma: no cover - interface
        raise NotImplementedError


def _dev(ctx: NekContext, a: np.ndarray) -> torch.Tensor:
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(ctx.device)


class DiagOperator(LinearOperator):
    """y = D x with D diagonal over every stored row (self-adjoint under W).

    ``diag`` is a padded host/device vector of length ``layout.ld`` (this rank's shard); padding
    rows are ignored.  ``time_scale`` multiplies the scalar time component.
    """

    def __init__(self, ctx: NekContext, diag, time_scale: float = 0.0):
        self.ctx = ctx
        d = diag if isinstance(diag, torch.Tensor) else _dev(ctx, diag)
        if d.numel() != ctx.layout.ld:
            raise ValueError("diag must have layout.ld entries")
        self.d = d.to(ctx.device, torch.float64).contiguous()
        self.time_scale = float(time_scale)

    def matvec(self, x: NekVector, y: NekVector) -> None:
        self.ctx.call("nkv_op_diag", self.d.data_ptr(), x.ptr, y.ptr, self.time_scale, self.ctx.stream)

    rmatvec = matvec


class Rot2Operator(LinearOperator):
    """Per grid point, (vx, vy) -> r R(theta) (vx, vy); other weighted fields and pressure are
    multiplied by ``d_rest``.  W-normal (the 2x2 blocks share one weight), eigenvalues
    r e^{±i theta}: conjugate pairs for the complex handling of ``eig`` / ``select_eigenvalues``
    (SURVEY.md §8(d) config 2).  ``rmatvec`` applies r R(-theta)."""

    def __init__(self, ctx: NekContext, c, s, d_rest=None):
        self.ctx = ctx
        lay = ctx.layout
        self.c = c if isinstance(c, torch.Tensor) else _dev(ctx, c)
        self.s = s if isinstance(s, torch.Tensor) else _dev(ctx, s)
        if self.c.numel() != lay.sv or self.s.numel() != lay.sv:
            raise ValueError("c, s must have layout.sv entries")
        self.d_rest = None
        if d_rest is not None:
            self.d_rest = d_rest if isinstance(d_rest, torch.Tensor) else _dev(ctx, d_rest)
            if self.d_rest.numel() != lay.ld:
                raise ValueError("d_rest must have layout.ld entries")

    def _apply(self, x, y, transpose):
        dr = self.d_rest.data_ptr() if self.d_rest is not None else None
        self.ctx.call("nkv_op_rot2", self.c.data_ptr(), self.s.data_ptr(), dr, x.ptr, y.ptr, int(transpose),
                      self.ctx.stream)

    def matvec(self, x: NekVector, y: NekVector) -> None:
        self._apply(x, y, False)

    def rmatvec(self, x: NekVector, y: NekVector) -> None:
        self._apply(x, y, True)


class ShiftedOperator(LinearOperator):
    """y = A x + shift * x  (e.g. the Newton–Krylov Jacobian-minus-identity J = D - I, config 4;
    the reference's newton_linearized_map returns Phi'(q) - q, core/matvec.f90:520-571)."""

    def __init__(self, base: LinearOperator, shift: float):
        self.base, self.shift = base, float(shift)

    def matvec(self, x: NekVector, y: NekVector) -> None:
        self.base.matvec(x, y)
        y.axpby(1.0, x, self.shift)

    def rmatvec(self, x: NekVector, y: NekVector) -> None:
        self.base.rmatvec(x, y)
        y.axpby(1.0, x, self.shift)


class RankTwoPerturbed(LinearOperator):
    """A x = D x + sigma * (u <v, x>_W + v' <u', x>_W): a base operator D (config 5: diagonal) plus
    a rank-2 non-normal term, so direct and adjoint eigenvectors differ.
    The adjoint under W is A^T x = D^T x + sigma * (v <u, x>_W + u' <v', x>_W)."""

    def __init__(self, diag_op: LinearOperator, u: NekVector, v: NekVector, u2: NekVector, v2: NekVector,
                 sigma: float):
        self.d, self.u, self.v, self.u2, self.v2, self.sigma = diag_op, u, v, u2, v2, float(sigma)

    def matvec(self, x: NekVector, y: NekVector) -> None:
        self.d.matvec(x, y)
        a = x.ctx.dot(self.v, x, time=False)
        b = x.ctx.dot(self.u2, x, time=False)
        y.axpby(1.0, self.u, self.sigma * a)
        y.axpby(1.0, self.v2, self.sigma * b)

    def rmatvec(self, x: NekVector, y: NekVector) -> None:
        self.d.rmatvec(x, y)
        a = x.ctx.dot(self.u, x, time=False)
        b = x.ctx.dot(self.v2, x, time=False)
        y.axpby(1.0, self.v, self.sigma * a)
        y.axpby(1.0, self.u2, self.sigma * b)


class CallableOperator(LinearOperator):
    """Wrap plain callables ``f(x, y)`` (e.g. a user's time-stepper driving the GPU state)."""

    def __init__(self, matvec, rmatvec=None):
        self._mv, self._rmv = matvec, rmatvec

    def matvec(self, x, y):
        self._mv(x, y)

    def rmatvec(self, x, y):
        if self._rmv is None:
            raise NotImplementedError("operator has no adjoint")
        self._rmv(x, y)


class LegacyMatvec(LinearOperator):
    """The legacy ``matvec(f, q)`` dispatcher (core/matvec.f90:56-146): ``uparam(1) = mode``
    selects the map applied to q, in the reference's order and with its ``k_*`` time handling
    (k_sub2 / k_cmult / k_add2 update ``time``, krylov_subspace.f90:94-127).  ``op.matvec`` is the
    forward linearised map, ``op.rmatvec`` the adjoint map; ``fd_op.matvec`` (optional) the
    finite-difference forward map used when ``iffindiff`` (:113-118, :536-541).

    ============  =======  =======================================================================
    mode          evop     f =
    ============  =======  =======================================================================
    [3.0, 3.2)    ``d``    forward map (or FD map) of q                                   (:111-119)
    [3.2, 3.3)    ``a``    adjoint map of q                                               (:122-125)
    [3.3, 3.4)    ``p``    adjoint(forward(q)), transient_growth_map                 (:128-131, :478-495)
    4.x           —        -(adjoint(q) - q), ts_force_sensitivity_map               (:134-136, :499-516)
    2.x           ``n``    forward(q) - q, newton_linearized_map                     (:139-143, :520-571)
    ============  =======  =======================================================================

    Mode 2.1 (Newton for a periodic orbit, :550-563) borders the map with the period row:
    f += b_fc * q%time and f%time = k_dot(b_ic, q); other 2.x modes set f%time = 0.  ``b_fc`` /
    ``b_ic`` are the time derivatives compute_bvec produces (:575-613, one Nek step — out of scope
    here, so the caller supplies them); they are copied with time = 0 as compute_bvec leaves them
    (:610).  The reference silently leaves f untouched for a mode that selects nothing; here that
    is refused at construction.  No host synchronisation: q%time and the period dot stay on the
    device."""

    def __init__(self, mode: float, op: LinearOperator, fd_op: LinearOperator | None = None,
                 b_fc: NekVector | None = None, b_ic: NekVector | None = None):
        mode = float(mode)
        fl = int(np.floor(mode))
        if 3.0 <= mode < 3.2:
            self.evop = "d"
        elif 3.2 <= mode < 3.3:
            self.evop = "a"
        elif 3.3 <= mode < 3.4:
            self.evop = "p"
        elif fl == 4:
            self.evop = None
        elif fl == 2:
            self.evop = "n"
        else:
            raise ValueError(f"uparam(1)={mode} selects no map (core/matvec.f90:110-143)")
        self.mode, self.op, self.fd_op = mode, op, fd_op
        self.upo = mode == 2.1
        self._wrk = None
        self._t = None
        if self.upo:
            if b_fc is None or b_ic is None:
                raise ValueError("uparam(1)=2.1 needs b_fc and b_ic (compute_bvec, core/matvec.f90:555-560)")
            ctx = b_fc.ctx
            self.b_fc, self.b_ic = ctx.vector(), ctx.vector()
            for dst, src in ((self.b_fc, b_fc), (self.b_ic, b_ic)):
                dst.copy_from(src, time=False)
            self._t = torch.zeros(1, dtype=torch.float64, device=ctx.device)

    def _forward(self, q: NekVector, f: NekVector) -> None:
        (self.fd_op if self.fd_op is not None else self.op).matvec(q, f)

    def matvec(self, q: NekVector, f: NekVector) -> None:
        from .vector import k_cmult, k_sub2

        ctx = q.ctx
        m, fl = self.mode, int(np.floor(self.mode))
        if 3.0 <= m < 3.2:
            self._forward(q, f)
        elif 3.2 <= m < 3.3:
            self.op.rmatvec(q, f)
        elif 3.3 <= m < 3.4:
            if self._wrk is None:
                self._wrk = ctx.vector()
            self.op.matvec(q, self._wrk)
            self.op.rmatvec(self._wrk, f)
        elif fl == 4:
            self.op.rmatvec(q, f)
            k_sub2(f, q)
            k_cmult(f, -1.0)
        else:
            self._forward(q, f)
            k_sub2(f, q)
            lay = ctx.layout
            tslot = f.storage[lay.time_offset:lay.time_offset + 1]
            if self.upo:
                q_time = q.ptr + 8 * lay.time_offset
                ctx.call("nkv_axpy_dev", f.ptr, q_time, 1.0, self.b_fc.ptr, NKV_TIME, ctx.stream)
                ctx.dot_dev(self.b_ic, q, self._t, time=ctx.time_in_dot)
                tslot.copy_(self._t)
            else:
                tslot.zero_()


class ComplexDiagOperator(LinearOperator):
    """y = C x, C complex diagonal, on complex vectors stored as re/im pair vectors
    (:class:`~nekstab_next_amd.layout.PairLayout`); ``rmatvec`` applies conj(C) — the adjoint under
    the cmplx dot re.re + im.im.  ``cr``/``ci`` are padded pair-layout vectors read at the re rows
    (:func:`~nekstab_next_amd.synthetic.resolvent_diag`).  The synthetic stand-in for nekStab's
    ``resolvent_op`` (core/linear_operators.f90:309-431), whose body is a forced Nek5000 run."""

    def __init__(self, ctx: NekContext, cr, ci):
        from .layout import PairLayout

        if not isinstance(ctx.layout, PairLayout):
            raise ValueError("ComplexDiagOperator needs a NekContext on a PairLayout")
        self.ctx = ctx
        self.cr = cr if isinstance(cr, torch.Tensor) else _dev(ctx, cr)
        self.ci = ci if isinstance(ci, torch.Tensor) else _dev(ctx, ci)
        if self.cr.numel() != ctx.layout.ld or self.ci.numel() != ctx.layout.ld:
            raise ValueError("cr, ci must have layout.ld entries")

    def matvec(self, x: NekVector, y: NekVector) -> None:
        self.ctx.call("nkv_op_cdiag", self.cr.data_ptr(), self.ci.data_ptr(), x.ptr, y.ptr, 0, self.ctx.stream)

    def rmatvec(self, x: NekVector, y: NekVector) -> None:
        self.ctx.call("nkv_op_cdiag", self.cr.data_ptr(), self.ci.data_ptr(), x.ptr, y.ptr, 1, self.ctx.stream)
