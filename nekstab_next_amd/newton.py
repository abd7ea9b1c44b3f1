"""Newton–Krylov for fixed points of a time-stepper (nekStab's ``newton_krylov``, the caller of
config 4's GMRES).

Reference: ``core/newton_krylov.f90:1-166``.  Per Newton iteration i (at most 100, :44):

    f = F(q)                          nonlinear_forward_map (:97): a Nek5000 run, the caller's map
    residual = ||f||**2               k_norm (:102), written to residu_newton.dat (:109)
    exit if residual < tol            (:112; tol = max(param(21), param(22)), :37-41)
    ts_gmres(f, dq, 100, k_dim)       on the linearised map at q (:120): the legacy dispatcher's
                                      newton_linearized_map, uparam(1) = 2.x (matvec.f90:520-571)
    q = q - dq                        k_sub2 (:125), time included

and on convergence q is written as the base flow ``BF_<session>0.f00001`` (:155-164).  The
caller supplies ``nonlinear(q, f)`` (f <- F(q)) and ``linearized(q)`` (a LinearOperator: the
forward map of the linearisation about q; for uparam(1) = 2.1 wrap the period row with
:class:`~.operators.LegacyMatvec` yourself and pass ``mode=2.1``).  Out of scope, as in SURVEY §2:
the dynamic tolerance schedule (``ifdyntol``, ``spec_tole``, :93, :114-117, :383-435), the orbit
storage for UPOs (:82-91) and the Nek5000 output of intermediate iterates (``nwt``, ``ic_``)."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

from .config import GmresConfig
from .gmres import ts_gmres
from .operators import LegacyMatvec
from .vector import NekContext, NekVector, k_dot, k_sub2


def fortran_e(x: float, w: int, d: int) -> str:
    """Fortran ``Ew.d`` edit descriptor as gfortran writes it: a 0.ddddddd mantissa, then E and a
    signed two-digit exponent (three digits without the E above 99), right-justified in w
    columns; e.g. E15.7 of 1.234567e-3 is ``  0.1234567E-02``."""
    import math

    if x != x:
        return "NaN".rjust(w)
    if math.isinf(x):
        return ("-Infinity" if x < 0 else "Infinity").rjust(w)
    sign = "-" if (x < 0 or (x == 0 and math.copysign(1.0, x) < 0)) else ""
    a = abs(x)
    if a == 0.0:
        mant, exp = "0" * d, 0
    else:
        # round to d significant digits, then take the decimal exponent of the rounded value
        m, e = f"{a:.{d - 1}e}".split("e")
        exp = int(e) + 1
        mant = m.replace(".", "")
    ex = f"E{exp:+03d}" if abs(exp) <= 99 else f"{exp:+04d}"
    return f"{sign}0.{mant}{ex}".rjust(w)


@dataclass
class NewtonResult:
    converged: bool
    iterations: int
    residuals: list = field(default_factory=list)       # ||F(q)||^2 per iteration (residu_newton.dat)
    gmres: list = field(default_factory=list)           # the GmresInfo of every linear solve
    path: str | None = None


def newton_krylov(ctx: NekContext, nonlinear, linearized, q: NekVector, tol: float = 1e-9, maxiter: int = 100,
                  gmres: GmresConfig | None = None, mode: float = 2.0, fd: bool = False, outdir: str | None = None,
                  session: str = "nek") -> NewtonResult:
    """q is updated in place (the current estimate, as nekStab's ``q``).  ``gmres`` defaults to the
    reference's inner solve: maxiter 100 (:44), ``k_dim`` from the configuration, the same
    tolerance; ``fd`` selects the finite-difference exits (``iffindiff``).  ``mode`` is uparam(1)
    for the linearised map (2.0 / 2.1 / 2.2)."""
    gcfg = gmres or GmresConfig(maxiter=100, tol=tol, findiff=fd)
    res = NewtonResult(False, 0)
    f = ctx.vector()
    dq = ctx.vector()
    lines = []
    for i in range(1, maxiter + 1):
        nonlinear(q, f)
        residual = k_dot(f, f)
        res.residuals.append(residual)
        res.iterations = i
        lines.append(f"{i:6d}{fortran_e(residual, 15, 7)}\n")   # (I6,1E15.7), newton_krylov.f90:109
        if residual < tol:
            res.converged = True
            break
        op = linearized(q)
        if not isinstance(op, LegacyMatvec):
            op = LegacyMatvec(mode, op)
        res.gmres.append(ts_gmres(ctx, op, f, dq, gcfg))
        k_sub2(q, dq)
    if outdir is not None:
        from . import fld

        lay = ctx.layout
        # rank 0's residual history and every rank's base flow in one agreed block: a failure on
        # any rank is raised on every rank
        with fld.collective_output(ctx.comm):
            os.makedirs(outdir, exist_ok=True)
            if ctx.comm.rank == 0:
                with open(os.path.join(outdir, "residu_newton.dat"), "w") as fh:
                    fh.writelines(lines)
            if res.converged:
                res.path = os.path.join(outdir, fld.fld_name("BF_", session, lay.rank, 1))
                fld.write_fld(res.path, fld.fld_from_vector(lay, q.to_packed(), time=q.time, istep=res.iterations))
    return res
