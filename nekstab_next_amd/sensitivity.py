"""Direct/adjoint mode bi-orthogonalisation (the device part of nekStab's sensitivity tools).

Reference: ``biorthogonalize`` (core/sensitivity.f90:393-469): normalise the direct mode so that
||Re||^2 + ||Im||^2 = 1 — with ``opcmult``, i.e. the velocity components only (:429-430) — form
the complex W-inner product <adjoint, direct> from four real ``inner_product`` calls, and rescale
the adjoint mode (all fields incl. pressure and scalars; ``time`` untouched) so that it becomes 1.
The gradient post-processing (wave-maker, base-flow sensitivity) needs Nek5000's gradm1/dsavg and
is out of scope.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from .vector import NekContext, NekVector


def _scal_velocity(ctx: NekContext, x: NekVector, c: float) -> None:
    """opcmult: scale vx, vy, [vz] only (a sub-layout covering the first ldim fields)."""
    lay = ctx.layout
    sub = lay.c_struct()
    sub.n_wf = lay.ldim
    sub.n_p = 0
    sub.sp = 0
    _lib.check(ctx.lib.nkv_scal(ctypes.byref(sub), x.ptr, float(c), 0, ctx.stream), "nkv_scal(opcmult)")


def biorthogonalize(ctx: NekContext, dRe: NekVector, dIm: NekVector, aRe: NekVector, aIm: NekVector):
    """In place.  Returns the complex <adjoint, direct>_W before the rescaling."""
    ip = lambda p, q: ctx.dot(p, q, time=False)  # noqa: E731  (inner_product: no time component)
    alpha = ip(dRe, dRe)
    beta = ip(dIm, dIm)
    gamma = 1.0 / np.sqrt(alpha + beta)
    _scal_velocity(ctx, dRe, gamma)
    _scal_velocity(ctx, dIm, gamma)
    gamma = ip(aRe, dRe) + ip(aIm, dIm)   # real part
    delta = ip(aRe, dIm) - ip(aIm, dRe)   # imaginary part
    den = gamma ** 2 + delta ** 2
    wk1 = ctx.vector()
    wk1.copy_from(aRe, time=False)
    wk1.axpby(gamma / den, aIm, -delta / den)   # (gamma aRe - delta aIm)/den
    aIm.axpby(gamma / den, aRe, delta / den)    # (gamma aIm + delta aRe)/den
    aRe.copy_from(wk1, time=False)
    return complex(gamma, delta)
