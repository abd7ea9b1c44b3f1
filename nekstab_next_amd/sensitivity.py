"""Direct/adjoint sensitivity post-processing on the device (nekStab's core/sensitivity.f90).

``biorthogonalize`` (core/sensitivity.f90:393-469): normalise the direct mode so that
||Re||^2 + ||Im||^2 = 1 — with ``opcmult``, i.e. the velocity components only (:429-430) — form
the complex W-inner product <adjoint, direct> from four real ``inner_product`` calls, and rescale
the adjoint mode (all fields incl. pressure and scalars; ``time`` untouched) so that it becomes 1.

``wave_maker`` (core/sensitivity.f90:3-77, Giannetti & Luchini 2007): load the direct mode
``dRe/dIm<session>0.f00001`` and the adjoint mode ``aRe/aIm<session>0.f00002`` (velocity only:
``ifto = ifpo = .false.``, :40), bi-orthogonalise them, form the pointwise product
|u_d| |u_a| = sqrt(sum_c dRe_c^2 + dIm_c^2) sqrt(sum_c aRe_c^2 + aIm_c^2) (:69-71, one streaming
kernel, ``nkv_wavemaker``) and write it as the temperature field of ``wm_<session>0.f00001``
(:73-74).  It needs no derivatives.  The base-flow sensitivity (``bf_sensitivity``, :81-269) does
— Nek5000's ``gradm1``/``dsavg`` on the spectral-element mesh — and stays out of scope.

``ts_steady_force_sensitivity`` (:273-346): GMRES on the time-stepper form of the steady-force
sensitivity problem, ``ts_gmres`` over the legacy dispatcher's mode-4 map; the forced Nek5000 run
that recasts the right-hand side is the caller's.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import _lib
from .layout import NekLayout
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


def velocity_layout(lay: NekLayout) -> NekLayout:
    """The vector ``wave_maker`` works on: vx, vy, [vz] only — ``ifto = ifpo = .false.``
    (sensitivity.f90:40), so the dots (inner_product, eigensolvers.f90:46-53) and the copies and
    scalings (nopcopy/opcmult, nek_vectors.f90:279-298) skip pressure and temperature."""
    return NekLayout(lay.ldim, lay.lx1, lay.lx2, lay.nelgv, n_scalars=0, ifpo=False, rank=lay.rank, world=lay.world)


def wavemaker_field(ctx: NekContext, dRe: NekVector, dIm: NekVector, aRe: NekVector, aIm: NekVector,
                    out: torch.Tensor | None = None) -> torch.Tensor:
    """sensitivity.f90:69-71 on the device: one field segment (``sv`` doubles) holding
    sqrt(sum_c dRe_c^2 + dIm_c^2) * sqrt(sum_c aRe_c^2 + aIm_c^2) over the velocity components."""
    lay = ctx.layout
    if out is None:
        out = torch.empty(lay.sv, dtype=torch.float64, device=ctx.device)
    if out.numel() < lay.sv:
        raise ValueError(f"out holds {out.numel()} doubles, {lay.sv} needed")
    ctx.call("nkv_wavemaker", dRe.ptr, dIm.ptr, aRe.ptr, aIm.ptr, out.data_ptr(), lay.ldim, ctx.stream)
    return out


def wave_maker(ctx: NekContext, directory: str, session: str = "nek", d_num: int = 1, a_num: int = 2,
               outdir: str | None = None, coords: dict | None = None) -> dict:
    """``wave_maker`` (sensitivity.f90:3-77) on a velocity-only context (``velocity_layout``).

    Reads the direct mode ``dRe/dIm<session>0.f<d_num>`` and the adjoint mode
    ``aRe/aIm<session>0.f<a_num>`` (the reference's file numbers 1 and 2, :43-58; multi-file sets:
    each rank reads its own elements), bi-orthogonalises them on the device, forms the wave-maker
    field and writes it as the temperature of ``wm_<session><rank>.f00001`` in ``outdir``
    (default ``directory``).  As in the reference the header carries the time of the last file
    loaded (Nek5000's ``load_fld`` sets ``time``), no velocity (``ifvo = .false.``) and no
    pressure (``ifpo = .false.``); ``coords`` ({"x","y"[,"z"]} per local point) adds an X group.
    Returns the wave-maker (packed, this rank's points), <adjoint, direct>_W before the rescaling
    and the file written."""
    from . import fld

    lay = ctx.layout
    if lay.n_scalars or lay.n_p or lay.n_wf != lay.ldim:
        raise ValueError("wave_maker works on a velocity-only context (sensitivity.velocity_layout)")
    vecs, last = [], None
    for prefix, num in (("dRe", d_num), ("dIm", d_num), ("aRe", a_num), ("aIm", a_num)):
        files = fld.read_fld_set(directory, prefix, session, num)
        last = files[0]
        v = ctx.vector()
        v.from_packed(fld.vector_from_fld(lay, files))
        vecs.append(v)
    dRe, dIm, aRe, aIm = vecs
    ip = biorthogonalize(ctx, dRe, dIm, aRe, aIm)
    wm_dev = wavemaker_field(ctx, dRe, dIm, aRe, aIm)
    ctx.check_nan()
    wm = wm_dev[: lay.n_v].cpu().numpy()
    e0, e1 = lay.elem_range()
    f = fld.FldFile(lay.lx1, lay.lx1, lay.lx1 if lay.ldim == 3 else 1, lay.nelgv, last.time, last.istep, lay.rank,
                    lay.world, "", np.arange(e0 + 1, e1 + 1, dtype=np.int32), {})
    if coords:
        f.fields.update({k: np.asarray(v).reshape(lay.nelv, lay.pts_v) for k, v in coords.items()})
        f.rdcode += "X"
    f.fields["t"] = wm.reshape(lay.nelv, lay.pts_v)
    f.rdcode += "T"
    out = outdir or directory
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, fld.fld_name("wm_", session, lay.rank, 1))
    fld.write_fld(path, f)
    return dict(wavemaker=wm, inner_product=ip, path=path, vectors=(dRe, dIm, aRe, aIm))



def ts_steady_force_sensitivity(ctx: NekContext, op, directory: str, session: str = "nek", part: str = "r",
                                recast=None, k_dim: int = 100, tol: float = 1e-9, outdir: str | None = None,
                                mode: str | None = None) -> dict:
    """``ts_steady_force_sensitivity`` (sensitivity.f90:273-346, Marquet, Sipp & Jacquin 2008): the
    sensitivity of the flow to a steady force, by GMRES on the time-stepper form of the adjoint
    problem.  ``part`` "r" (uparam(1) = 4.41) reads the velocity of ``sr_<session>0.f00001``, "i"
    (4.42) that of ``si_<session>0.f00001`` (``opcopy``, :317-325; the other fields start at zero);
    ``recast(rhs)`` is ``initialize_rhs_ts_steady_force_sensitivity`` (:350-391), a forced adjoint
    Nek5000 integration that maps the forcing to the time-stepper right-hand side in place — the
    caller's (identity when omitted).  Then k_normalize (alpha), ``ts_gmres(rhs, sol, 10, k_dim)``
    on ``ts_force_sensitivity_map`` (q - exp(tL^T) q: :class:`~.operators.LegacyMatvec` mode 4.x
    over ``op.rmatvec``), sol *= alpha, and ``outpost`` of sol as ``fsr``/``fsi`` (Nek5000 names the
    file ``fsr<session>0.f00001``).  Returns the solution, alpha, the GMRES record and the file."""
    from . import fld
    from .config import GmresConfig
    from .gmres import ts_gmres
    from .operators import LegacyMatvec
    from .vector import k_cmult, k_normalize

    if part not in ("r", "i"):
        raise ValueError("part must be 'r' (uparam(1) = 4.41) or 'i' (4.42)")
    lay = ctx.layout
    files = fld.read_fld_set(directory, f"s{part}_", session, 1)
    if not files:
        raise FileNotFoundError(f"{fld.fld_name(f's{part}_', session, 0, 1)} not found in {directory}")
    full = fld.vector_from_fld(lay, files)
    host = np.zeros(lay.ld)
    for c in range(lay.ldim):   # opcopy: the velocity components only
        host[c * lay.sv: c * lay.sv + lay.n_v] = full[c * lay.sv: c * lay.sv + lay.n_v]
    rhs = ctx.vector().from_packed(host)
    if recast is not None:
        recast(rhs)
    alpha = k_normalize(rhs)
    sol = ctx.vector()
    cfg = GmresConfig(k_dim=k_dim, maxiter=10, tol=tol, **({"mode": mode} if mode else {}))
    info = ts_gmres(ctx, LegacyMatvec(4.41 if part == "r" else 4.42, op), rhs, sol, cfg)
    k_cmult(sol, alpha)
    ctx.check_nan()
    out = outdir or directory
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, fld.fld_name(f"fs{part}", session, lay.rank, 1))
    fld.write_fld(path, fld.fld_from_vector(lay, sol.to_packed(), time=files[0].time, istep=1))
    return dict(solution=sol, alpha=alpha, info=info, path=path)
