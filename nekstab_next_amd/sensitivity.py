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
(:73-74).  It needs no derivatives.

``bf_sensitivity`` (:81-269, Marquet et al.): the same four files and bi-orthogonalisation, then
Nek5000's ``gradm1`` of every velocity component of the four modes (``nkv_gradm1``: one element per
LDS tile, the geometric factors recomputed from the GLL coordinates on the fly, so a gradient reads
the coordinates and the field once and writes its ldim components), ``dsavg`` of each gradient
(direct-stiffness averaging: ``seeds.FaceAverage`` on one rank, the caller's gather-scatter on
several), the pointwise terms tr, ti, pr, pi and sr = tr + pr, si = ti + pi in one streaming kernel
(``nkv_bf_sensitivity``), written as the velocity of ``tr_``, ``ti_``, ``pr_``, ``pi_``, ``sr_``,
``si_<session>0.f00001`` — the files ``ts_steady_force_sensitivity`` reads back (sr/si).

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


def _load_modes(ctx: NekContext, directory: str, session: str, d_num: int, a_num: int, who: str):
    """The four load_fld calls (sensitivity.f90:43-60, 143-160): dRe/dIm<session>0.f<d_num> and
    aRe/aIm<session>0.f<a_num> into velocity-only device vectors (each rank its own elements).
    Returns the vectors and the last file read (its time goes into the outputs' headers)."""
    from . import fld

    lay = ctx.layout
    if lay.n_scalars or lay.n_p or lay.n_wf != lay.ldim:
        raise ValueError(f"{who} works on a velocity-only context (sensitivity.velocity_layout)")
    vecs, last = [], None
    for prefix, num in (("dRe", d_num), ("dIm", d_num), ("aRe", a_num), ("aIm", a_num)):
        files = fld.read_fld_set(directory, prefix, session, num, lay=lay, comm=ctx.comm)   # this rank's elements only
        last = files[0]
        v = ctx.vector()
        v.from_packed(fld.vector_from_fld(lay, files))
        vecs.append(v)
    return vecs, last


def _out_file(lay: NekLayout, last, coords: dict | None):
    """An empty field file of this rank's elements with the header of ``last`` (+ X if coords)."""
    from . import fld

    e0, e1 = lay.elem_range()
    f = fld.FldFile(lay.lx1, lay.lx1, lay.lx1 if lay.ldim == 3 else 1, lay.nelgv, last.time, last.istep, lay.rank,
                    lay.world, "", np.arange(e0 + 1, e1 + 1, dtype=np.int32), {})
    if coords:
        f.fields.update({k: np.asarray(v).reshape(lay.nelv, lay.pts_v) for k, v in coords.items()})
        f.rdcode += "X"
    return f


def gll_derivative(n: int) -> np.ndarray:
    """Nek5000's dxm1 (dgll): D[i, j] = P_N(z_i) / (P_N(z_j) (z_i - z_j)) for i != j,
    D[0, 0] = -N(N+1)/4, D[N, N] = N(N+1)/4, zero elsewhere on the diagonal (row-major, n x n).
    Nodes (Newton on P_N') and Legendre values in extended precision, then rounded: the matrix is
    within an ulp of the exact one (a gradient amplifies D's error by the element's aspect)."""
    from .fld import gll_points

    ld = np.longdouble
    N = n - 1

    def legendre(x):   # P_N and P_N' by the three-term recurrence
        p0, p1 = np.ones_like(x), x.copy()
        if N == 0:
            return p0, np.zeros_like(x)
        for k in range(2, N + 1):
            p0, p1 = p1, ((2 * k - 1) * x * p1 - (k - 1) * p0) / k
        return p1, N * (x * p1 - p0) / (x * x - 1)

    z = gll_points(n).astype(ld)
    inner = z[1:-1].copy()
    for _ in range(8):   # Newton on P_N'(z) = 0; P_N'' from Legendre's equation
        p, dp = legendre(inner)
        ddp = (2 * inner * dp - N * (N + 1) * p) / (1 - inner * inner)
        inner = inner - dp / ddp
    z[1:-1] = inner
    with np.errstate(divide="ignore", invalid="ignore"):   # P_N' at the end points is not used
        PN, _ = legendre(z)
    PN[0], PN[-1] = ld((-1) ** N), ld(1)
    D = np.zeros((n, n), dtype=ld)
    for i in range(n):
        for j in range(n):
            if i != j:
                D[i, j] = PN[i] / (PN[j] * (z[i] - z[j]))
    D[0, 0] = ld(-N * (N + 1)) / 4
    D[N, N] = ld(N * (N + 1)) / 4
    return D.astype(np.float64)


class Gradm1:
    """Nek5000's ``gradm1`` on this rank's elements (``nkv_gradm1``): holds the GLL derivative
    matrix and the coordinates {"x", "y"[, "z"]} (n_v each) on the device."""

    def __init__(self, ctx: NekContext, coords: dict):
        lay = ctx.layout
        self.ctx = ctx
        self.D = torch.as_tensor(gll_derivative(lay.lx1)).to(ctx.device)
        self.xyz = []
        for k in ("x", "y", "z")[: lay.ldim]:
            a = np.asarray(coords[k], dtype=np.float64)
            if a.size != lay.n_v:
                raise ValueError(f"coords[{k!r}]: {a.size} points, the layout has n_v={lay.n_v}")
            self.xyz.append(torch.as_tensor(a).to(ctx.device) if a.size else
                            torch.zeros(1, dtype=torch.float64, device=ctx.device))

    def __call__(self, u_ptr: int, grad_ptr: int, nfld: int = 1, u_stride: int = 0, g_stride: int | None = None) -> None:
        """Gradients of ``nfld`` fields (field f: n_v doubles at ``u_ptr + 8 f u_stride``) into
        ``grad_ptr + 8 (f ldim + d) g_stride`` (d = x, y[, z]; ``g_stride`` default n_v); the
        geometric factors are formed once for all of them."""
        lay = self.ctx.layout
        three = lay.ldim == 3
        self.ctx.call("nkv_gradm1", lay.lx1, lay.ldim, self.D.data_ptr(), self.xyz[0].data_ptr(),
                      self.xyz[1].data_ptr(), self.xyz[2].data_ptr() if three else None, u_ptr, int(nfld),
                      int(u_stride), grad_ptr, int(lay.n_v if g_stride is None else g_stride), self.ctx.stream)


class NormGrad:
    """Nek5000-side ``norm_grad`` (core/utils.f90:446-486) on the device: ``gradm1`` of vx, vy[, vz]
    of a state vector (one ``nkv_gradm1`` launch for the ldim components), then the sum of the
    ``glsc3(g, bm1s, g)`` of every gradient component — dudx, dudy, dvdx, dvdy, and in 3-D also
    dudz, dvdz, dwdx, dwdy, dwdz, i.e. all ldim x ldim of them (:476-485) — as ONE weighted dot over
    the ldim^2 gradient segments plus one all-reduce (glsc3's per-term all-reduces summed in
    another order: the same value to rounding).  No ``dsavg`` (commented out in the reference,
    :470-472).  The squared norm, no square root, as the reference compares it (with 1.1,
    eigensolvers.f90:592).  ``coords``: this rank's GLL coordinates."""

    def __init__(self, ctx: NekContext, coords: dict):
        from .layout import _roundup

        lay = ctx.layout
        self.ctx = ctx
        self.grad_op = coords if isinstance(coords, Gradm1) else Gradm1(ctx, coords)
        nf = lay.ldim * lay.ldim
        self.L = lay.c_struct()
        self.L.n_wf = nf
        self.L.n_p = 0
        self.L.sp = 0
        self.L.ld = _roundup(nf * lay.sv + 1, 4096)
        self.grad = torch.zeros(self.L.ld, dtype=torch.float64, device=ctx.device)
        self.out = torch.zeros(1, dtype=torch.float64, device=ctx.device)

    def __call__(self, v: NekVector) -> float:
        ctx, lay = self.ctx, self.ctx.layout
        gp = self.grad.data_ptr()
        self.grad_op(v.ptr, gp, nfld=lay.ldim, u_stride=lay.sv, g_stride=lay.sv)
        _lib.check(ctx.lib.nkv_dot(ctypes.byref(self.L), ctx.w.data_ptr(), gp, gp, self.out.data_ptr(),
                                   ctx.ws.data_ptr(), 0, ctx.stream), "nkv_dot(norm_grad)")
        ctx.comm.allreduce_(self.out)
        val = float(self.out.item())
        if val != val:
            ctx.check_nan()
        return val


BF_OUTPUTS = ("tr_", "ti_", "pr_", "pi_", "sr_", "si_")


def bf_sensitivity_fields(ctx: NekContext, dRe: NekVector, dIm: NekVector, aRe: NekVector, aIm: NekVector,
                          grad_op: Gradm1, face_average=None) -> tuple[torch.Tensor, torch.Tensor]:
    """sensitivity.f90:170-259 on bi-orthogonalised velocity-only vectors: gradm1 + dsavg of the
    4 x ldim components (``face_average(ptr)`` averages one field segment in place; None skips
    dsavg), then the pointwise terms.  Returns (out, grad): out holds 6 x ldim field segments
    [tr, ti, pr, pi, sr, si][component], grad 4 x ldim x ldim [mode][component][direction]."""
    lay = ctx.layout
    d, sv = lay.ldim, lay.sv
    grad = torch.zeros(4 * d * d * sv, dtype=torch.float64, device=ctx.device)
    out = torch.zeros(6 * d * sv, dtype=torch.float64, device=ctx.device)
    gp = grad.data_ptr()
    for md, v in enumerate((dRe, dIm, aRe, aIm)):   # one launch per mode: its d components together
        grad_op(v.ptr, gp + 8 * md * d * d * sv, nfld=d, u_stride=sv, g_stride=sv)
    if face_average is not None:
        for q in range(4 * d * d):
            face_average(gp + 8 * q * sv)
    ctx.call("nkv_bf_sensitivity", dRe.ptr, dIm.ptr, aRe.ptr, aIm.ptr, gp, out.data_ptr(), d, ctx.stream)
    return out, grad


def bf_sensitivity(ctx: NekContext, directory: str, coords: dict, session: str = "nek", d_num: int = 1,
                   a_num: int = 2, outdir: str | None = None, face_average="auto", write_coords: bool = False) -> dict:
    """``bf_sensitivity`` (sensitivity.f90:81-269) on a velocity-only context (``velocity_layout``):
    the four mode files (as ``wave_maker``), ``biorthogonalize`` (:163-166), gradm1 + dsavg
    (:170-199) and the terms (:202-235, 258-259) on the device, then ``outpost`` of the velocity of
    tr_, ti_, pr_, pi_, sr_, si_<session><rank>.f00001 into ``outdir`` (default ``directory``;
    ``ifto = ifpo = .false.``, :138; header time of the last file loaded).  ``coords``: this rank's
    GLL coordinates (``seeds.coords_from_fld``).  ``face_average``: "auto" = one-rank averaging
    over coincident points (``seeds.FaceAverage``; refused at world > 1), a callable ``f(ptr)``
    (the case's gather-scatter on one field segment), or None (no dsavg).  Returns the six
    outputs (this rank's points, [component] arrays), <adjoint, direct>_W and the files."""
    from . import fld

    lay = ctx.layout
    (dRe, dIm, aRe, aIm), last = _load_modes(ctx, directory, session, d_num, a_num, "bf_sensitivity")
    if isinstance(face_average, str):
        if face_average != "auto":
            raise ValueError("face_average: 'auto', a callable f(ptr) or None")
        from .seeds import FaceAverage

        face_average = FaceAverage(ctx, coords).apply
    ip = biorthogonalize(ctx, dRe, dIm, aRe, aIm)
    out, _ = bf_sensitivity_fields(ctx, dRe, dIm, aRe, aIm, Gradm1(ctx, coords), face_average)
    ctx.check_nan()
    host = out.view(6, lay.ldim, lay.sv)[:, :, : lay.n_v].cpu().numpy()
    dst = outdir or directory
    os.makedirs(dst, exist_ok=True)
    result, paths = {}, []
    with fld.collective_output(ctx.comm):   # outpost is collective: the sets are whole on return
        for t, prefix in enumerate(BF_OUTPUTS):
            f = _out_file(lay, last, coords if write_coords else None)
            for c, nm in enumerate(("vx", "vy", "vz")[: lay.ldim]):
                f.fields[nm] = host[t, c].reshape(lay.nelv, lay.pts_v)
            f.rdcode += "U"
            path = os.path.join(dst, fld.fld_name(prefix, session, lay.rank, 1))
            fld.write_fld(path, f)
            result[prefix.rstrip("_")] = [host[t, c].copy() for c in range(lay.ldim)]
            paths.append(path)
    return dict(fields=result, inner_product=ip, paths=paths, vectors=(dRe, dIm, aRe, aIm))


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
    (dRe, dIm, aRe, aIm), last = _load_modes(ctx, directory, session, d_num, a_num, "wave_maker")
    ip = biorthogonalize(ctx, dRe, dIm, aRe, aIm)
    wm_dev = wavemaker_field(ctx, dRe, dIm, aRe, aIm)
    ctx.check_nan()
    wm = wm_dev[: lay.n_v].cpu().numpy()
    f = _out_file(lay, last, coords)
    f.fields["t"] = wm.reshape(lay.nelv, lay.pts_v)
    f.rdcode += "T"
    out = outdir or directory
    os.makedirs(out, exist_ok=True)
    path = os.path.join(out, fld.fld_name("wm_", session, lay.rank, 1))
    with fld.collective_output(ctx.comm):
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
    files = fld.read_fld_set(directory, f"s{part}_", session, 1, lay=lay, comm=ctx.comm)
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
    with fld.collective_output(ctx.comm):
        fld.write_fld(path, fld.fld_from_vector(lay, sol.to_packed(), time=files[0].time, istep=1))
    return dict(solution=sol, alpha=alpha, info=info, path=path)
