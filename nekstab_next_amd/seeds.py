"""The reference's default seed vector of the eigensolvers: hash noise on the GLL mesh.

References: ``prepare_seed`` (core/linear_stab.f90:243-293; the LightKrylov drivers) and the seed
branches of ``krylov_schur`` (core/eigensolvers.f90:190-223), with ``ifseed_nois = .true.`` the
default (core/main.f90:29); the noise is ``op_add_noise`` / ``add_noise_scal`` (core/utils.f90:
258-359) over the hash ``mth_rand`` (:408-418).

* the pointwise noise runs on the device (``nkv_mth_rand_add``), one weighted field per launch, from
  this rank's GLL coordinates (``coords_from_fld``: the X block of any field file of the case);
* Nek5000's ``dssum`` + ``vmult`` (direct-stiffness averaging of the points elements share) and
  ``dsavg`` are restated on one rank from the coordinates (``FaceAverage``: groups of coincident
  points, averaged on the device by ``nkv_group_average``).  On several ranks the points on a
  shard boundary would need Nek's gather-scatter across ranks: pass your own ``face_average``;
* ``bcdirVC`` / ``bcdirSC`` (Dirichlet masks: walls, inflow) need the case's boundary conditions,
  which field files do not hold: pass them as ``mask`` (a vector of 0/1 multipliers, 1 elsewhere).

The hash is ``cos(1e3 sin(1e3 sin r))`` with r ~ 1e7: one unit in the last place of any ``sin`` moves
the result by up to ~1e-3, so the noise is reproducible only with the same math library rounding;
the tests compare the device against glibc's (the reference's gfortran libm) point by point.
"""
from __future__ import annotations

import numpy as np
import torch

from .vector import NekContext, NekVector

# op_add_noise's per-component constants (utils.f90:324-331)
NOISE_FC = ((3.0e4, -1.5e3, 0.5e5), (2.3e4, 2.3e3, -2.0e5), (2.0e4, 1.0e3, 1.0e5))
# add_noise_scal's constants for the temperature (linear_stab.f90:260; eigensolvers.f90:196)
SCAL_FC = (9.0e4, 3.0e3, 4.0e5)


def coords_from_fld(lay, files) -> dict:
    """This rank's GLL coordinates {"x", "y"[, "z"]} (n_v each, Nek point order) from field files
    holding a mesh block (rdcode with X), mapped by their element map like ``vector_from_fld``."""
    from . import fld

    if isinstance(files, fld.FldFile):
        files = [files]
    e0, e1 = lay.elem_range()
    names = ["x", "y", "z"][: lay.ldim]
    out = {nm: np.zeros(lay.n_v) for nm in names}
    seen = np.zeros(lay.nelv, dtype=bool)
    for f in files:
        if "x" not in f.fields:
            continue
        if f.nx != lay.lx1 or f.ldim != lay.ldim:
            raise ValueError(f"field file is lx1={f.nx} ldim={f.ldim}, layout lx1={lay.lx1} ldim={lay.ldim}")
        g = f.emap.astype(np.int64) - 1
        sel = np.nonzero((g >= e0) & (g < e1))[0]
        loc = g[sel] - e0
        for nm in names:
            out[nm].reshape(lay.nelv, lay.pts_v)[loc] = f.fields[nm][sel]
        seen[loc] = True
    if not np.all(seen):
        raise ValueError(f"{int(np.count_nonzero(~seen))} local elements have no coordinates in the files")
    return out


_SPLIT = 2e-4   # cells: coordinates this close across a rounding half-step are the same point


def coincident_groups(coords: dict, rel_tol: float = 1e-9) -> tuple[np.ndarray, np.ndarray]:
    """CSR groups (start, members) of the points with equal coordinates (to ``rel_tol`` of the mesh
    extent), groups of two or more only — the points Nek5000's gather-scatter sums over.

    Points are bucketed by their coordinates rounded to cells of ``rel_tol * extent``; two copies of
    one GLL point that differ by a few ulps can straddle a rounding half-step and land in
    neighbouring cells, so two points in neighbouring cells whose every coordinate agrees to
    2e-4 cells (both then lie within 2e-4 cells of that half-step) are one group as well.  Members of a group are in ascending point order (the summation order)."""
    xs = [np.asarray(coords[k], dtype=np.float64) for k in ("x", "y", "z") if k in coords]
    n = xs[0].size
    if n == 0:
        return np.zeros(1, np.int64), np.zeros(0, np.int64)
    ext = max(float(np.ptp(x)) for x in xs) or 1.0
    tol = rel_tol * ext
    sc = [x / tol for x in xs]
    keys = [np.round(v).astype(np.int64) for v in sc]
    order = np.lexsort(keys[::-1])
    ks = np.stack([k[order] for k in keys], axis=1)
    new = np.ones(n, dtype=bool)
    new[1:] = np.any(ks[1:] != ks[:-1], axis=1)
    gid = np.empty(n, dtype=np.int64)
    gid[order] = np.cumsum(new) - 1
    near = [np.abs(v - np.floor(v) - 0.5) <= _SPLIT for v in sc]
    flagged = np.flatnonzero(np.any(near, axis=0))
    if flagged.size:
        # a split pair lies within 1e-4 cells of the same half-step on either side: both flagged
        table = {}
        for p in flagged.tolist():
            table.setdefault(tuple(int(k[p]) for k in keys), []).append(p)
        parent = {}

        def find(g):
            while parent.get(g, g) != g:
                g = parent[g]
            return g

        for p in flagged.tolist():
            kp = [int(k[p]) for k in keys]
            cs = [c for c in range(len(xs)) if near[c][p]]
            for mask in range(1, 1 << len(cs)):
                alt = list(kp)
                for b, c in enumerate(cs):
                    if mask >> b & 1:
                        alt[c] += 1 if sc[c][p] > kp[c] else -1
                for q in table.get(tuple(alt), ()):
                    if all(abs(x[p] - x[q]) <= _SPLIT * tol for x in xs):
                        a, b2 = find(int(gid[p])), find(int(gid[q]))
                        if a != b2:
                            parent[max(a, b2)] = min(a, b2)
        if parent:
            roots = {g: find(g) for g in list(parent)}
            moved = np.array(list(roots), dtype=np.int64)
            lut = np.arange(int(gid.max()) + 1, dtype=np.int64)
            lut[moved] = np.array([roots[g] for g in moved.tolist()], dtype=np.int64)
            gid = lut[gid]
    counts = np.bincount(gid)
    idx = np.flatnonzero(counts[gid] > 1)                 # ascending point order
    members = idx[np.lexsort((idx, gid[idx]))].astype(np.int64)
    g_multi = gid[members]
    starts = np.flatnonzero(np.r_[True, g_multi[1:] != g_multi[:-1]]) if members.size else np.zeros(0, np.int64)
    return np.r_[starts, members.size].astype(np.int64), members


class FaceAverage:
    """``dssum`` then ``vmult`` (and ``dsavg``, the same again) on one rank: each group of coincident
    points gets its mean (``nkv_group_average``)."""

    def __init__(self, ctx: NekContext, coords: dict, rel_tol: float = 1e-9):
        if ctx.comm.world > 1:
            raise ValueError("FaceAverage averages one rank's points only; at world > 1 pass the case's own "
                             "gather-scatter as face_average (shard-boundary points are shared across ranks)")
        start, members = coincident_groups(coords, rel_tol)
        self.ctx = ctx
        self.n_groups = start.size - 1
        self.start = torch.as_tensor(start).to(ctx.device)
        self.members = torch.as_tensor(members if members.size else np.zeros(1, np.int64)).to(ctx.device)

    def apply(self, ptr: int) -> None:
        """Average one field segment (n_v points at device address ``ptr``) in place."""
        self.ctx.call_nl("nkv_group_average", self.n_groups, self.start.data_ptr(), self.members.data_ptr(), ptr,
                         self.ctx.stream)

    def __call__(self, vec: NekVector, fields) -> None:
        ctx, lay = self.ctx, self.ctx.layout
        for f in fields:
            ctx.call_nl("nkv_group_average", self.n_groups, self.start.data_ptr(), self.members.data_ptr(),
                        vec.ptr + 8 * f * lay.sv, ctx.stream)


def _coord_tensors(ctx: NekContext, coords: dict):
    lay = ctx.layout
    out = []
    for k in ("x", "y", "z")[: lay.ldim]:
        a = np.asarray(coords[k], dtype=np.float64)
        if a.size != lay.n_v:
            raise ValueError(f"coords[{k!r}]: {a.size} points, the layout has n_v={lay.n_v}")
        out.append(torch.as_tensor(a).to(ctx.device) if lay.n_v else torch.zeros(2, dtype=torch.float64,
                                                                                 device=ctx.device))
    return out


def mth_rand_add(ctx: NekContext, vec: NekVector, field: int, coords: dict, fc) -> None:
    """vec's weighted field ``field`` += mth_rand(il, jl, kl, ieg, xl, fc) at every point
    (utils.f90:408-418; ieg from this rank's element range)."""
    lay = ctx.layout
    if not 0 <= field < lay.n_wf:
        raise ValueError(f"field {field} outside 0..{lay.n_wf - 1}")
    ct = _coord_tensors(ctx, coords)
    lz1 = lay.lx1 if lay.ldim == 3 else 1
    ctx.call("nkv_mth_rand_add", lay.lx1, lay.lx1, lz1, lay.elem_range()[0], ct[0].data_ptr(), ct[1].data_ptr(),
             ct[2].data_ptr() if lay.ldim == 3 else None, float(fc[0]), float(fc[1]), float(fc[2]),
             vec.ptr + 8 * field * lay.sv, ctx.stream)


def _finish(ctx: NekContext, vec: NekVector, fields, face_average, mask) -> None:
    if face_average is not None:
        face_average(vec, fields)   # opdssum + opcolv(vmult)   (utils.f90:339-340; add_noise_scal :284-285)
        face_average(vec, fields)   # dsavg                      (:342-344; :286)
    if mask is not None:            # bcdirVC / bcdirSC          (:347; :287)
        ctx.call("nkv_op_diag", mask.ptr, vec.ptr, vec.ptr, 1.0, ctx.stream)


def op_add_noise(ctx: NekContext, vec: NekVector, coords: dict, face_average=None, mask: NekVector | None = None):
    """vx, vy[, vz] += op_add_noise's hash noise (utils.f90:297-359)."""
    lay = ctx.layout
    for c in range(lay.ldim):
        mth_rand_add(ctx, vec, c, coords, NOISE_FC[c])
    _finish(ctx, vec, range(lay.ldim), face_average, mask)


def add_noise_scal(ctx: NekContext, vec: NekVector, field: int, coords: dict, fc, face_average=None,
                   mask: NekVector | None = None):
    """One scalar field += add_noise_scal's hash noise (utils.f90:258-295)."""
    mth_rand_add(ctx, vec, field, coords, fc)
    _finish(ctx, vec, (field,), face_average, mask)


def noise_seed(ctx: NekContext, coords: dict, ifto: bool | None = None, ifpsco=(), face_average=None,
               mask: NekVector | None = None) -> NekVector:
    """The noise branch of ``prepare_seed`` (linear_stab.f90:254-265): zero, op_add_noise on the
    velocity, add_noise_scal on t(:,1) if ``ifto`` (default: the layout has a scalar), and for every
    passive scalar m = 2..ldimt with ``ifpsco(m-1)`` another add_noise_scal with (90 m, 300 m, 40 m)
    — into t(:,1) again, as the reference writes it (:262).  Not normalised: pass the result to
    ``krylov_schur.prepare_seed`` / ``seed_mode="normalize"`` (:287-291), or as the ``"noise"``
    seed of the in-tree solver (eigensolvers.f90:192-203: k_normalize, one matvec)."""
    lay = ctx.layout
    if ifto is None:
        ifto = lay.n_scalars > 0
    if (ifto or any(ifpsco)) and lay.n_scalars == 0:
        raise ValueError("ifto / ifpsco need a scalar field in the layout")
    seed = ctx.vector()
    seed.zero()
    op_add_noise(ctx, seed, coords, face_average, mask)
    t1 = lay.ldim
    if ifto:
        add_noise_scal(ctx, seed, t1, coords, SCAL_FC, face_average, mask)
    for m, on in enumerate(ifpsco, start=2):
        if on:
            add_noise_scal(ctx, seed, t1, coords, (9.0e1 * m, 3.0e2 * m, 4.0e1 * m), face_average, mask)
    return seed


def symmetric_seed(ctx: NekContext, coords: dict, base: NekVector | None = None, bm1=None) -> NekVector:
    """``add_symmetric_seed(wrk%vx, wrk%vy, wrk%vz, wrk%t(:,1))`` (utils.f90:361-406, called at
    eigensolvers.f90:205-208 when ``ifseed_symm``): on a copy of ``base`` (zero by default) vx, vz
    and t(:,1) become cos(alpha z) sin(2 pi y), -(2 pi / alpha) cos(alpha z) cos(2 pi y) and
    cos(alpha z) cos(2 pi y) with alpha = 2 pi / (zmax - zmin) over all ranks; vy keeps the base's
    values (the reference never writes qy); then vx, vy, vz and t(:,1) are scaled by
    1e-6 / (0.5 sum_c glsc3(q_c, bm1, q_c)) over the velocity components.  ``bm1``: the mass matrix
    (this rank's n_v points) when the context's dot weights are not bm1 — with a sponge the
    context holds bm1s, zero in the sponge (forcing.f90:101-104), while add_symmetric_seed
    weights with bm1 (utils.f90:394-396); default: the context's weights.
    The in-tree solver takes the result as Q(1) unnormalised (``seed_mode="symm"``).  3-D with a
    scalar field only (in 2-D the reference divides by zmax - zmin = 0)."""
    lay = ctx.layout
    if lay.ldim != 3 or lay.n_scalars < 1:
        raise ValueError("add_symmetric_seed needs a 3-D layout with a scalar field (qp = t(:,1))")
    _, y, z = _coord_tensors(ctx, coords)
    zl = np.asarray(coords["z"], dtype=np.float64)
    zmin = ctx.comm.min_scalar(float(zl.min()) if zl.size else np.inf, device=ctx.device)
    zmax = ctx.comm.max_scalar(float(zl.max()) if zl.size else -np.inf, device=ctx.device)
    alpha = 2.0 * np.pi / (zmax - zmin)
    seed = ctx.vector()
    if base is None:
        seed.zero()
    else:
        seed.copy_from(base)
    sv = lay.sv
    ctx.call("nkv_symmetric_seed", y.data_ptr(), z.data_ptr(), float(alpha), seed.ptr, seed.ptr + 8 * 2 * sv,
             seed.ptr + 8 * 3 * sv, ctx.stream)
    vel = ctx.vector()
    vel.copy_from(seed)
    vel.storage[3 * sv:lay.n_wf * sv].zero_()       # amp over vx, vy, vz only (glsc3 x 3, :394-396)
    if bm1 is None:
        amp = ctx.dot(vel, vel, time=False)
    else:
        b = np.asarray(bm1, dtype=np.float64).ravel()
        if b.size != lay.n_v:   # as NekContext's weights: exactly this shard's points (a global bm1
            # passed on rank r > 0 would silently weight with rank 0's points)
            raise ValueError(f"bm1 holds {b.size} points, this rank's shard has n_v={lay.n_v}")
        wb = torch.zeros(max(lay.sv, 4096), dtype=torch.float64, device=ctx.device)
        wb[: lay.n_v] = torch.as_tensor(b[: lay.n_v])
        out = ctx.scal[1:2]
        ctx.call("nkv_dot", wb.data_ptr(), vel.ptr, vel.ptr, out.data_ptr(), ctx.ws.data_ptr(), 0, ctx.stream)
        amp = float(ctx.comm.allreduce_(out).item())
        ctx.check_nan()   # the dot's NaN flag, as ctx.dot surfaces it (nek_vectors.f90:108-111)
    amp = 1e-6 / (0.50 * amp)
    for c in (0, 1, 2, 3):                          # opcmult(qx, qy, qz, amp); cmult(qp, amp)
        seg = seed.storage[c * sv:(c + 1) * sv]
        seg.mul_(amp)
    return seed
