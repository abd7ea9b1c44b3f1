"""The reference's default seed on the device (ifseed_nois = .true., main.f90:29; prepare_seed's
noise branch, linear_stab.f90:254-265): nkv_mth_rand_add (mth_rand, utils.f90:408-418, with
correctly rounded sin/cos) and nkv_group_average (dssum + vmult on one rank) against the oracle.

Parity: the hash cos(1e3 sin(1e3 sin r)) moves by up to ~1e-3 for one ulp of any sin, so it is
pinned to the formula with correctly rounded sin/cos (mpmath at 160 bits) at EVERY point, and to
glibc (the reference's gfortran libm, which misrounds ~0.1 % of near-midpoint arguments) at >= 98 %
of the points."""
import os

import numpy as np
import pytest
import torch

import oracle as orc
from seed_helpers import box_mesh_coords

from nekstab_next_amd import seeds
from nekstab_next_amd._lib import NkvError
from nekstab_next_amd.layout import NekLayout, cylinder_layout
from nekstab_next_amd.vector import NekContext

GOLD = os.path.join(os.path.dirname(__file__), "golden")
pytestmark = pytest.mark.gpu


def _field(lay, v, c):
    return v.to_packed()[c * lay.sv: c * lay.sv + lay.n_v]


def _pinned_noise(lay, co, c_fc, got, e_first=0):
    """The oracle's pointwise noise for one field, glibc at the points where the device agrees with
    it and correctly rounded (checked against the device) where it does not."""
    nz = lay.lx1 if lay.ldim == 3 else 1
    z = co.get("z") if lay.ldim == 3 else None
    ref = orc.noise_field(lay.lx1, lay.lx1, nz, e_first, co["x"], co["y"], z, c_fc)
    miss = np.flatnonzero(ref != got)
    assert miss.size <= 0.02 * got.size, (miss.size, got.size)
    cr = orc.noise_field(lay.lx1, lay.lx1, nz, e_first, co["x"], co["y"], z, c_fc, kind="cr", points=miss)
    np.testing.assert_array_equal(got[miss], cr[miss])
    ref[miss] = cr[miss]
    return ref, miss.size / got.size


def _cases():
    d = np.load(os.path.join(GOLD, "cyl_mesh_xy.npz"))
    lay3 = NekLayout(ldim=3, lx1=6, lx2=4, nelgv=3 * 2 * 4, n_scalars=1)
    return {"cyl": (cylinder_layout(1996), {"x": d["x"], "y": d["y"]}),
            "box3d": (lay3, box_mesh_coords(lay3, (3, 2, 4)))}


@pytest.mark.parametrize("case", ["cyl", "box3d"])
def test_mth_rand_add_vs_oracle(gpu, case):
    """Pointwise noise of every velocity component (op_add_noise's fc, utils.f90:324-331) and of the
    temperature (add_noise_scal's, linear_stab.f90:260): the device equals the formula with correctly
    rounded libm at every point; the other fields stay untouched."""
    lay, co = _cases()[case]
    ctx = NekContext(lay, max_cols=4)
    for c in range(lay.n_wf):
        fc = seeds.NOISE_FC[c] if c < lay.ldim else seeds.SCAL_FC
        v = ctx.vector()
        v.fill_hash(3)
        before = v.to_packed()
        seeds.mth_rand_add(ctx, v, c, co, fc)
        after = v.to_packed()
        noise = after[c * lay.sv: c * lay.sv + lay.n_v] - before[c * lay.sv: c * lay.sv + lay.n_v]
        v0 = ctx.vector()
        v0.zero()
        seeds.mth_rand_add(ctx, v0, c, co, fc)
        got = _field(lay, v0, c)
        _, frac = _pinned_noise(lay, co, fc, got)
        print(f"{case} field {c}: {100 * (1 - frac):.3f} % of the points equal glibc's bit for bit")
        np.testing.assert_allclose(noise, got, rtol=0, atol=1e-15 * 8)
        mask = np.ones(after.size, bool)
        mask[c * lay.sv: c * lay.sv + lay.n_v] = False
        np.testing.assert_array_equal(after[mask], before[mask])


@pytest.mark.parametrize("case", ["cyl", "box3d"])
def test_noise_seed_vs_oracle(gpu, case):
    """noise_seed = prepare_seed's noise branch: zero; op_add_noise (dssum/vmult + dsavg by
    coincident points); add_noise_scal into t(:,1) (ifto), and for ifpsco(1) once more into t(:,1)
    with (180, 600, 80) as the reference writes it (linear_stab.f90:262); the Dirichlet mask last.
    Bit for bit against the oracle pipeline on the pinned pointwise noise."""
    lay, co = _cases()[case]
    ctx = NekContext(lay, max_cols=4)
    fa = seeds.FaceAverage(ctx, co)
    mask = ctx.vector()
    mvec = np.ones(lay.ld)
    rng = np.random.default_rng(2)
    for c in range(lay.n_wf):
        mvec[c * lay.sv: c * lay.sv + lay.n_v] = (rng.random(lay.n_v) > 0.1).astype(float)
    mask.from_packed(mvec)
    ps = (True,) if lay.n_scalars else ()
    seed = seeds.noise_seed(ctx, co, face_average=fa, mask=mask, ifpsco=ps)
    out = seed.to_packed()
    # oracle: the same sequence on the pinned pointwise noise of each add
    for c in range(lay.ldim):
        raw0 = ctx.vector()
        raw0.zero()
        seeds.mth_rand_add(ctx, raw0, c, co, seeds.NOISE_FC[c])
        q, _ = _pinned_noise(lay, co, seeds.NOISE_FC[c], _field(lay, raw0, c))
        q = orc.coincident_average(orc.coincident_average(q, co), co)
        q = q * mvec[c * lay.sv: c * lay.sv + lay.n_v]
        np.testing.assert_array_equal(out[c * lay.sv: c * lay.sv + lay.n_v], q)
    if lay.n_scalars:
        t1 = lay.ldim
        q = np.zeros(lay.n_v)
        for fc in (seeds.SCAL_FC, (180.0, 600.0, 80.0)):
            raw0 = ctx.vector()
            raw0.zero()
            seeds.mth_rand_add(ctx, raw0, t1, co, fc)
            n, _ = _pinned_noise(lay, co, fc, _field(lay, raw0, t1))
            q = orc.coincident_average(orc.coincident_average(q + n, co), co)
            q = q * mvec[t1 * lay.sv: t1 * lay.sv + lay.n_v]
        np.testing.assert_array_equal(out[t1 * lay.sv: t1 * lay.sv + lay.n_v], q)
    assert np.all(out[lay.n_wf * lay.sv:] == 0.0)   # pressure and time stay zero


def test_noise_on_a_shard(gpu):
    """Rank 1 of 3 computes its elements' noise with its own global element numbers (ieg =
    e_first + e + 1): equal to that slice of the one-rank noise (no averaging: shard-boundary points
    need the case's gather-scatter, and FaceAverage refuses world > 1)."""
    class Part:
        rank, world, backend, force = 1, 3, None, False

        def allreduce_(self, t):
            return t

    lay, co = _cases()["cyl"]
    ctx1 = NekContext(lay, max_cols=4)
    full = ctx1.vector()
    full.zero()
    seeds.mth_rand_add(ctx1, full, 0, co, seeds.NOISE_FC[0])
    sh = lay.shard(1, 3)
    e0, e1 = sh.elem_range()
    ctx = NekContext(sh, max_cols=4, comm=Part())
    pts = slice(e0 * sh.pts_v, e1 * sh.pts_v)
    v = ctx.vector()
    v.zero()
    seeds.mth_rand_add(ctx, v, 0, {k: a[pts] for k, a in co.items()}, seeds.NOISE_FC[0])
    np.testing.assert_array_equal(_field(sh, v, 0), _field(lay, full, 0)[pts])
    with pytest.raises(ValueError):
        seeds.FaceAverage(ctx, {k: a[pts] for k, a in co.items()})


def test_seed_entry_checks(gpu):
    lay, co = _cases()["box3d"]
    ctx = NekContext(lay, max_cols=4)
    v = ctx.vector()
    x = torch.as_tensor(co["x"]).cuda()
    st = ctx.stream
    with pytest.raises(NkvError):   # 3-D without z
        ctx.call("nkv_mth_rand_add", lay.lx1, lay.lx1, lay.lx1, 0, x.data_ptr(), x.data_ptr(), None, 1.0, 1.0, 1.0,
                 v.ptr, st)
    with pytest.raises(NkvError):   # lx1^3 does not divide n_v
        ctx.call("nkv_mth_rand_add", 7, 7, 7, 0, x.data_ptr(), x.data_ptr(), x.data_ptr(), 1.0, 1.0, 1.0, v.ptr, st)
    with pytest.raises(NkvError):
        ctx.call_nl("nkv_group_average", 3, None, None, v.ptr, st)
    with pytest.raises(ValueError):
        seeds.mth_rand_add(ctx, v, lay.n_wf, co, seeds.SCAL_FC)


def test_symmetric_seed_vs_oracle(gpu):
    """add_symmetric_seed (utils.f90:361-406) as the in-tree solver calls it (eigensolvers.f90:
    205-208: wrk%vx, wrk%vy, wrk%vz, wrk%t(:,1)): vy kept from the base vector, the amplitude from the
    velocity dots with the weights; against the oracle (1e-13 relative: smooth functions, the
    device's own sin/cos); then Krylov–Schur from it unnormalised (seed_mode "symm", MGS on the
    non-orthonormal basis) against the oracle's run from the same Q(1)."""
    import ctypes

    from helpers import olayout, oracle_diag_matvec

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.operators import DiagOperator

    lay, co = _cases()["box3d"]
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=24)
    base = ctx.vector()
    base.fill_hash(9)
    seed = seeds.symmetric_seed(ctx, co, base)
    got = seed.to_packed()
    qy = base.to_packed()[lay.sv: lay.sv + lay.n_v]
    ref = orc.add_symmetric_seed(co["y"], co["z"], qy, w, co["z"].min(), co["z"].max())
    for c, r in zip((0, 1, 2, 3), ref):
        g = got[c * lay.sv: c * lay.sv + lay.n_v]
        np.testing.assert_allclose(g, r, rtol=0, atol=1e-13 * np.max(np.abs(r)))
    b = base.to_packed()
    np.testing.assert_array_equal(got[4 * lay.sv:], b[4 * lay.sv:])   # pressure and time untouched
    # Krylov-Schur from the unnormalised seed
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    dref = syn.to_reference_order(lay, d)
    q1 = syn.to_reference_order(lay, got)
    cfg = KrylovSchurConfig(k_dim=16, schur_tgt=5, seed_mode="symm")
    res = krylov_schur(ctx, DiagOperator(ctx, d), seed, cfg)
    r = orc.krylov_schur(L, w, oracle_diag_matvec(L, dref), q1, 16, 5)
    assert res.schur_cnt == r["schur_cnt"] and res.mstart_history == r["mstart"]
    sel = np.abs(r["residual"]) < cfg.eigen_tol
    for v in r["vals"][sel]:
        assert np.min(np.abs(res.vals - v)) <= 1e-10 * abs(v)
    with pytest.raises(ValueError):
        seeds.symmetric_seed(NekContext(cylinder_layout(20), max_cols=4), {"x": np.zeros(720), "y": np.zeros(720)})


def test_symmetric_seed_amplitude_with_sponge_uses_bm1(gpu):
    """With a sponge the context's dot weights are bm1s (zero in the sponge, forcing.f90:101-104),
    but add_symmetric_seed's amplitude weights with bm1 (utils.f90:394-396): passing ``bm1`` gives
    the oracle's seed computed with bm1; without it the amplitude follows the context's bm1s."""
    from nekstab_next_amd import synthetic as syn

    lay, co = _cases()["box3d"]
    w = syn.mass_weights(lay)
    ws = syn.sponge(w)
    assert np.any(ws[: lay.n_v] == 0.0) and np.any(ws[: lay.n_v] != 0.0)
    ctx = NekContext(lay, weights=ws, max_cols=4)
    base = ctx.vector()
    base.fill_hash(9)
    qy = base.to_packed()[lay.sv: lay.sv + lay.n_v]
    for bm1, wref in ((w, w), (None, ws)):
        got = seeds.symmetric_seed(ctx, co, base, bm1=bm1).to_packed()
        ref = orc.add_symmetric_seed(co["y"], co["z"], qy, wref[: lay.n_v], co["z"].min(), co["z"].max())
        for c, r in zip((0, 1, 2, 3), ref):
            g = got[c * lay.sv: c * lay.sv + lay.n_v]
            np.testing.assert_allclose(g, r, rtol=0, atol=1e-13 * np.max(np.abs(r)))
