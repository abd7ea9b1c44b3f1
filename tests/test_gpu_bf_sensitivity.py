"""GPU parity of ``bf_sensitivity`` (core/sensitivity.f90:81-269) against the oracle's restatement.

* ``nkv_gradm1`` (Nek5000's gradm1 with glmapm1's geometric factors from the GLL coordinates) vs
  ``oracle.gradm1`` on the reference's curved cylinder mesh (2-D, lx1=6, E=1996) and on deformed
  3-D boxes (lx1 = 5, 8; ragged element counts): gate 1e-12 of the gradient's scale; linear fields
  give their constant gradient on the device too;
* ``nkv_bf_sensitivity`` (the pointwise terms) bit-identical to ``oracle.bf_sensitivity_terms`` on
  the same gradients (both follow the reference's opaddcol3 order without contraction);
* the whole chain — four mode files written by the oracle's own #std writer, bi-orthogonalisation,
  gradm1 + dsavg, the terms, six output files — vs the oracle's chain (its reader, its
  coincident-point averaging) to 1e-11, the files read back by the oracle's reader bit for bit;
* a BASELINE config-5-sized mesh (3-D, lx1=8, E=22,088: N_v = 11.3M points per field): the chain's
  size-independent property (linear modes: constant gradients, so every term is a known
  pointwise polynomial) and the gradient kernel's time."""
import numpy as np
import pytest
import torch

import nekio
import oracle as orc
from seed_helpers import box_mesh_coords
from test_bf_sensitivity import _cyl, deformed_box

from nekstab_next_amd import _lib
from nekstab_next_amd import fld
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.sensitivity import BF_OUTPUTS, Gradm1, bf_sensitivity, bf_sensitivity_fields, velocity_layout
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu


def _ctx(lay):
    vlay = velocity_layout(lay)
    return NekContext(vlay, weights=syn.mass_weights(vlay), max_cols=4)


def _grad_device(ctx, coords, u):
    lay = ctx.layout
    op = Gradm1(ctx, coords)
    ut = torch.as_tensor(np.asarray(u, dtype=np.float64)).to(ctx.device)
    out = torch.full((lay.ldim, lay.n_v), np.nan, dtype=torch.float64, device=ctx.device)
    op(ut.data_ptr(), out.data_ptr())
    torch.cuda.synchronize()
    return list(out.cpu().numpy())


def _cases():
    yield "cyl", NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1996), None
    for lx1, ne in ((5, (3, 2, 2)), (8, (2, 3, 2)), (8, (1, 1, 1)), (6, (5, 3, 3))):
        yield f"box{lx1}_{np.prod(ne)}", NekLayout(ldim=3, lx1=lx1, lx2=lx1 - 2, nelgv=int(np.prod(ne))), ne


def _coords(lay, ne):
    return _cyl() if ne is None else deformed_box(lay, ne)


@pytest.mark.parametrize("name,lay,ne", list(_cases()), ids=[c[0] for c in _cases()])
def test_gradm1_kernel_vs_oracle(gpu, name, lay, ne):
    ctx = _ctx(lay)
    co = _coords(lay, ne)
    rng = np.random.default_rng(11)
    x, y = co["x"], co["y"]
    z = co.get("z", 0.0 * x)
    u = np.sin(1.3 * x) * np.cos(0.7 * y) + 0.2 * z * x + 1e-3 * rng.standard_normal(x.size)
    got = _grad_device(ctx, co, u)
    ref = orc.gradm1(lay.lx1, lay.ldim, co, u)
    for g, r in zip(got, ref):
        assert np.all(np.isfinite(g))
        assert np.max(np.abs(g - r)) <= 1e-12 * np.max(np.abs(r))
    # linear fields: the constant gradient on the device as well
    coef = (0.3, -1.7, 0.45)[: lay.ldim]
    lin = sum(c * co[k] for c, k in zip(coef, "xyz")) + 2.0
    for g, c in zip(_grad_device(ctx, co, lin), coef):
        np.testing.assert_allclose(g, c, rtol=0, atol=1e-9)


def test_gradm1_argument_checks(gpu):
    lay = NekLayout(ldim=3, lx1=5, lx2=3, nelgv=2)
    ctx = _ctx(lay)
    co = box_mesh_coords(lay, (2, 1, 1))
    op = Gradm1(ctx, co)
    u = torch.zeros(lay.n_v, dtype=torch.float64, device=ctx.device)
    o = torch.zeros(3 * lay.n_v, dtype=torch.float64, device=ctx.device)
    xp = [t.data_ptr() for t in op.xyz]
    lib, D, n = ctx.lib, op.D.data_ptr(), lay.n_v

    def call(lx1, ldim, x=xp, nfld=1, us=0, gs=n, grad=o.data_ptr()):
        return lib.nkv_gradm1(ctx._Lp, lx1, ldim, D, *x, u.data_ptr(), nfld, us, grad, gs, ctx.stream)

    assert call(5, 3) == _lib.NKV_OK
    assert call(5, 4) == _lib.NKV_EINVAL
    assert call(5, 3, x=[xp[0], xp[1], None]) == _lib.NKV_EINVAL and "zm" in _lib.last_error()
    assert call(6, 3) == _lib.NKV_EINVAL        # 216 points per element do not divide n_v
    assert call(11, 3) == _lib.NKV_EINVAL
    assert call(5, 3, nfld=0) == _lib.NKV_EINVAL
    assert call(5, 3, nfld=2, us=n - 1) == _lib.NKV_EINVAL and "strides" in _lib.last_error()
    assert call(5, 3, gs=n - 1) == _lib.NKV_EINVAL
    assert call(5, 3, grad=None) == _lib.NKV_EINVAL
    assert lib.nkv_bf_sensitivity(ctx._Lp, u.data_ptr(), u.data_ptr(), u.data_ptr(), None, u.data_ptr(),
                                  u.data_ptr(), 3, ctx.stream) == _lib.NKV_EINVAL


def test_gradm1_several_fields_one_launch(gpu):
    """nfld fields at a stride in one launch equal one launch per field, bit for bit."""
    ne = (3, 2, 2)
    lay = NekLayout(ldim=3, lx1=6, lx2=4, nelgv=12)
    ctx = _ctx(lay)
    co = deformed_box(lay, ne)
    op = Gradm1(ctx, co)
    n, stride = lay.n_v, lay.n_v + 78   # every field 16-byte aligned, as every pointer of the ABI
    rng = np.random.default_rng(2)
    u = torch.as_tensor(rng.standard_normal(3 * stride)).to(ctx.device)
    many = torch.full((3 * 3, n + 6), np.nan, dtype=torch.float64, device=ctx.device)
    op(u.data_ptr(), many.data_ptr(), nfld=3, u_stride=stride, g_stride=n + 6)
    for f in range(3):
        one = torch.empty((3, n), dtype=torch.float64, device=ctx.device)
        op(u.data_ptr() + 8 * f * stride, one.data_ptr())
        assert torch.equal(one, many[3 * f: 3 * f + 3, :n])
    assert torch.all(torch.isnan(many[:, n:]))


@pytest.mark.parametrize("ldim", [2, 3])
def test_bf_terms_kernel_bit_exact(gpu, ldim):
    lay = NekLayout(ldim=ldim, lx1=6, lx2=4, nelgv=37)
    ctx = _ctx(lay)
    vl = ctx.layout
    rng = np.random.default_rng(3 * ldim)
    vecs, comps = [], []
    for _ in range(4):
        v = ctx.vector()
        host = np.zeros(vl.ld)
        cs = [rng.standard_normal(vl.n_v) for _ in range(ldim)]
        for c in range(ldim):
            host[c * vl.sv: c * vl.sv + vl.n_v] = cs[c]
        v.from_packed(host)
        vecs.append(v)
        comps.append(cs)
    G = rng.standard_normal((4, ldim, ldim, vl.n_v))
    grad = torch.zeros(4 * ldim * ldim * vl.sv, dtype=torch.float64, device=ctx.device)
    gv = grad.view(4, ldim, ldim, vl.sv)
    gv[..., : vl.n_v] = torch.as_tensor(G).to(ctx.device)
    out = torch.full((6 * ldim * vl.sv,), np.nan, dtype=torch.float64, device=ctx.device)
    ctx.call("nkv_bf_sensitivity", *(v.ptr for v in vecs), grad.data_ptr(), out.data_ptr(), ldim, ctx.stream)
    got = out.view(6, ldim, vl.sv)[:, :, : vl.n_v].cpu().numpy()
    g = {(m, "uvw"[c], "xyz"[d]): G[mi, c, d] for mi, m in enumerate(("dRe", "dIm", "aRe", "aIm"))
         for c in range(ldim) for d in range(ldim)}
    ref = orc.bf_sensitivity_terms(ldim, *comps, g)
    for t, name in enumerate(("tr", "ti", "pr", "pi", "sr", "si")):
        assert np.array_equal(got[t], np.array(ref[name])), name


def _write_modes(tmp, lay, co, session):
    """dRe/dIm (file 1) and aRe/aIm (file 2): smooth fields of the coordinates plus small hashed
    noise, written by the oracle's own #std writer (pressure present; the reader ignores it)."""
    g = nekio.Geom(lay.ldim, lay.lx1, lay.lx2, lay.nelgv)
    x, y = co["x"], co["y"]
    z = co.get("z", np.zeros_like(x))
    rng = np.random.default_rng(5)
    nv = lay.n_v
    for k, (prefix, num) in enumerate((("dRe", 1), ("dIm", 1), ("aRe", 2), ("aIm", 2))):
        ref = np.zeros(lay.ldim * nv + lay.n_p + 1)
        for c in range(lay.ldim):
            f = np.sin((1.0 + 0.3 * k) * x + 0.5 * c) * np.cos((0.6 + 0.1 * c) * y - 0.2 * k) + 0.1 * (c + 1) * z
            ref[c * nv:(c + 1) * nv] = f + 1e-4 * rng.standard_normal(nv)
        ref[lay.ldim * nv: lay.ldim * nv + lay.n_p] = rng.standard_normal(lay.n_p)
        nekio.write_std(str(tmp / fld.fld_name(prefix, session, 0, num)), g, ref, time=float(num), istep=num)


@pytest.mark.parametrize("case", ["cyl", "box"])
def test_bf_sensitivity_chain_vs_oracle(gpu, tmp_path, case):
    if case == "cyl":
        lay, co = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1996), _cyl()
    else:
        ne = (3, 3, 2)
        lay = NekLayout(ldim=3, lx1=6, lx2=4, nelgv=18)
        co = deformed_box(lay, ne)
    _write_modes(tmp_path, lay, co, "bfs")
    ctx = _ctx(lay)
    res = bf_sensitivity(ctx, str(tmp_path), co, session="bfs", write_coords=True)

    g = nekio.Geom(lay.ldim, lay.lx1, lay.lx2, lay.nelgv)
    nvel = lay.ldim * lay.n_v

    def load(prefix, num):
        v = nekio.read_std_vector([str(tmp_path / fld.fld_name(prefix, "bfs", 0, num))], g)
        return np.concatenate([v[:nvel], np.zeros(1)])

    L = orc.OLayout(lay.n_v, 0, lay.ldim, False, lay.ldim)
    w = syn.mass_weights(ctx.layout)
    terms, vecs, _ = orc.bf_sensitivity(L, w, lay.lx1, co, load("dRe", 1), load("dIm", 1), load("aRe", 2),
                                        load("aIm", 2))
    assert abs(res["inner_product"]) > 1e-3
    for name in ("tr", "ti", "pr", "pi", "sr", "si"):
        ref = np.array(terms[name])
        got = np.array(res["fields"][name])
        scale = np.max(np.abs(ref))
        assert scale > 0 and np.max(np.abs(got - ref)) <= 1e-11 * scale, name
    # the six files: velocity (and mesh) only, header time of the last mode file, read back bit for bit
    assert [p.rsplit("/", 1)[1] for p in res["paths"]] == [fld.fld_name(p, "bfs", 0, 1) for p in BF_OUTPUTS]
    for path, name in zip(res["paths"], ("tr", "ti", "pr", "pi", "sr", "si")):
        tok, ids, fields = nekio.read_std(path)
        assert tok[11] == "XU" and float(tok[7]) == 2.0
        assert np.array_equal(ids, np.arange(1, lay.nelgv + 1))
        for c, nm in enumerate(("vx", "vy", "vz")[: lay.ldim]):
            assert np.array_equal(fields[nm].ravel(), res["fields"][name][c])
        assert np.array_equal(fields["x"].ravel(), co["x"])


def test_bf_sensitivity_config5_mesh(gpu, tmp_path):
    """3-D, lx1=8, E=22,088 (BASELINE config 5's mesh: 11.3M points per field) on a deformed box:
    modes linear in the coordinates have constant gradients, so after dsavg every term is a known
    linear combination of the modes — checked pointwise; the gradient kernel's time is reported."""
    ne = (22, 22, 22088 // 484 + 1)
    nel = 22088
    lay = NekLayout(ldim=3, lx1=8, lx2=6, nelgv=nel)
    box = box_mesh_coords(NekLayout(ldim=3, lx1=8, lx2=6, nelgv=int(np.prod(ne))), ne, L=(1.0, 1.0, 2.0))
    co = {k: v[: nel * 512] for k, v in box.items()}
    del box
    ctx = _ctx(lay)
    vl = ctx.layout
    A = np.array([[[0.3, -0.2, 0.1], [0.05, 0.4, -0.3], [0.2, 0.1, 0.6]],
                  [[-0.1, 0.2, 0.3], [0.5, -0.4, 0.1], [0.0, 0.3, -0.2]],
                  [[0.7, 0.1, -0.5], [0.2, 0.2, 0.2], [-0.3, 0.4, 0.1]],
                  [[0.1, -0.6, 0.2], [0.3, 0.0, -0.1], [0.4, -0.2, 0.5]]])   # [mode][comp][dir]
    vecs = []
    for m in range(4):
        host = np.zeros(vl.ld)
        for c in range(3):
            host[c * vl.sv: c * vl.sv + vl.n_v] = A[m, c, 0] * co["x"] + A[m, c, 1] * co["y"] + A[m, c, 2] * co["z"]
        vecs.append(ctx.vector().from_packed(host))
    op = Gradm1(ctx, co)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tmp = torch.empty(9 * vl.sv, dtype=torch.float64, device=ctx.device)
    for nfld, bytes_per_pt in ((1, 7), (3, 15)):   # x, y, z + nfld fields read, 3 nfld gradients written
        op(vecs[0].ptr, tmp.data_ptr(), nfld=nfld, u_stride=vl.sv, g_stride=vl.sv)
        torch.cuda.synchronize()
        s.record()
        for _ in range(5):
            op(vecs[0].ptr, tmp.data_ptr(), nfld=nfld, u_stride=vl.sv, g_stride=vl.sv)
        e.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(e) / 5
        gbs = bytes_per_pt * 8 * vl.n_v / (ms * 1e-3) / 1e9
        print(f"gradm1 lx1=8 E={nel} nfld={nfld}: {ms:.3f} ms per launch, {gbs:.0f} GB/s of algorithmic traffic")
    out, grad = bf_sensitivity_fields(ctx, *vecs, op, face_average=None)
    torch.cuda.synchronize()
    G = grad.view(4, 3, 3, vl.sv)[..., : vl.n_v]
    for m in range(4):
        for c in range(3):
            for d in range(3):
                assert torch.max(torch.abs(G[m, c, d] - A[m, c, d])).item() < 1e-9
    got = out.view(6, 3, vl.sv)[:, :, : vl.n_v]
    modes = [[torch.as_tensor(A[m, c, 0] * co["x"] + A[m, c, 1] * co["y"] + A[m, c, 2] * co["z"]) for c in range(3)]
             for m in range(4)]
    dR, dI, aR, aI = A
    tr2 = [-(modes[2][0] * dR[0, i] + modes[2][1] * (dR[1, i] if i < 2 else dR[2, 2]) + modes[2][2] * dR[2, i])
           - (modes[3][0] * dI[0, i] + modes[3][1] * (dI[1, i] if i < 2 else dI[2, 2]) + modes[3][2] * dI[2, i])
           for i in range(3)]
    pr2 = [sum(modes[0][j] * aR[i, j] + modes[1][j] * aI[i, j] for j in range(3)) for i in range(3)]
    for i in range(3):
        assert torch.max(torch.abs(got[0, i].cpu() - tr2[i])).item() < 1e-8
        assert torch.max(torch.abs(got[2, i].cpu() - pr2[i])).item() < 1e-8
        assert torch.max(torch.abs(got[4, i].cpu() - (tr2[i] + pr2[i]))).item() < 1e-8
