"""GPU parity of the spurious-mode filter in ``outpost_ks`` (core/eigensolvers.f90:587-595) and of
``norm_grad`` (core/utils.f90:446-486) against the oracle's restatement.

* :class:`NormGrad` (``nkv_gradm1`` + one weighted dot over the ldim^2 gradient segments) vs
  ``oracle.norm_grad`` (gradm1 + glsc3 in the reference's order) on the reference's curved cylinder
  mesh (2-D, lx1=6, E=1996) and on deformed 3-D boxes: 1e-12 relative;
* a W-self-adjoint operator on the cylinder mesh with three exactly known eigenvectors, the
  dominant one oscillatory (squared gradient norm ~ 10^2, "spurious") and two smooth ones: the
  product's Krylov–Schur + ``outpost_ks(coords=...)`` skips the dominant mode and writes the two
  smooth ones as files 1 and 2 (the reference's ``outp`` numbering); the oracle's mode loop
  (``oracle.outpost_ks_modes``) on the product's own basis and Ritz vectors takes the same
  decisions with the same gradient norms (1e-12) and the same mode files (1e-12), and the oracle's
  own Krylov–Schur on the same operator takes the same decisions.
"""
import os

import numpy as np
import pytest

import oracle as orc
from helpers import olayout
from test_bf_sensitivity import _cyl, deformed_box

from nekstab_next_amd import fld
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.krylov_schur import krylov_schur, outpost_ks
from nekstab_next_amd.layout import NekLayout, cylinder_layout
from nekstab_next_amd.operators import CallableOperator, DiagOperator
from nekstab_next_amd.sensitivity import NormGrad
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu


def _cases():
    yield "cyl", cylinder_layout(1996), None
    for lx1, ne in ((5, (3, 2, 2)), (8, (2, 3, 2))):
        yield f"box{lx1}", NekLayout(ldim=3, lx1=lx1, lx2=lx1 - 2, nelgv=int(np.prod(ne)), n_scalars=1), ne


def _fields(lay, co, seed):
    """Smooth velocity components on the mesh plus a little noise (reference point order)."""
    rng = np.random.default_rng(seed)
    x, y = co["x"], co["y"]
    z = co.get("z", 0.0 * x)
    out = []
    for c in range(lay.ldim):
        a, b = rng.uniform(0.2, 1.5, 2)
        out.append(np.sin(a * x + c) * np.cos(b * y) + 0.3 * z * y + 1e-3 * rng.standard_normal(x.size))
    return out


@pytest.mark.parametrize("name,lay,ne", list(_cases()), ids=[c[0] for c in _cases()])
def test_norm_grad_vs_oracle(gpu, name, lay, ne):
    co = _cyl() if ne is None else deformed_box(lay, ne)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=4)
    comps = _fields(lay, co, 3)
    host = np.zeros(lay.ld)
    for c, u in enumerate(comps):
        host[c * lay.sv: c * lay.sv + lay.n_v] = u
    host[lay.n_wf * lay.sv: lay.n_wf * lay.sv + lay.n_p] = 7.0   # pressure / scalars: not in norm_grad
    if lay.n_scalars:
        host[lay.ldim * lay.sv: lay.ldim * lay.sv + lay.n_v] = 5.0
    v = ctx.vector().from_packed(host)
    got = NormGrad(ctx, co)(v)
    ref = orc.norm_grad(lay.lx1, lay.ldim, co, syn.mass_weights(lay)[: lay.n_v], comps)
    assert ref > 0 and abs(got - ref) <= 1e-12 * ref, (got, ref)


def _modes(lay, co):
    """Three W-orthonormal velocity fields (padded device layout, pressure 0): the first
    oscillatory (a spurious-looking mode), the other two smooth."""
    x, y = co["x"], co["y"]
    w = syn.mass_weights(lay)[: lay.n_v]
    raw = [(np.sin(6.0 * x) * np.cos(6.0 * y), np.cos(5.0 * x + 1.0) * np.sin(7.0 * y)),
           (np.cos(0.05 * x), 0.3 * np.sin(0.04 * y)),
           (0.2 * np.sin(0.03 * y + 0.4), np.cos(0.06 * x - 0.2))]
    vs = []
    for u, v in raw:
        vec = np.zeros(lay.ld)
        vec[: lay.n_v], vec[lay.sv: lay.sv + lay.n_v] = u, v
        for q in vs:   # Gram–Schmidt in the W inner product (weighted fields only)
            vec -= (np.sum(w * vec[: lay.n_v] * q[: lay.n_v]) + np.sum(w * vec[lay.sv: lay.sv + lay.n_v]
                                                                        * q[lay.sv: lay.sv + lay.n_v])) * q
        nrm = np.sqrt(np.sum(w * vec[: lay.n_v] ** 2) + np.sum(w * vec[lay.sv: lay.sv + lay.n_v] ** 2))
        vs.append(vec / nrm)
    return vs


MU = (0.97, 0.95, 0.93)


def _operator(ctx, vs, d):
    """A = P D P + sum_k mu_k v_k <v_k, .>_W with P = I - sum_k v_k <v_k, .>_W: eigenpairs (mu_k, v_k)
    exactly, the rest of the spectrum that of the compressed bulk D (<= 0.5)."""
    D = DiagOperator(ctx, d)
    V = [ctx.vector().from_packed(v) for v in vs]
    t = ctx.vector()

    def mv(x, y):
        c = [ctx.dot(v, x, time=False) for v in V]
        t.copy_from(x, time=False)
        for ck, v in zip(c, V):
            t.axpby(1.0, v, -ck)
        D.matvec(t, y)
        e = [ctx.dot(v, y, time=False) for v in V]
        for ck, ek, mu, v in zip(c, e, MU, V):
            y.axpby(1.0, v, mu * ck - ek)

    return CallableOperator(mv, mv)


def _oracle_operator(lay, vs, d):
    L = olayout(lay)
    w = syn.mass_weights(lay)[: lay.n_v]
    wf = np.concatenate([w] * lay.n_wf + [np.zeros(lay.n_p + 1)])
    V = [syn.to_reference_order(lay, v) for v in vs]
    dr = syn.to_reference_order(lay, d)

    def mv(x, y):
        c = [float(np.sum(wf * v * x)) for v in V]
        t = x.copy()
        for ck, v in zip(c, V):
            t[:-1] -= ck * v[:-1]
        yy = dr * t
        yy[-1] = 0.0
        e = [float(np.sum(wf * v * yy)) for v in V]
        for ck, ek, mu, v in zip(c, e, MU, V):
            yy[:-1] += (mu * ck - ek) * v[:-1]
        y[:] = yy

    return L, mv


def test_outpost_ks_skips_spurious_mode_vs_oracle(gpu, tmp_path):
    lay = cylinder_layout(1996)
    co = _cyl()
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=32)
    vs = _modes(lay, co)
    rng = np.random.default_rng(4)
    d = syn.from_reference_order(lay, np.concatenate([0.5 * rng.uniform(0.0, 1.0, lay.N), [0.0]]))
    A = _operator(ctx, vs, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    cfg = KrylovSchurConfig(k_dim=24, schur_tgt=3)
    res = krylov_schur(ctx, A, seed, cfg)
    assert res.converged >= 3
    np.testing.assert_allclose(res.vals[:3].real, MU, rtol=1e-10)
    out = outpost_ks(ctx, res, str(tmp_path), evop="d", session="cyl", coords=co, orthonormality=False)
    assert out["skipped"] == [0] and out["modes"][:2] == [1, 2], out
    g0 = out["grad_norms"][0]
    assert max(g0) > 1.1 and all(max(out["grad_norms"][i]) < 1e-2 for i in (1, 2))

    # the oracle's mode loop on the product's own basis and Ritz vectors
    L = olayout(lay)
    w = syn.mass_weights(lay)[: lay.n_v]
    k = cfg.k_dim
    Q = np.stack([syn.to_reference_order(lay, res.Q[i].to_packed()) for i in range(k)])
    ref = orc.outpost_ks_modes(L, w, Q, res.vecs, res.converged, k, lay.lx1, co)
    assert [r[0] for r in ref if r[1] is None] == out["skipped"]
    assert [r[0] for r in ref if r[1] is not None] == out["modes"]
    for i, num, g_re, g_im, re, im in ref:
        p_re, p_im = out["grad_norms"][i]
        assert abs(p_re - g_re) <= 1e-12 * max(g_re, 1e-300) and abs(p_im - g_im) <= 1e-12 * max(g_im, 1e-16), i
        if num is None:
            assert not os.path.exists(tmp_path / fld.fld_name("dRe", "cyl", 0, out["modes"].__len__() + 1))
            continue
        for part, vec in (("dRe", re), ("dIm", im)):
            f = fld.read_fld(str(tmp_path / fld.fld_name(part, "cyl", 0, num)))
            assert f.time == float(num)
            got = syn.to_reference_order(lay, fld.vector_from_fld(lay, f))
            assert np.max(np.abs(got[:-1] - vec[:-1])) <= 1e-12 * max(np.max(np.abs(vec)), 1e-300)
    # Spectre_NS*_conv.dat: one line per written mode
    with open(tmp_path / "Spectre_NSd_conv.dat") as fh:
        assert len(fh.readlines()) == len(out["modes"])

    # the oracle's own Krylov–Schur on the same operator takes the same decisions
    L2, mv = _oracle_operator(lay, vs, d)
    q1 = orc.prepare_seed(L2, w, syn.to_reference_order(lay, seed.to_packed()))
    full = orc.krylov_schur(L2, w, mv, q1, k, cfg.schur_tgt)
    ref2 = orc.outpost_ks_modes(L2, w, full["Q"], full["vecs"], full["converged"], k, lay.lx1, co)
    assert [r[0] for r in ref2 if r[1] is None][:1] == [0]
    assert [r[0] for r in ref2 if r[1] is not None][:2] == [1, 2]
    for (i, num, g_re, g_im, _, _), (i2, num2, g2_re, g2_im, _, _) in zip(ref[:3], ref2[:3]):
        assert (i, num) == (i2, num2)
        assert abs(g_re - g2_re) <= 1e-6 * g2_re + 1e-12
