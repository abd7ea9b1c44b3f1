"""bf_sensitivity (core/sensitivity.f90:81-269), CPU side: the oracle's restatement of Nek5000's
gradm1 / glmapm1 geometric factors and of the pointwise terms, pinned by known answers.

* the GLL derivative matrix (the oracle's barycentric one and the product's dgll formula) maps
  z^k to k z^(k-1) exactly for k <= N, and the two agree;
* gradm1 of a linear field is its constant gradient on the reference's own curved cylinder mesh
  (E=1996, lx1=6, the X block of examples/cylinder/BF_1cyl0.f00001) and on a deformed 3-D box: an
  isoparametric element holds a linear function of x, y, z exactly; on an affine box a polynomial
  of degree <= N per coordinate is differentiated exactly;
* the line-by-line opaddcol3 restatement equals the tensor form of Marquet et al.'s terms
  (tr_i = -sum_j aRe_j d_i dRe_j - ..., pr_i = sum_j dRe_j d_j aRe_i + ...), with the reference's
  dwdz-for-dvdz slip of lines 204/207/213/216 in the z component in 3-D."""
import os

import numpy as np
import pytest

import oracle as orc
from seed_helpers import box_mesh_coords

from nekstab_next_amd.fld import gll_points
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.sensitivity import gll_derivative

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cyl():
    d = np.load(os.path.join(GOLD, "cyl_mesh_xy.npz"))
    return {"x": d["x"], "y": d["y"]}


def deformed_box(lay, ne, L=(2.0, 1.0, 3.0), amp=0.04):
    """box_mesh_coords moved by a smooth map of the position (coincident points stay coincident,
    elements become curved; the map's Jacobian stays positive for amp << 1)."""
    c = box_mesh_coords(lay, ne, L)
    x, y, z = c["x"], c["y"], c["z"]
    return {"x": x + amp * np.sin(2.0 * y) * np.cos(z), "y": y + amp * np.sin(x + z), "z": z + amp * np.cos(1.5 * x) * y}


@pytest.mark.parametrize("n", [2, 4, 6, 8, 10])
def test_gll_derivative_known_answer(n):
    z = gll_points(n)
    Do = orc.gll_derivative(n)
    Dp = gll_derivative(n)
    np.testing.assert_allclose(Do, Dp, rtol=0, atol=1e-12 * n * n)
    for k in range(n):
        exact = k * z ** (k - 1) if k else np.zeros(n)
        np.testing.assert_allclose(Do @ z ** k, exact, rtol=0, atol=1e-12 * n * n)
        np.testing.assert_allclose(Dp @ z ** k, exact, rtol=0, atol=1e-12 * n * n)


def test_gradm1_linear_field_on_cylinder_mesh():
    co = _cyl()
    u = 0.3 * co["x"] - 1.7 * co["y"] + 2.0
    ux, uy = orc.gradm1(6, 2, co, u)
    assert ux.size == 1996 * 36
    np.testing.assert_allclose(ux, 0.3, rtol=0, atol=1e-9)
    np.testing.assert_allclose(uy, -1.7, rtol=0, atol=1e-9)


@pytest.mark.parametrize("lx1", [5, 8])
def test_gradm1_3d_known_answers(lx1):
    ne = (2, 2, 3)
    lay = NekLayout(ldim=3, lx1=lx1, lx2=lx1 - 2, nelgv=int(np.prod(ne)))
    box = box_mesh_coords(lay, ne)
    x, y, z = box["x"], box["y"], box["z"]
    N = lx1 - 1   # degree <= N in each coordinate: exact on the affine box
    u = x ** N * y ** 2 * z ** (N - 1) + 0.5 * y ** N
    ux, uy, uz = orc.gradm1(lx1, 3, box, u)
    scale = np.max(np.abs(u)) * 10
    np.testing.assert_allclose(ux, N * x ** (N - 1) * y ** 2 * z ** (N - 1), rtol=0, atol=1e-11 * scale)
    np.testing.assert_allclose(uy, 2 * x ** N * y * z ** (N - 1) + 0.5 * N * y ** (N - 1), rtol=0, atol=1e-11 * scale)
    np.testing.assert_allclose(uz, (N - 1) * x ** N * y ** 2 * z ** (N - 2), rtol=0, atol=1e-11 * scale)
    curved = deformed_box(lay, ne)
    v = -0.4 * curved["x"] + 1.1 * curved["y"] + 0.25 * curved["z"] - 3.0
    vx, vy, vz = orc.gradm1(lx1, 3, curved, v)
    for got, want in ((vx, -0.4), (vy, 1.1), (vz, 0.25)):
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-10)


@pytest.mark.parametrize("ldim", [2, 3])
def test_bf_terms_tensor_form(ldim):
    rng = np.random.default_rng(7 + ldim)
    n = 257
    modes = {m: rng.standard_normal((ldim, n)) for m in ("dRe", "dIm", "aRe", "aIm")}
    # g[m][c, d] = d(comp c)/d(x_d)
    grads = {m: rng.standard_normal((ldim, ldim, n)) for m in modes}
    g = {(m, "uvw"[c], "xyz"[d]): grads[m][c, d] for m in modes for c in range(ldim) for d in range(ldim)}
    t = orc.bf_sensitivity_terms(ldim, *(list(modes[m]) for m in ("dRe", "dIm", "aRe", "aIm")), g)
    dR, dI, aR, aI = (grads[m] for m in ("dRe", "dIm", "aRe", "aIm"))
    if ldim == 3:   # lines 204/207/213/216: the z component of the v-row takes dw/dz of the direct mode
        dR, dI = dR.copy(), dI.copy()
        dRv, dIv = dR.copy(), dI.copy()
        dRv[1, 2], dIv[1, 2] = grads["dRe"][2, 2], grads["dIm"][2, 2]
    else:
        dRv, dIv = dR, dI

    def direct_term(a, G, Gv):   # sum_j a_j dG_j/dx_i, with the v-row's z slip
        out = np.zeros((ldim, n))
        for j in range(ldim):
            src = Gv if j == 1 else G
            for i in range(ldim):
                out[i] += a[j] * src[j, i]
        return out

    tr = -direct_term(modes["aRe"], dR, dRv) - direct_term(modes["aIm"], dI, dIv)
    ti = direct_term(modes["aRe"], dI, dIv) - direct_term(modes["aIm"], dR, dRv)
    pr = np.einsum("jn,ijn->in", modes["dRe"], aR) + np.einsum("jn,ijn->in", modes["dIm"], aI)
    pi = np.einsum("jn,ijn->in", modes["dRe"], aI) - np.einsum("jn,ijn->in", modes["dIm"], aR)
    for name, ref in (("tr", tr), ("ti", ti), ("pr", pr), ("pi", pi), ("sr", tr + pr), ("si", ti + pi)):
        np.testing.assert_allclose(np.array(t[name]), ref, rtol=0, atol=1e-13)


@pytest.mark.parametrize("three", [False, True])
def test_norm_grad_linear_fields_known_answer(three):
    """oracle.norm_grad (utils.f90:446-486): linear velocity components have constant gradients,
    so the squared gradient norm is sum(coefficients^2) * sum(bm1s) — on the reference's curved
    cylinder mesh and on a deformed 3-D box."""
    if three:
        lay = NekLayout(ldim=3, lx1=5, lx2=3, nelgv=12)
        co = deformed_box(lay, (3, 2, 2))
    else:
        lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1996)
        co = _cyl()
    d = lay.ldim
    rng = np.random.default_rng(2)
    A = rng.uniform(-1, 1, (d, d))
    comps = [sum(A[c, k] * co["xyz"[k]] for k in range(d)) + 0.5 for c in range(d)]
    w = rng.uniform(0.5, 1.5, lay.n_v)
    got = orc.norm_grad(lay.lx1, d, co, w, comps)
    assert abs(got - np.sum(A * A) * w.sum()) <= 1e-9 * got
