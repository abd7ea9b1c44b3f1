"""Seed noise (CPU): the oracle's mth_rand / op_add_noise restatement (utils.f90:258-418) against
the frozen fixture on the reference's cylinder mesh, its libm sensitivity, the product's
coincident-point grouping (dssum + vmult on one rank) against the oracle's independent one, and
the mesh-coordinate reader."""
import os

import numpy as np
import pytest

import oracle as orc
from seed_helpers import box_mesh_coords

from nekstab_next_amd import fld
from nekstab_next_amd import seeds
from nekstab_next_amd.layout import NekLayout, cylinder_layout

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _cyl():
    d = np.load(os.path.join(GOLD, "cyl_mesh_xy.npz"))
    return {"x": d["x"], "y": d["y"]}


def _checksum(a):
    return np.array([np.sum(a), np.sum(a * a), a[0], a[-1]])


def test_noise_oracle_vs_golden():
    """op_add_noise's vx / vy noise (fc from utils.f90:324-327) with dssum/vmult + dsavg on the
    cylinder mesh (E=1996, lx1=6, the reference's BF_1cyl0.f00001 X block): equal to the frozen
    oracle output (written by tests/golden/make_golden.py)."""
    co = _cyl()
    g = np.load(os.path.join(GOLD, "noise_cyl.npz"))
    for c, fc in enumerate(seeds.NOISE_FC[:2]):
        q = orc.noise_field(6, 6, 1, 0, co["x"], co["y"], None, fc)
        q = orc.coincident_average(orc.coincident_average(q, co), co)
        np.testing.assert_array_equal(_checksum(q), g[f"c{c}_checksum"])
        np.testing.assert_array_equal(q[::97], g[f"c{c}_sample"])
        assert np.all(np.abs(q) <= 1.0)


def test_mth_rand_known_value_and_libm_sensitivity():
    """mth_rand at one point by hand (utils.f90:415-417), and how much the hash depends on the last
    bit of sin: glibc against correctly rounded sin/cos agree on >= 98 % of a sample of cylinder
    points and differ by up to O(1e-3) elsewhere (which is why the device computes correctly
    rounded sin/cos, tests/test_gpu_seeds.py)."""
    import math

    x, y, ieg, ix, iy = 0.25, -1.5, 17.0, 3.0, 2.0
    fc = seeds.NOISE_FC[0]
    r = fc[0] * (ieg + x * math.sin(y)) + fc[1] * ix * iy + fc[2] * ix
    assert orc.mth_rand(ix, iy, 1.0, ieg, (x, y, 0.0), fc, False) == math.cos(1e3 * math.sin(1e3 * math.sin(r)))
    co = _cyl()
    pts = np.arange(0, co["x"].size, 37)
    a = orc.noise_field(6, 6, 1, 0, co["x"], co["y"], None, fc, points=pts)[pts]
    b = orc.noise_field(6, 6, 1, 0, co["x"], co["y"], None, fc, kind="cr", points=pts)[pts]
    assert np.mean(a == b) >= 0.98


@pytest.mark.parametrize("case", ["cyl", "box3d"])
def test_coincident_groups_vs_oracle(case):
    """The product's CSR groups of coincident points (seeds.coincident_groups, summed in member
    order as nkv_group_average does) equal the oracle's dict grouping bit for bit; every shared
    GLL point of a conforming mesh is found (the box's 3-D corners: 8 elements; the cylinder's
    unstructured 2-D mesh has vertices shared by 4 and by 5 elements)."""
    if case == "cyl":
        co = _cyl()
    else:
        lay = NekLayout(ldim=3, lx1=5, lx2=3, nelgv=24, n_scalars=1)
        co = box_mesh_coords(lay, (2, 3, 4))
    q = np.random.default_rng(5).standard_normal(co["x"].size)
    start, members = seeds.coincident_groups(co)
    got = q.copy()
    for a, b in zip(start[:-1], start[1:]):
        s = 0.0
        for i in members[a:b]:
            s = s + q[i]
        got[members[a:b]] = s * (1.0 / (b - a))
    np.testing.assert_array_equal(got, orc.coincident_average(q, co))
    sizes = np.diff(start)
    assert sizes.min() >= 2 and sizes.max() == (5 if case == "cyl" else 8)


def test_coincident_groups_across_a_rounding_half_step():
    """Two copies of one point a few ulps apart on either side of a rounding half-step of the
    grouping grid (cells of 1e-9 x extent) are one group: in x, in y, and in both; the
    oracle's independent grouping agrees, and points 0.01 cells apart stay apart."""
    ext = 1.0
    tol = 1e-9 * ext
    c = (123456 + 0.5) * tol
    lo, hi = np.nextafter(c, -1.0), np.nextafter(np.nextafter(c, 2.0), 2.0)
    assert int(np.round(lo / tol)) != int(np.round(hi / tol))   # the pair does straddle the half-step
    far = c + 0.01 * tol
    x = np.array([0.0, ext, lo, hi, 0.3, 0.3, lo, hi, 0.7, far, c - 0.2 * tol])
    y = np.array([0.0, ext, 0.5, 0.5, lo, hi, lo, hi, 0.1, 0.9, 0.9])
    co = {"x": x, "y": y}
    start, members = seeds.coincident_groups(co)
    groups = sorted([int(i) for i in members[a:b]] for a, b in zip(start[:-1], start[1:]))
    assert groups == [[2, 3], [4, 5], [6, 7]], groups
    q = np.random.default_rng(3).standard_normal(x.size)
    got = q.copy()
    for g in groups:
        got[g] = (q[g[0]] + q[g[1]]) * 0.5
    np.testing.assert_array_equal(got, orc.coincident_average(q, co))


def test_coords_from_fld_element_map(tmp_path):
    """Mesh coordinates from a field file whose element map is permuted (as BF_1cyl0.f00001's is:
    50, 51, ...), on one rank and as the shard of rank 1 of 3."""
    lay = cylinder_layout(1996)
    co = _cyl()
    perm = np.random.default_rng(1).permutation(lay.nelgv)
    f = fld.FldFile(6, 6, 1, lay.nelgv, 0.0, 0, 0, 1, "XU", (perm + 1).astype(np.int32),
                    {"x": co["x"].reshape(-1, 36)[perm], "y": co["y"].reshape(-1, 36)[perm],
                     "vx": np.zeros((lay.nelgv, 36)), "vy": np.zeros((lay.nelgv, 36))})
    path = str(tmp_path / "msh0.f00001")
    fld.write_fld(path, f)
    got = seeds.coords_from_fld(lay, fld.read_fld(path))
    np.testing.assert_array_equal(got["x"], co["x"])
    np.testing.assert_array_equal(got["y"], co["y"])
    sh = lay.shard(1, 3)
    e0, e1 = sh.elem_range()
    got = seeds.coords_from_fld(sh, fld.read_fld(path))
    np.testing.assert_array_equal(got["y"], co["y"][e0 * 36:e1 * 36])
    with pytest.raises(ValueError):
        seeds.coords_from_fld(lay, fld.FldFile(6, 6, 1, 1996, rdcode="U", emap=np.arange(1, 3, dtype=np.int32),
                                                 fields={"x": np.zeros((2, 36)), "y": np.zeros((2, 36))}))
