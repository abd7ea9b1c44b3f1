"""Nek5000 field-file I/O and the HES/Spectre checkpoint text formats (CPU only)."""
import os

import numpy as np
import pytest

from nekstab_next_amd import checkpoint as ck
from nekstab_next_amd import fld
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout, cylinder_layout

BF = "/root/reference/examples/cylinder/BF_1cyl0.f00001"


@pytest.mark.skipif(not os.path.exists(BF), reason="reference data file not present (GPU box)")
def test_reference_base_flow_roundtrip(tmp_path):
    """The cylinder base flow shipped with the reference (#std 8 6 6 1 1996 ... XUP) reads into the
    cylinder layout and writes back byte-compatible field data."""
    f = fld.read_fld(BF)
    assert (f.nx, f.ny, f.nz, f.nelgt, f.rdcode) == (6, 6, 1, 1996, "XUP")
    assert sorted(f.emap.tolist()) == list(range(1, 1997))
    lay = cylinder_layout(1996)
    v = fld.vector_from_fld(lay, f)
    # velocity lands element-by-element at its global id
    e = int(f.emap[0]) - 1
    np.testing.assert_array_equal(v[e * 36:(e + 1) * 36], f.fields["vx"][0])
    np.testing.assert_array_equal(v[lay.sv + e * 36: lay.sv + (e + 1) * 36], f.fields["vy"][0])
    # write (with coordinates) and read back: velocity exact, pressure through lx1 -> lx2 -> lx1
    order = np.argsort(f.emap)
    coords = {"x": f.fields["x"][order], "y": f.fields["y"][order]}
    g = fld.fld_from_vector(lay, v, time=f.time, istep=f.istep, coords=coords)
    p = tmp_path / "BF_copy0.f00001"
    fld.write_fld(str(p), g)
    h = fld.read_fld(str(p))
    assert h.rdcode == "XUP" and os.path.getsize(p) == os.path.getsize(BF)
    np.testing.assert_array_equal(h.fields["vx"], f.fields["vx"][order])
    np.testing.assert_array_equal(h.fields["x"], f.fields["x"][order])
    v2 = fld.vector_from_fld(lay, h)
    np.testing.assert_allclose(v2, v, rtol=0, atol=1e-14)


def test_pressure_mesh_mapping_is_exact_on_polynomials():
    for ldim, lx1 in ((2, 6), (3, 8)):
        lx2 = lx1 - 2
        xg = fld.gauss_points(lx2)
        if ldim == 2:
            X, Y = np.meshgrid(xg, xg)
            p2 = (1 + X ** 3 - 2 * X * Y + Y ** 2).reshape(1, -1)
        else:
            Z, Y, X = np.meshgrid(xg, xg, xg, indexing="ij")
            p2 = (1 + X ** 3 - 2 * X * Y * Z + Y ** 2).reshape(1, -1)
        p1 = fld.map_pressure_to_mesh1(p2, lx1, lx2, ldim)
        back = fld.map_pressure_to_mesh2(p1, lx1, lx2, ldim)
        np.testing.assert_allclose(back, p2, atol=1e-13)


@pytest.mark.parametrize("world", [1, 3])
def test_multifile_vector_roundtrip(tmp_path, world):
    g = NekLayout(ldim=3, lx1=5, lx2=3, nelgv=11, n_scalars=2)
    full = syn.hash_vector(g, 9)
    for r in range(world):
        s = g.shard(r, world)
        fld.write_fld(str(tmp_path / fld.fld_name("KRY", "box", r, 7)), fld.fld_from_vector(s, syn.hash_vector(s, 9), 1.5, 7))
    files = fld.read_fld_set(str(tmp_path), "KRY", "box", 7)
    assert len(files) == world and files[0].rdcode == "UPTS01"
    back = fld.vector_from_fld(g, files)
    live = np.concatenate([np.arange(f * g.sv, f * g.sv + g.n_v) for f in range(g.n_wf)])
    np.testing.assert_array_equal(back[live], full[live])
    pr = np.arange(g.n_wf * g.sv, g.n_wf * g.sv + g.n_p)
    np.testing.assert_allclose(back[pr], full[pr], atol=1e-13)


def test_hes_text_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    k = 9
    H = np.zeros((k + 1, k))
    H[np.triu_indices(k + 1, -1)[0][: (k + 1) * k], 0] = 0
    H = np.triu(rng.standard_normal((k + 1, k)), -1)
    p = tmp_path / "HESnek0009"
    ck.write_hes(str(p), H, k)
    H2 = ck.read_hes(str(p), k, 12)
    np.testing.assert_array_equal(H2[: k + 1, :k], H)
    assert not np.any(H2[:, k:])
    # the reference's list-directed output (several values per line) reads the same way
    with open(tmp_path / "HESref", "w") as fh:
        for i in range(k + 1):
            fh.write("  ".join(repr(float(x)) for x in H[i]) + "\n")
    np.testing.assert_array_equal(ck.read_hes(str(tmp_path / "HESref"), k, k)[: k + 1, :k], H)


def test_log_transform():
    assert ck.log_transform(complex(2.0, 0.0)) == complex(np.log(2.0), 0.0)
    v = ck.log_transform(complex(-1.0, 0.0))
    assert v.imag == 0.0  # aimag(x) == 0 -> real part only (eigensolvers.f90:867)
    z = complex(0.3, 0.4)
    assert abs(ck.log_transform(z) - np.log(z)) < 1e-15
