"""Layout/shard arithmetic, shard-independent generators, and the C ABI surface (CPU only: the
library is loaded and its exports checked; no compute entry point is called without a GPU)."""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle as orc
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NKV_TILE, NekLayout, box3d_layout, cylinder_layout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_baseline_config_sizes():
    assert cylinder_layout(1996).N == 175648 and cylinder_layout(1996).N_w == 143712
    assert cylinder_layout(22728).N == 2000064
    c3 = box3d_layout(44176)
    assert (c3.n_v, c3.N_w, c3.n_p, c3.N) == (22618112, 90472448, 9542016, 100014464)
    assert box3d_layout(22088).N == 50007232


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shards_partition_elements(world):
    g = box3d_layout(44176)
    shards = [g.shard(r, world) for r in range(world)]
    assert sum(s.nelv for s in shards) == g.nelgv
    assert sum(s.N for s in shards) == g.N
    off = 0
    for s in shards:
        assert s.v_offset == off * g.pts_v and s.p_offset == off * g.pts_p
        off += s.nelv
        assert s.sv % NKV_TILE == 0 and s.sp % NKV_TILE == 0 and s.ld % NKV_TILE == 0
        assert s.sv >= s.n_v and s.ld >= s.rows + 1


@pytest.mark.parametrize("world", [2, 3, 4])
def test_generators_are_shard_independent(world):
    g = NekLayout(ldim=3, lx1=4, lx2=2, nelgv=13, n_scalars=1)
    full = syn.to_reference_order(g, syn.hash_vector(g, 77))
    dfull, _ = syn.laplacian_shift_invert(g)
    dfull = syn.to_reference_order(g, dfull)
    wfull = syn.mass_weights(g)
    parts = {f: [] for f in range(g.n_wf + 1)}
    dparts = {f: [] for f in range(g.n_wf + 1)}
    wparts = []
    for r in range(world):
        s = g.shard(r, world)
        v = syn.to_reference_order(s, syn.hash_vector(s, 77))
        d, _ = syn.laplacian_shift_invert(s)
        d = syn.to_reference_order(s, d)
        for f in range(g.n_wf):
            parts[f].append(v[f * s.n_v:(f + 1) * s.n_v])
            dparts[f].append(d[f * s.n_v:(f + 1) * s.n_v])
        parts[g.n_wf].append(v[g.n_wf * s.n_v: g.n_wf * s.n_v + s.n_p])
        dparts[g.n_wf].append(d[g.n_wf * s.n_v: g.n_wf * s.n_v + s.n_p])
        wparts.append(syn.mass_weights(s))
    cat = np.concatenate([np.concatenate(parts[f]) for f in range(g.n_wf + 1)] + [np.zeros(1)])
    np.testing.assert_array_equal(cat, full)
    dcat = np.concatenate([np.concatenate(dparts[f]) for f in range(g.n_wf + 1)] + [np.zeros(1)])
    np.testing.assert_array_equal(dcat, dfull)
    np.testing.assert_array_equal(np.concatenate(wparts), wfull)


def test_host_generator_matches_oracle_c_and_numpy():
    g = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=50)
    L = orc.OLayout(g.n_v, g.n_p, g.n_wf)
    a = syn.to_reference_order(g, syn.hash_vector(g, 5))
    np.testing.assert_array_equal(a, orc.fill_hash(L, 5))
    np.testing.assert_array_equal(a, orc.fill_hash_np(g.n_wf, g.n_v, g.n_p, 5))


def test_gll_weights():
    for n in range(2, 12):
        w = syn.gll_weights(n)
        assert abs(w.sum() - 2.0) < 1e-13 and np.all(w > 0)


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "nekkrylov.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(nkv_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from nekstab_next_amd import _lib

    lib = _lib.load()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert sorted(_lib.EXPORTED) == syms  # the ctypes table types every declared entry point
    assert lib.nkv_abi_version() == _lib.NKV_ABI_VERSION == 3


def test_header_constants_match_python():
    from nekstab_next_amd import _lib

    txt = open(os.path.join(ROOT, "include", "nekkrylov.h")).read()
    defs = {k: int(v, 0) for k, v in re.findall(r"#define (NKV_[A-Z0-9_]+)\s+(0x[0-9a-f]+|\d+)u?", txt)}
    for name in ("NKV_TILE", "NKV_MAX_COLS", "NKV_ROT_MAX_OUT", "NKV_OK", "NKV_EINVAL", "NKV_EHIP", "NKV_ENAN", "NKV_ESHAPE", "NKV_ECALLBACK",
                 "NKV_TIME", "NKV_ACCUMULATE", "NKV_OVERWRITE", "NKV_NORM2", "NKV_TIME_DOT", "NKV_X_IS_LAST"):
        assert defs[name] == getattr(_lib, name), name


def test_context_rejects_too_many_columns():
    from nekstab_next_amd.vector import NekContext

    with pytest.raises(ValueError, match="max_cols"):
        NekContext(NekLayout(ldim=2, lx1=4, lx2=2, nelgv=4), max_cols=1024)


def test_workspace_size_is_host_only():
    from nekstab_next_amd import _lib

    lib = _lib.load()
    L = box3d_layout(100).c_struct()
    n = lib.nkv_workspace_bytes(ctypes.byref(L), 128)
    assert n >= 256 + 8 * 128


def test_product_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from nekstab_next_amd.vector import NekContext

    with pytest.raises(RuntimeError, match="no CPU fallback"):
        NekContext(NekLayout(ldim=2, lx1=4, lx2=2, nelgv=4))


def test_c_host_example_builds():
    """The plain-C host (examples/c_host: gcc + HIP runtime API + libnekkrylov.so, no Python)
    compiles and links against the header and library as shipped."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(["make", "-s", "-B", "-C", os.path.join(root, "examples", "c_host")], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert os.path.exists(os.path.join(root, "examples", "c_host", "arnoldi_c"))


def test_fortran_host_example_builds():
    """The Fortran host (examples/fortran_host: the bind(C) module of INTEGRATION.md §2 compiled
    with amdflang, linked to libnekkrylov.so) builds against the header's ABI as shipped."""
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(["make", "-s", "-B", "-C", os.path.join(root, "examples", "fortran_host")],
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert os.path.exists(os.path.join(root, "examples", "fortran_host", "arnoldi_f"))


def test_layout_init_matches_neklayout_and_refuses_cht():
    """nkv_layout_init (ABI 3) pads a shard exactly as NekLayout.c_struct does, on the host (no GPU
    call), and refuses nelt != nelv with a dotted scalar: the reference weights
    the scalar over nelt elements with the nelv-element bm1s (krylov_subspace.f90:36-44,
    NEKSTAB:86), so conjugate heat transfer has no reference result.  NekLayout refuses it too."""
    import ctypes

    from nekstab_next_amd import _lib
    from nekstab_next_amd.layout import NekLayout

    lib = _lib.load()
    for ldim, lx1, lx2, E, ns, ifpo in ((3, 8, 6, 44176, 1, True), (2, 6, 4, 1996, 0, True), (3, 5, 3, 17, 2, True),
                                        (2, 6, 4, 100, 1, False), (3, 8, 6, 0, 1, True)):
        lay = NekLayout(ldim, lx1, lx2, E, ns, ifpo)
        want = lay.c_struct()
        got = _lib.nkv_layout()
        rc = lib.nkv_layout_init(ctypes.byref(got), ldim, lx1, lx2, lay.nelv, lay.nelv, ns, int(ifpo), 1)
        assert rc == _lib.NKV_OK, _lib.last_error()
        for k in ("n_v", "n_p", "sv", "sp", "ld", "n_wf", "rank0"):
            assert getattr(got, k) == getattr(want, k), (k, ldim, lx1, E)
    bad = _lib.nkv_layout()
    assert lib.nkv_layout_init(ctypes.byref(bad), 3, 8, 6, 100, 120, 1, 1, 1) == _lib.NKV_ESHAPE
    assert "conjugate heat transfer" in _lib.last_error()
    # without a dotted scalar the temperature mesh is irrelevant to the dot
    assert lib.nkv_layout_init(ctypes.byref(bad), 3, 8, 6, 100, 120, 0, 1, 1) == _lib.NKV_OK
    assert lib.nkv_layout_init(ctypes.byref(bad), 4, 8, 6, 100, 100, 0, 1, 1) == _lib.NKV_EINVAL
    with pytest.raises(ValueError, match="conjugate heat transfer"):
        NekLayout(3, 8, 6, 100, 1, nelgt=120)
    NekLayout(3, 8, 6, 100, 0, nelgt=120)   # no dotted scalar: accepted
    assert NekLayout(3, 8, 6, 100, 1, nelgt=100).shard(1, 2).nelgt == 100
