"""Host-side restart logic: the product's Python restatement (nekstab_next_amd.lapack) against the
oracle's independent C transliteration of the same Fortran (CPU only)."""
import numpy as np
import pytest

import oracle as orc
from nekstab_next_amd import lapack


@pytest.fixture
def same_lapack():
    """Bit-equality of the two restatements of the code AROUND LAPACK (conjugate assembly,
    sort_eigendecomp, select) needs both sides on one library: the oracle runs on the product's
    OpenBLAS here.  Product-on-OpenBLAS vs oracle-on-MKL is tests/test_lapack_split.py."""
    prev = orc.use_lapack("openblas")
    yield
    orc.use_lapack(prev)


def _spectrum(rng, n, pairs=True, ties=False):
    vals = []
    while len(vals) < n:
        r = rng.uniform(0.0, 1.0)
        if pairs and len(vals) <= n - 2 and rng.random() < 0.4:
            t = rng.uniform(0.1, 3.0)
            vals += [r * np.exp(1j * t), r * np.exp(-1j * t)]
        else:
            vals.append(complex(rng.choice([-1, 1]) * r, 0.0))
    v = np.asarray(vals[:n])
    if ties:
        v[: n // 3] = np.round(v[: n // 3].real, 1)
    return v


@pytest.mark.parametrize("n", [1, 2, 3, 7, 8, 9, 16, 33, 64, 100, 128, 200])
def test_quicksort2_python_equals_c(n):
    rng = np.random.default_rng(n)
    for t in range(30):
        arr = rng.integers(0, 5, n).astype(float) if t % 3 == 0 else rng.random(n)
        idx_c, _ = orc.quicksort2(arr)
        np.testing.assert_array_equal(lapack.quicksort2(arr), idx_c)


def test_quicksort2_small_n_sorts_and_known_quirk():
    rng = np.random.default_rng(1)
    for n in range(1, 8):  # below the insertion-sort threshold the result is a true argsort
        a = rng.random(n)
        assert np.all(np.diff(a[lapack.quicksort2(a)]) >= 0)
    # n >= 8: the partition overwrites the pivot slot (utils.f90:106-109) -> index 1 lost, 0 doubled
    x = np.array([3.0, 1.0, 2.0, 0.5, 7.0, 6.0, 5.0, 4.0])
    assert lapack.quicksort2(x).tolist() == [3, 2, 0, 0, 7, 6, 5, 4]


@pytest.mark.parametrize("k", [10, 16, 24, 64, 128])
@pytest.mark.parametrize("nev", [1, 2, 5])
def test_select_eigenvalues_python_equals_c(k, nev):
    rng = np.random.default_rng(k * 10 + nev)
    for t in range(20):
        vals = _spectrum(rng, k, pairs=(t % 2 == 0), ties=(t % 5 == 0))
        s_c, c_c = orc.select_eigenvalues(vals, 0.1, nev)
        s_p, c_p = lapack.select_eigenvalues(vals, 0.1, nev)
        np.testing.assert_array_equal(s_p, s_c)
        assert c_p == c_c


def test_select_eigenvalues_real_boundary_quirk():
    """Two real eigenvalues at the nev+4 boundary: 0 == -0 selects one more (eigensolvers.f90:747)."""
    vals = np.array([0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7], dtype=complex)
    sel, cnt = lapack.select_eigenvalues(vals, 0.1, 1, faithful=False)
    assert cnt == 6  # nev+4 = 5 largest + 1 via the imaginary-part equality
    sel_c, cnt_c = orc.select_eigenvalues(vals, 0.1, 1)
    assert cnt_c == cnt


@pytest.mark.parametrize("n", [5, 16, 40])
def test_eig_and_sort_python_equals_oracle(n, same_lapack):
    rng = np.random.default_rng(n)
    A = np.triu(rng.standard_normal((n, n)), -1)  # upper Hessenberg
    v1, V1 = lapack.eig(A)
    v2, V2 = orc.eig(A)
    np.testing.assert_array_equal(v1, v2)
    np.testing.assert_array_equal(V1, V2)
    # eigen-relation A V = V diag(v)
    assert np.max(np.abs(A @ V1 - V1 * v1)) < 1e-10 * max(1, np.abs(v1).max())
    assert np.all(np.diff(np.abs(v1)) <= 1e-15)


def test_schur_ordschur_lstsq(same_lapack):
    rng = np.random.default_rng(3)
    n = 20
    A = np.triu(rng.standard_normal((n, n)), -1) * 0.3
    A[0, 0] = 0.98
    T, Z, vals = lapack.schur(A)
    T2, Z2, vals2 = orc.schur_sorted(A)
    np.testing.assert_array_equal(T, T2)
    np.testing.assert_array_equal(Z, Z2)
    assert np.max(np.abs(Z @ T @ Z.T - A)) < 1e-12
    sel, cnt = lapack.select_eigenvalues(vals, 0.1, 2)
    Ts, Zs, m = lapack.ordschur(T, Z, sel)
    Ts2, Zs2 = orc.ordschur(T2, Z2, sel)
    np.testing.assert_array_equal(Ts, Ts2)
    assert m == cnt
    assert np.max(np.abs(Zs @ Ts @ Zs.T - A)) < 1e-12
    B = rng.standard_normal((n + 1, n))
    b = rng.standard_normal(n + 1)
    np.testing.assert_allclose(lapack.lstsq(B, b), np.linalg.lstsq(B, b, rcond=None)[0], rtol=1e-10)
    np.testing.assert_array_equal(lapack.lstsq(B, b), orc.lstsq(B, b))


@pytest.mark.parametrize("n", [2, 5, 16, 64, 128])
def test_sort_eigendecomp_python_equals_c(n):
    """sort_eigendecomp (lapack_wrapper.f90:181-228): exchange sort by |lambda|, strict <, columns
    of the eigenvector matrix moved with their values — product vs the oracle's C, bit for bit,
    conjugate pairs (equal moduli) keeping LAPACK's order."""
    rng = np.random.default_rng(n)
    for _ in range(10):
        vals = _spectrum(rng, n, ties=True)
        vecs = rng.standard_normal((n, n)) + 1j * rng.standard_normal((n, n))
        v1, e1 = lapack.sort_eigendecomp(vals.copy(), vecs.copy())
        v2, e2 = orc.sort_eigendecomp(vals.copy(), vecs.copy())
        np.testing.assert_array_equal(v1, v2)
        np.testing.assert_array_equal(e1, e2)


def test_breakdown_column_rule():
    """Invariant-subspace detection on the host H (krylov_schur.breakdown_column): the first Arnoldi
    column from ``c0`` whose subdiagonal is below tol x its column norm, or that is non-finite."""
    from nekstab_next_amd.krylov_schur import breakdown_column

    k = 6
    H = np.triu(np.ones((k + 1, k)), -1)
    assert breakdown_column(H, 0, k, 1e-8) == -1
    H[4, 3] = 1e-12
    assert breakdown_column(H, 0, k, 1e-8) == 3
    assert breakdown_column(H, 4, k, 1e-8) == -1      # columns before c0 are the restart block
    assert breakdown_column(H, 0, k, 1e-13) == -1
    H[2, 1] = np.nan
    assert breakdown_column(H, 0, k, 1e-8) == 1
    H[2, 1] = 1.0
    H[:, 5] = 0.0
    assert breakdown_column(H, 4, k, 1e-8) == 5


def test_givens_residual_equals_least_squares_residual():
    """gmres.GivensResidual: the O(k)-per-column residual of the GMRES least-squares problem equals
    ||beta e_1 - H y|| with y from dgels (lapack.lstsq, the reference's newton_krylov.f90:255-258)
    at every column, including an exactly zero subdiagonal (lucky breakdown: residual 0)."""
    from nekstab_next_amd import lapack
    from nekstab_next_amd.gmres import GivensResidual

    rng = np.random.default_rng(3)
    for trial in range(20):
        k = int(rng.integers(1, 60))
        H = np.triu(rng.standard_normal((k + 1, k)), -1)
        H[np.arange(1, k + 1), np.arange(k)] = np.abs(H[np.arange(1, k + 1), np.arange(k)]) * 10.0 ** rng.uniform(-6, 0, k)
        beta = float(rng.uniform(0.1, 10))
        e = np.zeros(k + 1)
        e[0] = beta
        g = GivensResidual(beta, k)
        for c in range(1, k + 1):
            got = g.add_column(H[: c + 1, c - 1])
            y = lapack.lstsq(np.asfortranarray(H[: c + 1, :c]), e[: c + 1])
            ref = float(np.linalg.norm(e[: c + 1] - H[: c + 1, :c] @ y))
            assert abs(got - ref) <= 1e-12 * beta + 1e-10 * ref, (trial, c, got, ref)
    H = np.array([[2.0, 1.0], [0.0, 3.0], [0.0, 0.0]])   # H(2,1) = 0: exact after one column
    g = GivensResidual(1.0, 2)
    assert g.add_column(H[:2, 0]) == 0.0


def test_givens_column_rejects_bad_input():
    """nkv_givens_column has no status channel: bad input returns NaN (so a residual test on it never
    passes) and leaves a message in nkv_last_error."""
    from nekstab_next_amd import _lib

    lib = _lib.load()
    a = np.zeros(4)
    p = a.ctypes.data
    assert np.isnan(lib.nkv_givens_column(-1, p, p, p, p))
    assert np.isnan(lib.nkv_givens_column(0, None, p, p, p))
    assert "givens" in _lib.last_error()
    assert not np.isnan(lib.nkv_givens_column(0, p, p, p, p))


def test_residu_newton_fortran_e_format():
    """residu_newton.dat is written (I6,1E15.7) (newton_krylov.f90:109): gfortran's Ew.d form,
    0.ddddddd mantissa and a signed two-digit exponent."""
    from nekstab_next_amd.newton import fortran_e

    assert f"{3:6d}{fortran_e(1.234567e-3, 15, 7)}" == "     3  0.1234567E-02"
    assert fortran_e(0.0, 15, 7) == "  0.0000000E+00"
    assert fortran_e(-2.5, 15, 7) == " -0.2500000E+01"
    assert fortran_e(0.999999999, 15, 7) == "  0.1000000E+01"     # rounding carries into the exponent
    assert fortran_e(4.56e-120, 15, 7) == "  0.4560000-119"       # three-digit exponent drops the E
    assert fortran_e(123.456789, 15, 7) == "  0.1234568E+03"


def test_explicit_reference_order_kept_for_nonorthonormal_bases():
    """A noise/load/symm seed runs modified Gram–Schmidt; an explicit request for the reference's
    own order (mode "mgs2" / "mgs2-native") is kept, not replaced by the lagged or ICWY form
    (ADVICE r3)."""
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import _MGS2, _nonorth_of

    cfg = KrylovSchurConfig()
    assert cfg.nonorth_mode == "mgs2-lagged"
    assert _nonorth_of("mgs2", cfg) == "mgs2" and _nonorth_of("mgs2-native", cfg) == "mgs2-native"
    assert _nonorth_of("dcgs2", cfg) == "mgs2-lagged" and _nonorth_of("dcgs2-native", cfg) == "mgs2-lagged-native"
    # with time in k_dot the restart breaks the Arnoldi relation the lagged form uses: ICWY
    assert _nonorth_of("dcgs2", cfg, time_in_dot=True) == "mgs2-icwy"
    assert _nonorth_of("dcgs2-native", cfg, time_in_dot=True) == "mgs2-icwy-native"
    icwy = KrylovSchurConfig(nonorth_mode="mgs2-icwy")
    assert _nonorth_of("dcgs2", icwy) == "mgs2-icwy" and _nonorth_of("cgs2-native", icwy) == "mgs2-icwy-native"
    assert _nonorth_of("cgs2", KrylovSchurConfig(nonorth_mode="mgs2")) in _MGS2


def test_segment_entry_points_are_noops_on_an_empty_shard():
    """More ranks than elements: a rank's segment-only arrays (the wave-maker's and bf_sensitivity's
    outputs, gradients, seed fields) are empty tensors whose data pointer is NULL.  Those entry
    points return OK on an empty shard before any pointer check or launch (no device is touched,
    so this runs on the CPU) and still reject a NULL pointer on a non-empty one."""
    import ctypes

    from nekstab_next_amd import _lib
    from nekstab_next_amd.layout import cylinder_layout

    from nekstab_next_amd.sensitivity import velocity_layout

    lib = _lib.load()
    lay = velocity_layout(cylinder_layout(2)).shard(0, 3)
    assert lay.n_v == 0 and lay.sv == 0
    L = ctypes.byref(lay.c_struct())
    assert lib.nkv_wavemaker(L, None, None, None, None, None, 2, None) == 0
    assert lib.nkv_gradm1(L, lay.lx1, 2, None, None, None, None, None, 2, 0, None, 0, None) == 0
    assert lib.nkv_bf_sensitivity(L, None, None, None, None, None, None, 2, None) == 0
    assert lib.nkv_mth_rand_add(L, lay.lx1, lay.lx1, 1, 0, None, None, None, 1.0, 1.0, 1.0, None, None) == 0
    assert lib.nkv_symmetric_seed(L, None, None, 1.0, None, None, None, None) == 0
    full = velocity_layout(cylinder_layout(2))
    assert lib.nkv_wavemaker(ctypes.byref(full.c_struct()), None, None, None, None, None, 2, None) != 0
    assert "NULL" in _lib.last_error()


def test_graph_replay_refused_for_host_synchronising_modes():
    """the lagged MGS modes synchronise with the host every step, so a HIP-graph capture
    of their factorisation would fail; FactorizationGraph.usable() refuses them (krylov_schur then
    launches eagerly), and still refuses every mode at world size > 1."""
    from types import SimpleNamespace

    from nekstab_next_amd.arnoldi import FactorizationGraph

    def fg(mode, world=1):
        return FactorizationGraph(SimpleNamespace(comm=SimpleNamespace(world=world)), None, None, None, None, mode)

    for mode in ("mgs2-lagged", "mgs2-lagged-native"):
        assert not fg(mode).usable()
    for mode in ("dcgs2", "cgs2", "mgs2", "mgs2-icwy", "dcgs2-native"):
        assert fg(mode).usable() and not fg(mode, world=2).usable()
