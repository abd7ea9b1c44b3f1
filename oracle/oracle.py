"""CPU oracle for nekStab's Krylov hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product (``nekstab_next_amd``)
never imports it.

What it restates (each function cites the reference line it follows):
* vector algebra, ``update_hessenberg_matrix`` (MGS2), ``k_matmul``, the restart rotation, the
  ordering rules ``quicksort2`` / ``select_eigenvalues`` / ``sort_eigendecomp``: plain C in
  ``nekstab_oracle.c`` (reference operation order, no FP contraction);
* the drivers ``arnoldi_factorization``, ``krylov_schur``, ``schur_condensation``, ``eig``,
  ``ts_gmres``, ``biorthogonalize``, ``wave_maker``, ``bf_sensitivity`` (with Nek5000's
  ``gradm1``), the legacy ``matvec`` dispatcher,
  ``ts_steady_force_sensitivity``, ``newton_krylov``, the seed noise ``mth_rand`` with its
  direct-stiffness averaging: this file, calling Intel MKL (``mkl_lapack.py``: the LAPACK the
  reference's build links, bin/mks:32-44) for dgeev / dgees / dtrsen / dgels with the reference's
  arguments and workspace sizes.  The product calls SciPy's OpenBLAS, so the dense half of every
  product-vs-oracle check compares two independent LAPACK implementations.
  ``NEKSTAB_ORACLE_LAPACK=openblas`` (or ``use_lapack("openblas")``) runs the oracle on SciPy's
  OpenBLAS instead: the fixtures record both side by side (tests/golden/make_golden.py).

Parity status: **parity unpinned** against reference outputs.  The reference ships no tests or
golden vectors for this path, and its Fortran cannot be built here without
writing stand-ins for Nek5000's SIZE/TOTAL include files and routines (glsc3, rzero, ...), which
this build does not do.  The restatement is pinned instead to closed-form known answers
(synthetic operators with exact spectra / exact solutions, tests/test_oracle_known_answers.py)
and to fixtures it generated (tests/golden/).
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_double, c_int, c_int32, c_int64, c_uint64

import numpy as np
from scipy.linalg import lapack as _lp

import mkl_lapack as _mkl

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")


class orc_layout(Structure):
    _fields_ = [("nv", c_int64), ("np", c_int64), ("nwf", c_int32), ("time_in_dot", c_int32)]


_D = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_I = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_LP = POINTER(orc_layout)

_SIGS = {
    "orc_set_threads": (None, [c_int]),
    "orc_max_threads": (c_int, []),
    "orc_vector_len": (c_int64, [_LP]),
    "orc_glsc3": (c_double, [_D, _D, _D, c_int64]),
    "orc_k_dot": (c_double, [_LP, _D, _D, _D]),
    "orc_real_dot": (c_double, [_LP, _D, _D, _D]),
    "orc_k_cmult": (None, [_LP, _D, c_double]),
    "orc_k_add2": (None, [_LP, _D, _D]),
    "orc_k_sub2": (None, [_LP, _D, _D]),
    "orc_k_sub3": (None, [_LP, _D, _D, _D]),
    "orc_k_zero": (None, [_LP, _D]),
    "orc_k_copy": (None, [_LP, _D, _D]),
    "orc_real_axpby": (None, [_LP, _D, c_double, _D, c_double]),
    "orc_update_hessenberg": (None, [_LP, _D, _D, _D, _D, c_int, _D]),
    "orc_k_matmul": (None, [_LP, _D, _D, _D, c_int]),
    "orc_rotate": (None, [_LP, _D, c_int, _D]),
    "orc_op_diag": (None, [_LP, _D, _D, _D, c_double]),
    "orc_fill_hash": (None, [_LP, _D, c_uint64, c_int64, c_int64]),
    "orc_quicksort2": (None, [c_int, _D, _I]),
    "orc_select_eigenvalues": (c_int, [c_int, _D, _D, c_double, c_int, _I]),
    "orc_sort_eigendecomp": (None, [c_int, _D, _D, _D, _D]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(_LIB_PATH)
        for k, (r, a) in _SIGS.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def set_threads(n: int) -> None:
    lib().orc_set_threads(int(n))


_prod = None


def prod_lib():
    """The same restatement built with the reference's deployment flags (-Ofast -ffast-math,
    bin/mks:53-55): the timed CPU baseline only (bench.py).  Reassociated sums, so never the
    parity checker."""
    global _prod
    if _prod is None:
        path = os.path.join(_HERE, "liboracle_prod.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(path)
        for k, (r, a) in _SIGS.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _prod = L
    return _prod


_cgs2 = None


def cgs2_lib():
    """The timed "optimised CPU" line (oracle/cpu_cgs2.c: blocked OpenMP CGS2) — bench.py only."""
    global _cgs2
    if _cgs2 is None:
        path = os.path.join(_HERE, "libcpucgs2.so")
        if not os.path.exists(path):
            import subprocess

            subprocess.run(["make", "-s", "-C", _HERE], check=True)
        L = ctypes.CDLL(path)
        L.cpu_cgs2_set_threads.restype, L.cpu_cgs2_set_threads.argtypes = None, [c_int]
        L.cpu_cgs2_update_hessenberg.restype = None
        L.cpu_cgs2_update_hessenberg.argtypes = [_LP, _D, _D, _D, _D, c_int, _D]
        _cgs2 = L
    return _cgs2


class OLayout:
    """Unpadded reference layout [vx | vy | (vz) | t.. | pr | time] of one shard."""

    def __init__(self, nv: int, np_: int, nwf: int, time_in_dot: bool = False, ldim: int | None = None):
        self.c = orc_layout(nv, np_, nwf, int(time_in_dot))
        self.nv, self.np, self.nwf = nv, np_, nwf
        self.ldim = ldim if ldim is not None else min(nwf, 3)
        self.n = nwf * nv + np_
        self.len = self.n + 1

    @classmethod
    def from_nek(cls, ldim, lx1, lx2, nelv, n_scalars=0, ifpo=True, time_in_dot=False):
        return cls(lx1 ** ldim * nelv, (lx2 ** ldim * nelv) if ifpo else 0, ldim + n_scalars, time_in_dot, ldim)

    def zeros(self, k=None):
        return np.zeros(self.len if k is None else (k, self.len))


# ---- vector ops ---------------------------------------------------------------------------------

def k_dot(L: OLayout, w, p, q) -> float:
    return lib().orc_k_dot(ctypes.byref(L.c), w, p, q)


def real_dot(L: OLayout, w, p, q) -> float:
    return lib().orc_real_dot(ctypes.byref(L.c), w, p, q)


def k_normalize(L: OLayout, w, p) -> float:
    a = float(np.sqrt(k_dot(L, w, p, p)))
    lib().orc_k_cmult(ctypes.byref(L.c), p, 1.0 / a)
    return a


def fill_hash(L: OLayout, seed: int, voff: int = 0, poff: int = 0) -> np.ndarray:
    x = L.zeros()
    lib().orc_fill_hash(ctypes.byref(L.c), x, int(seed) & (2**64 - 1), int(voff), int(poff))
    return x


def fill_hash_np(nwf, nv, np_, seed, voff=0, poff=0) -> np.ndarray:
    """Pure-numpy twin of orc_fill_hash (vectorised uint64 arithmetic)."""
    M = np.uint64(0xFFFFFFFFFFFFFFFF)

    def mix(z):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))

    with np.errstate(over="ignore"):
        key0 = np.uint64((int(seed) * 0xD1342543DE82EF95) & int(M))
        out = []
        for f in range(nwf):
            g = np.arange(voff, voff + nv, dtype=np.uint64)
            z = mix(key0 + np.uint64((f * 0x9E3779B97F4A7C15) & int(M)) + g)
            out.append(2.0 * ((z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53) - 1.0)
        g = np.arange(poff, poff + np_, dtype=np.uint64)
        z = mix(key0 + np.uint64((31 * 0x9E3779B97F4A7C15) & int(M)) + g)
        out.append(2.0 * ((z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53) - 1.0)
    return np.concatenate(out + [np.zeros(1)])


# ---- ordering rules (C transliteration) ---------------------------------------------------------

def quicksort2(arr):
    a = np.ascontiguousarray(arr, dtype=np.float64).copy()
    idx = np.arange(1, a.size + 1, dtype=np.int32)
    lib().orc_quicksort2(a.size, a, idx)
    return idx - 1, a


def select_eigenvalues(vals, delta, nev):
    re = np.ascontiguousarray(vals.real, dtype=np.float64)
    im = np.ascontiguousarray(vals.imag, dtype=np.float64)
    sel = np.zeros(vals.size, dtype=np.int32)
    cnt = lib().orc_select_eigenvalues(vals.size, re, im, float(delta), int(nev), sel)
    return sel.astype(bool), int(cnt)


def sort_eigendecomp(vals, vecs):
    n = vals.size
    re, im = vals.real.copy(), vals.imag.copy()
    vre = np.ascontiguousarray(vecs.real.T).copy()  # column-major -> rows are columns
    vim = np.ascontiguousarray(vecs.imag.T).copy()
    lib().orc_sort_eigendecomp(n, re, im, vre, vim)
    return re + 1j * im, (vre + 1j * vim).T


# ---- dense steps (lapack_wrapper.f90) -----------------------------------------------------------

_LAPACK = os.environ.get("NEKSTAB_ORACLE_LAPACK", "mkl").lower()
if _LAPACK not in ("mkl", "openblas"):
    raise ValueError(f"NEKSTAB_ORACLE_LAPACK={_LAPACK!r}: expected 'mkl' or 'openblas'")


def lapack_name() -> str:
    """The LAPACK the oracle's dense steps run on: ``"mkl"`` (default) or ``"openblas"``."""
    return _LAPACK


def use_lapack(name: str) -> str:
    """Switch the oracle's LAPACK; returns the previous choice."""
    global _LAPACK
    name = name.lower()
    if name not in ("mkl", "openblas"):
        raise ValueError(name)
    prev, _LAPACK = _LAPACK, name
    return prev


def lapack_version() -> str:
    if _LAPACK == "mkl":
        return _mkl.version()
    import scipy

    return f"SciPy {scipy.__version__} OpenBLAS"


def _dgeev(A):
    n = A.shape[0]
    if _LAPACK == "mkl":
        return _mkl.dgeev(A)
    wr, wi, _, vr, info = _lp.dgeev(np.array(A, order="F", copy=True), compute_vl=0, compute_vr=1, lwork=4 * n)
    return wr, wi, vr, info


def eig(A):
    """lapack_wrapper.f90:114-177: dgeev('N','V', lwork=4n) on a copy, conjugate-pair assembly,
    sort_eigendecomp."""
    n = A.shape[0]
    wr, wi, vr, info = _dgeev(A)
    assert info == 0, info
    vecs = np.array(vr, dtype=np.complex128)
    i = 0
    while i < n - 1:  # do i = 1, n-1 with the same two branches
        if wi[i] > 0:
            vecs[:, i] = vr[:, i] + 1j * vr[:, i + 1]
            vecs[:, i + 1] = vr[:, i] - 1j * vr[:, i + 1]
        elif wi[i] == 0:
            vecs[:, i] = vr[:, i]
        i += 1
    return sort_eigendecomp(wr + 1j * wi, vecs)


def schur_sorted(A):
    """lapack_wrapper.f90:3-55: dgees('V','S', select_eigvals: sqrt(wr**2+wi**2) > 0.9, lwork=3n).
    ``info`` is ignored, as the reference does."""
    n = A.shape[0]
    if _LAPACK == "mkl":
        t, vs, wr, wi, _sdim, _info = _mkl.dgees(A)
    else:
        t, _, wr, wi, vs, _, _info = _lp.dgees(lambda a, b: int(np.sqrt(a ** 2 + b ** 2) > 0.9),
                                               np.array(A, order="F", copy=True), compute_v=1, sort_t=1,
                                               lwork=3 * n)
    return np.array(t, order="F"), np.array(vs, order="F"), wr + 1j * wi


def ordschur(T, Z, selected):
    """lapack_wrapper.f90:59-111: dtrsen('N','V'), lwork=n, liwork=1."""
    n = T.shape[0]
    if _LAPACK == "mkl":
        ts, qs, _m, info = _mkl.dtrsen(T, Z, selected)
    else:
        ts, qs, _, _, _m, _, _, info = _lp.dtrsen(selected.astype(np.int32), T, Z, job="N", wantq=1, lwork=n,
                                                  liwork=1)
    assert info == 0, info
    return np.array(ts, order="F"), np.array(qs, order="F")


def lstsq(A, b):
    """lapack_wrapper.f90:248-300: dgels('N'), lwork=2mn; x = b_tilde(1:n)."""
    m, n = A.shape
    if _LAPACK == "mkl":
        x, _info = _mkl.dgels(A, b)
        return x
    _, x, info = _lp.dgels(np.array(A, order="F", copy=True), np.array(b, copy=True), trans="N", lwork=2 * m * n)
    return np.array(x[:n])


# ---- drivers ------------------------------------------------------------------------------------

def arnoldi_factorization(L: OLayout, w, matvec, Q, H, mstart, mend):
    """krylov_decomposition.f90:2-99 with update_hessenberg_matrix in C.  Q: (k+1, L.len) array;
    H: (k+1, k) array, columns written in place (1-based mstart..mend)."""
    f = L.zeros()
    wrk = L.zeros()
    for mstep in range(mstart, mend + 1):
        matvec(Q[mstep - 1], f)
        col = np.zeros(mstep + 1)
        lib().orc_update_hessenberg(ctypes.byref(L.c), w, col, f, np.ascontiguousarray(Q[:mstep]), mstep, wrk)
        H[: mstep + 1, mstep - 1] = col
        Q[mstep] = f


def schur_condensation(L: OLayout, H, Q, k, schur_del, schur_tgt):
    """eigensolvers.f90:363-468.  Returns (mstart, selected)."""
    b_vec = np.zeros(k)
    b_vec[k - 1] = H[k, k - 1]
    T, vecs, vals = schur_sorted(H[:k, :k])
    selected, ms = select_eigenvalues(vals, schur_del, schur_tgt)
    T, vecs = ordschur(T, vecs, selected)
    H[:k, :k] = T
    H[:ms, ms:k] = 0.0
    H[ms:k + 1, :] = 0.0
    Qk = np.ascontiguousarray(Q[:k])
    lib().orc_rotate(ctypes.byref(L.c), Qk, k, np.ascontiguousarray(vecs.ravel(order="F")))
    Q[:k, :L.n] = Qk[:, :L.n]
    H[ms, :] = b_vec @ vecs
    mstart = ms + 1
    Q[mstart - 1, :L.n] = Q[k, :L.n]  # nopcopy: fields only
    return mstart, selected


def krylov_schur(L: OLayout, w, matvec, q1, k_dim, schur_tgt, eigen_tol=1e-6, schur_del=0.1, max_restarts=1000,
                 on_step=None, start=None, stop_after=None):
    """eigensolvers.f90:120-359 from a given first Krylov vector q1 (already normalised by the
    caller as prepare_seed does, linear_stab.f90:287-291).

    ``on_step(k, Q, H)``: called after Arnoldi step k (``if (ifres) call arnoldi_checkpoint``,
    krylov_decomposition.f90:84; nekio.checkpoint_writer).  ``start=(mstart, H, Qs)``: the restart
    branch (``uparam(2) = mstart > 0``, eigensolvers.f90:240-285): H and Q(1..mstart+1) as read from
    the files, then ``mstart = mstart + 1`` (:281) and the factorisation continues; ``q1`` is then
    ignored.  ``stop_after``: end the run after that Arnoldi step (a job killed mid-run)."""
    Q = np.zeros((k_dim + 1, L.len))
    H = np.zeros((k_dim + 1, k_dim))
    mstart, schur_cnt = 1, 0
    if start is None:
        Q[0] = q1
    else:
        ms, H0, Qs = start
        H[...] = H0
        Q[: ms + 1] = Qs[: ms + 1]
        mstart = ms + 1
    hist = dict(mstart=[], cnt=[], selected=[], H_first=None, H_restart=[])
    while True:
        if on_step is None and stop_after is None:
            arnoldi_factorization(L, w, matvec, Q, H, mstart, k_dim)
        else:
            for mstep in range(mstart, k_dim + 1):
                arnoldi_factorization(L, w, matvec, Q, H, mstep, mstep)
                if on_step is not None:
                    on_step(mstep, Q, H)
                if stop_after is not None and mstep >= stop_after:
                    return dict(stopped_at=mstep, Q=Q, H=H)
        if hist["H_first"] is None:
            hist["H_first"] = H.copy()
        vals, vecs = eig(H[:k_dim, :k_dim])
        residual = np.abs(H[k_dim, k_dim - 1] * vecs[k_dim - 1, :])
        cnt = int(np.count_nonzero(residual < eigen_tol))
        hist["cnt"].append(cnt)
        if schur_tgt <= 0 or cnt >= schur_tgt or schur_cnt >= max_restarts:
            break
        schur_cnt += 1
        hist["H_restart"].append(H.copy())   # the (k+1) x k matrix schur_condensation starts from
        mstart, sel = schur_condensation(L, H, Q, k_dim, schur_del, schur_tgt)
        hist["mstart"].append(mstart)
        hist["selected"].append(sel)
    return dict(vals=vals, vecs=vecs, residual=residual, converged=cnt, schur_cnt=schur_cnt, H=H, Q=Q, **hist)


def outpost_mode(L: OLayout, w, Q, vecs, i, k):
    """Eigenmode i as outpost_ks assembles it (eigensolvers.f90:565-585, 603-613):
    ``fp = matmul(q(:, 1:k), vecs(:, i))`` field by field in complex arithmetic — with a real basis
    the real and imaginary parts are the two real combinations Q y_re and Q y_im, summed over the
    columns in ascending order (k_matmul's order); ``norm`` of each part (sqrt of
    ``inner_product``: glsc3 with bm1s over vx, vy, [vz], t — pressure not dotted, :2-75);
    beta = 1/sqrt(alpha_r^2 + alpha_i^2) applied by ``nopcmult`` to every field incl. pressure.
    Returns (re, im, alpha_r, alpha_i) in reference order; the time slot stays 0 (a mode carries
    no time component)."""
    c = ctypes.byref(L.c)
    Qk = np.ascontiguousarray(Q[:k])
    re, im = L.zeros(), L.zeros()
    lib().orc_k_matmul(c, re, Qk, np.ascontiguousarray(vecs[:k, i].real), k)
    lib().orc_k_matmul(c, im, Qk, np.ascontiguousarray(vecs[:k, i].imag), k)
    re[-1] = im[-1] = 0.0
    nt = OLayout(L.nv, L.np, L.nwf, False, L.ldim)   # inner_product never includes time
    ar = float(np.sqrt(k_dot(nt, w, re, re)))
    ai = float(np.sqrt(k_dot(nt, w, im, im)))
    beta = 1.0 / np.sqrt(ar ** 2 + ai ** 2)
    lib().orc_k_cmult(c, re, beta)
    lib().orc_k_cmult(c, im, beta)
    re[-1] = im[-1] = 0.0
    return re, im, ar, ai


def get_vec(L: OLayout, Q, coeffs, k):
    """LightKrylov ``get_vec(vec, X(1:k), coeffs)`` as nekStab calls it (linear_stab.f90:362,372):
    vec = X(1:k) coeffs, real coefficients, the fields only (k_matmul order); time slot 0."""
    out = L.zeros()
    lib().orc_k_matmul(ctypes.byref(L.c), out, np.ascontiguousarray(Q[:k]), np.ascontiguousarray(coeffs[:k]), k)
    out[-1] = 0.0
    return out


def prepare_seed(L: OLayout, w, seed):
    """linear_stab.f90:287-291: X(1) = seed / sqrt(real_dot(seed, seed))."""
    x = seed.copy()
    a = np.sqrt(real_dot(L, w, x, x))
    lib().orc_k_cmult(ctypes.byref(L.c), x, 1.0 / a)
    return x


def ts_gmres(L: OLayout, w, matvec, rhs, maxiter, ksize, tol, findiff=False):
    """newton_krylov.f90:170-299 (+ initialize_gmres_vector :303-326).  Returns (sol, history)."""
    c = ctypes.byref(L.c)
    Q = np.zeros((ksize + 1, L.len))
    sol = L.zeros()
    Q[0] = rhs
    beta = k_normalize(L, w, Q[0])
    hist = dict(inner=[], outer=[], y=[])
    for _it in range(maxiter):
        H = np.zeros((ksize + 1, ksize))
        yvec = np.zeros(ksize)
        evec = np.zeros(ksize + 1)
        evec[0] = beta
        Q[1:] = 0.0
        k_used = ksize
        for k in range(1, ksize + 1):
            arnoldi_factorization(L, w, matvec, Q, H, k, k)
            yvec[:k] = lstsq(H[: k + 1, :k], evec[: k + 1])
            beta = float(np.linalg.norm(evec[: k + 1] - H[: k + 1, :k] @ yvec[:k]))
            hist["inner"].append(beta ** 2)
            k_used = k
            if beta ** 2 < tol or (findiff and beta ** 2 < 1e-8):
                break
        hist["y"].append(yvec[:k_used].copy())
        dq = L.zeros()
        lib().orc_k_matmul(c, dq, np.ascontiguousarray(Q[:k_used]), np.ascontiguousarray(yvec[:k_used]), k_used)
        lib().orc_k_add2(c, sol, dq)
        # initialize_gmres_vector(beta, Q(1)=sol, rhs): f = -(A sol - rhs); normalise
        Q[0] = sol
        f = L.zeros()
        matvec(Q[0], f)
        lib().orc_k_sub2(c, f, rhs)
        lib().orc_k_cmult(c, f, -1.0)
        beta = k_normalize(L, w, f)
        Q[0] = f
        hist["outer"].append(beta ** 2)
        if beta ** 2 < tol or (findiff and beta ** 2 < 1e-6):
            break
    return sol, hist


def legacy_matvec(L: OLayout, w, mode, fwd, adj, f, q, fd=None, b_fc=None, b_ic=None):
    """The legacy dispatcher ``matvec(f, q)`` on ``uparam(1) = mode`` (matvec.f90:56-146) over
    reference-order vectors; ``fwd`` / ``adj`` / ``fd`` are the forward, adjoint and finite-difference
    maps ``m(x, y)``.  Returns evop.  Mode 2.x is newton_linearized_map (:520-571): f = Phi'(q) - q
    (k_sub2, time included), and for 2.1 (the UPO period row) f += b_fc * q%time, then
    f%time = k_dot(b_ic, q) — compute_bvec's vectors carry time = 0 (:610); otherwise f%time = 0."""
    c = ctypes.byref(L.c)
    fwd_or_fd = fd if fd is not None else fwd
    if 3.0 <= mode < 3.2:
        fwd_or_fd(q, f)
        return "d"
    if 3.2 <= mode < 3.3:
        adj(q, f)
        return "a"
    if 3.3 <= mode < 3.4:       # transient_growth_map :478-495
        wrk = L.zeros()
        fwd(q, wrk)
        adj(wrk, f)
        return "p"
    if int(np.floor(mode)) == 4:  # ts_force_sensitivity_map :499-516
        adj(q, f)
        lib().orc_k_sub2(c, f, q)
        lib().orc_k_cmult(c, f, -1.0)
        return None
    if int(np.floor(mode)) == 2:
        fwd_or_fd(q, f)
        lib().orc_k_sub2(c, f, q)
        if mode == 2.1:
            bvec = b_fc * q[-1]
            bvec[-1] = 0.0
            lib().orc_k_add2(c, f, np.ascontiguousarray(bvec))
            bic = np.array(b_ic, dtype=np.float64)
            bic[-1] = 0.0
            f[-1] = k_dot(L, w, bic, q)
        else:
            f[-1] = 0.0
        return "n"
    raise ValueError(f"uparam(1)={mode} selects no map")


def ts_steady_force_sensitivity(L: OLayout, w, adj, rhs, k_dim, tol, part="r", recast=None):
    """sensitivity.f90:273-346 after the load: ``rhs`` holds the forcing's velocity (other fields 0);
    recast (the forced run, :331), k_normalize (:334), ts_gmres(rhs, sol, 10, k_dim) on the mode-4
    map of ``matvec`` (:337, matvec.f90:134-136, 499-516), sol *= alpha (:340).  Returns (sol, hist,
    alpha)."""
    rhs = np.array(rhs, dtype=np.float64)
    if recast is not None:
        recast(rhs)
    alpha = k_normalize(L, w, rhs)
    mode = 4.41 if part == "r" else 4.42
    sol, hist = ts_gmres(L, w, lambda x, y: legacy_matvec(L, w, mode, None, adj, y, x), rhs, 10, k_dim, tol)
    lib().orc_k_cmult(ctypes.byref(L.c), sol, alpha)
    return sol, hist, alpha


def newton_krylov(L: OLayout, w, nonlinear, linearized, q, tol, maxiter, ksize, gmres_maxiter=100, mode=2.0,
                  gmres_tol=None):
    """newton_krylov.f90:1-166 without the dynamic tolerance: f = F(q) (:97), residual = k_norm**2
    (:102), exit below tol (:112), ts_gmres(f, dq, 100, k_dim) on newton_linearized_map about q
    (:120, matvec.f90:520-571 via legacy_matvec), q = q - dq (k_sub2, :125).  ``linearized(q)``
    returns the forward map m(x, y) of the linearisation about q.  Returns (q, residuals, gmres
    histories)."""
    q = np.array(q, dtype=np.float64)
    c = ctypes.byref(L.c)
    residuals, hists = [], []
    for _i in range(maxiter):
        f = L.zeros()
        nonlinear(q, f)
        r = k_dot(L, w, f, f)
        residuals.append(r)
        if r < tol:
            break
        fwd = linearized(q)
        dq, hist = ts_gmres(L, w, lambda x, y: legacy_matvec(L, w, mode, fwd, None, y, x), f, gmres_maxiter, ksize,
                            tol if gmres_tol is None else gmres_tol)
        hists.append(hist)
        lib().orc_k_sub2(c, q, dq)
    return q, residuals, hists


def biorthogonalize(L: OLayout, w, dRe, dIm, aRe, aIm):
    """sensitivity.f90:393-469.  Inputs are modified copies; returns (dRe, dIm, aRe, aIm).

    The direct mode is normalised with opcmult (velocities only, not pressure/scalars, :429-430);
    inner products use the weighted fields (inner_product, eigensolvers.f90:3-56)."""
    dRe, dIm, aRe, aIm = (x.copy() for x in (dRe, dIm, aRe, aIm))
    ip = lambda p, q: k_dot(OLayout(L.nv, L.np, L.nwf, False, L.ldim), w, p, q)  # noqa: E731
    alpha = ip(dRe, dRe)
    beta = ip(dIm, dIm)
    gamma = 1.0 / np.sqrt(alpha + beta)
    nvel = L.ldim * L.nv
    dRe[:nvel] *= gamma
    dIm[:nvel] *= gamma
    alpha = ip(aRe, dRe)
    beta = ip(aIm, dIm)
    gamma = alpha + beta
    alpha = ip(aRe, dIm)
    beta = ip(aIm, dRe)
    delta = alpha - beta
    den = gamma ** 2 + delta ** 2
    n = L.n
    r = (gamma * aRe[:n] - delta * aIm[:n]) / den
    i = (gamma * aIm[:n] + delta * aRe[:n]) / den
    aRe[:n], aIm[:n] = r, i
    return dRe, dIm, aRe, aIm


def wavemaker_pointwise(L: OLayout, dRe, dIm, aRe, aIm):
    """sensitivity.f90:69-71 on reference-order vectors (velocity components c < ldim):
    wk1 = sqrt(vx_dRe**2 + vx_dIm**2 + vy_dRe**2 + ...), wk2 likewise for the adjoint mode,
    wavemaker = wk1*wk2.  Left-to-right sums as written (x**2 is the rounded x*x).  The 2-D
    reference adds its uninitialised vz_* arrays (never copied when .not. if3D, :45-60); they are
    taken as absent here."""
    nv = L.nv
    seg = lambda x, c: x[c * nv:(c + 1) * nv]  # noqa: E731
    wk1 = seg(dRe, 0) ** 2 + seg(dIm, 0) ** 2
    wk2 = seg(aRe, 0) ** 2 + seg(aIm, 0) ** 2
    for c in range(1, L.ldim):
        wk1 = wk1 + seg(dRe, c) ** 2
        wk1 = wk1 + seg(dIm, c) ** 2
        wk2 = wk2 + seg(aRe, c) ** 2
        wk2 = wk2 + seg(aIm, c) ** 2
    return np.sqrt(wk1) * np.sqrt(wk2)


def wave_maker(L: OLayout, w, dRe, dIm, aRe, aIm):
    """sensitivity.f90:3-77 after the four load_fld calls: ``ifto = ifpo = .false.`` (:40), so ``L``
    is the velocity-only layout (the dots, opcmult and nopcopy see vx, vy, [vz]);
    biorthogonalize (:63-66), then the pointwise product (:69-71).  Returns (wavemaker, the four
    bi-orthogonalised vectors)."""
    vecs = biorthogonalize(L, w, dRe, dIm, aRe, aIm)
    return wavemaker_pointwise(L, *vecs), vecs


def gll_derivative(n):
    """The GLL derivative matrix D[i, m] = l_m'(z_i) (Nek5000's dxm1 from dgll), correctly rounded:
    barycentric Lagrange differentiation at 60 digits (mpmath) on nodes refined at that precision
    from the oracle's own (``nekio._gll_nodes``) — an independent route to the matrix the product
    builds from Legendre values in extended precision."""
    import mpmath
    from nekio import _gll_nodes

    with mpmath.workdps(60):
        N = n - 1
        dP = lambda x: mpmath.diff(lambda t: mpmath.legendre(N, t), x)  # noqa: E731
        z = [mpmath.mpf(-1)] + [mpmath.findroot(dP, mpmath.mpf(float(a))) for a in _gll_nodes(n)[1:-1]] + [mpmath.mpf(1)]
        w = [1 / mpmath.fprod([z[i] - z[j] for j in range(n) if j != i]) for i in range(n)]
        D = np.zeros((n, n))
        for i in range(n):
            row = [(w[m] / w[i]) / (z[i] - z[m]) if m != i else mpmath.mpf(0) for m in range(n)]
            row[i] = -mpmath.fsum(row)
            D[i] = [float(v) if abs(v) > 1e-40 else 0.0 for v in row]   # interior diagonal: 0
    return D


def _mxm_r(D, A):
    """d/dr of element-major (nel, nz, ny, nx) data: sum_m D[i, m] A[..., m], m ascending (mxm)."""
    out = D[None, None, None, :, 0] * A[..., 0:1]
    for m in range(1, A.shape[-1]):
        out = out + D[None, None, None, :, m] * A[..., m:m + 1]
    return out


def _mxm_s(D, A):
    out = A[:, :, 0:1, :] * D[None, None, :, 0, None]
    for m in range(1, A.shape[2]):
        out = out + A[:, :, m:m + 1, :] * D[None, None, :, m, None]
    return out


def _mxm_t(D, A):
    out = A[:, 0:1] * D[None, :, 0, None, None]
    for m in range(1, A.shape[1]):
        out = out + A[:, m:m + 1] * D[None, :, m, None, None]
    return out


def gradm1(lx1, ldim, coords, u):
    """Nek5000's gradm1 (navier5.f; not in the reference tree, called at sensitivity.f90:170-199)
    with the geometric factors of its glmapm1 / xyzrst (coef.f), restated from the published
    source: xr = D x along r (mxm), xs, xt along s, t; 2-D jac = xr ys - xs yr, rx = ys, ry = -xs,
    sx = -yr, sy = xr; 3-D jac by addcol4 / subcol4 and the cofactors by ascol5; ux = (1/jac)
    (ur rx + us sx [+ ut tx]).  Element-major points (n_v), one field.  Returns [ux, uy(, uz)]."""
    D = gll_derivative(lx1)
    nz = lx1 if ldim == 3 else 1
    shp = (-1, nz, lx1, lx1)
    X, Y, U = (np.asarray(a, dtype=np.float64).reshape(shp) for a in (coords["x"], coords["y"], u))
    xr, yr, ur = _mxm_r(D, X), _mxm_r(D, Y), _mxm_r(D, U)
    xs, ys, us = _mxm_s(D, X), _mxm_s(D, Y), _mxm_s(D, U)
    if ldim == 2:
        jac = 0.0 + xr * ys
        jac = jac - xs * yr
        rx, ry, sx, sy = ys, -xs, -yr, xr
        jacmi = 1.0 / jac
        return [(jacmi * (ur * rx + us * sx)).ravel(), (jacmi * (ur * ry + us * sy)).ravel()]
    Z = np.asarray(coords["z"], dtype=np.float64).reshape(shp)
    zr, zs = _mxm_r(D, Z), _mxm_s(D, Z)
    xt, yt, zt, ut = _mxm_t(D, X), _mxm_t(D, Y), _mxm_t(D, Z), _mxm_t(D, U)
    jac = 0.0 + xr * ys * zt
    jac = jac + xt * yr * zs
    jac = jac + xs * yt * zr
    jac = jac - xr * yt * zs
    jac = jac - xs * yr * zt
    jac = jac - xt * ys * zr
    rx, ry, rz = ys * zt - yt * zs, xt * zs - xs * zt, xs * yt - xt * ys
    sx, sy, sz = yt * zr - yr * zt, xr * zt - xt * zr, xt * yr - xr * yt
    tx, ty, tz = yr * zs - ys * zr, xs * zr - xr * zs, xr * ys - xs * yr
    jacmi = 1.0 / jac
    return [(jacmi * (ur * rx + us * sx + ut * tx)).ravel(), (jacmi * (ur * ry + us * sy + ut * ty)).ravel(),
            (jacmi * (ur * rz + us * sz + ut * tz)).ravel()]


def norm_grad(lx1, ldim, coords, w, comps):
    """``norm_grad`` (core/utils.f90:446-486): gradm1 of vx_, vy_[, vz_] (:466-468; no dsavg, it is
    commented out at :470-472), then the glsc3 sums in the reference's order, left to right:
    norma = (norma + |dudx|^2) + |dudy|^2 (:476), (norma + |dvdx|^2) + |dvdy|^2 (:477), and in 3-D
    + |dudz|^2, + |dvdz|^2, + |dwdx|^2, + |dwdy|^2, + |dwdz|^2 (:480-484); |g|^2 = glsc3(g, bm1s, g)
    on one rank.  ``comps``: the velocity components (reference point order)."""
    g = [gradm1(lx1, ldim, coords, comps[c]) for c in range(ldim)]
    sq = lambda a: glsc3_np(a, w, a)  # noqa: E731
    norma = 0.0
    norma = norma + sq(g[0][0]) + sq(g[0][1])
    norma = norma + sq(g[1][0]) + sq(g[1][1])
    if ldim == 3:
        norma = norma + sq(g[0][2])
        norma = norma + sq(g[1][2])
        norma = norma + sq(g[2][0])
        norma = norma + sq(g[2][1])
        norma = norma + sq(g[2][2])
    return norma


def outpost_ks_modes(L: OLayout, w, Q, vecs, converged, k, lx1, coords, maxmodes=20, grad_tol=1.1):
    """The mode loop of ``outpost_ks`` (eigensolvers.f90:555-615) with the spurious-mode filter:
    for i = 1..converged (while outp < maxmodes) assemble fp = Q(:,1:k) vecs(:,i) (k_matmul order),
    take norm_grad of its real and imaginary parts BEFORE the nopcmult (:587-588), skip the mode if
    either exceeds 1.1 (:592-595), else outp = outp + 1 and the normalised Re/Im go out as file
    number outp (:600-615).  Returns [(i, outp or None, g_re, g_im, re, im)] (re/im normalised,
    None for skipped modes)."""
    c = ctypes.byref(L.c)
    Qk = np.ascontiguousarray(Q[:k])
    nv, ldim = L.nv, L.ldim
    out, outp = [], 0
    for i in range(converged):
        if outp >= maxmodes:
            continue
        re, im = L.zeros(), L.zeros()
        lib().orc_k_matmul(c, re, Qk, np.ascontiguousarray(vecs[:k, i].real), k)
        lib().orc_k_matmul(c, im, Qk, np.ascontiguousarray(vecs[:k, i].imag), k)
        re[-1] = im[-1] = 0.0
        nt = OLayout(L.nv, L.np, L.nwf, False, L.ldim)
        ar = float(np.sqrt(k_dot(nt, w, re, re)))
        ai = float(np.sqrt(k_dot(nt, w, im, im)))
        beta = 1.0 / np.sqrt(ar ** 2 + ai ** 2)
        g_re = norm_grad(lx1, ldim, coords, w, [re[d * nv:(d + 1) * nv] for d in range(ldim)])
        g_im = norm_grad(lx1, ldim, coords, w, [im[d * nv:(d + 1) * nv] for d in range(ldim)])
        if g_re > grad_tol or g_im > grad_tol:
            out.append((i, None, g_re, g_im, None, None))
            continue
        outp += 1
        lib().orc_k_cmult(c, re, beta)
        lib().orc_k_cmult(c, im, beta)
        re[-1] = im[-1] = 0.0
        out.append((i, outp, g_re, g_im, re, im))
    return out


def bf_sensitivity_terms(ldim, d_re, d_im, a_re, a_im, g):
    """sensitivity.f90:202-235, 258-259 line by line.  d_re ... : lists of velocity components
    [vx, vy(, vz)]; g[(mode, comp, dir)] the dsavg'd gradients, mode in 'dRe','dIm','aRe','aIm',
    comp in 'u','v','w', dir in 'x','y','z'.  opaddcol3(a1,a2,a3,b1,b2,b3,c1,c2,c3) is
    a_c = a_c + b_c*c_c with a3 only in 3-D.  The 2-D reference reads vz_* / dw* arrays it never set
    (opcopy skips vz, gradm1 skips z): those terms are absent here.  Returns dict tr, ti, pr, pi,
    sr, si of component lists."""
    n = d_re[0].size
    three = ldim == 3

    def G(md, c, d):
        return g.get((md, c, d))

    def opaddcol3(a, b, c1, c2, c3):
        if b is None:            # a vz_* multiplier in 2-D: the never-set array, absent
            return
        a[0] = a[0] + b * c1
        a[1] = a[1] + b * c2
        if three:
            a[2] = a[2] + b * c3

    vz = lambda v: v[2] if three else None  # noqa: E731
    neg = lambda v: None if v is None else -v  # noqa: E731
    tr = [np.zeros(n) for _ in range(ldim)]
    opaddcol3(tr, -a_re[0], G("dRe", "u", "x"), G("dRe", "u", "y"), G("dRe", "u", "z"))
    opaddcol3(tr, -a_re[1], G("dRe", "v", "x"), G("dRe", "v", "y"), G("dRe", "w", "z"))
    opaddcol3(tr, neg(vz(a_re)), G("dRe", "w", "x"), G("dRe", "w", "y"), G("dRe", "w", "z"))
    opaddcol3(tr, -a_im[0], G("dIm", "u", "x"), G("dIm", "u", "y"), G("dIm", "u", "z"))
    opaddcol3(tr, -a_im[1], G("dIm", "v", "x"), G("dIm", "v", "y"), G("dIm", "w", "z"))
    opaddcol3(tr, neg(vz(a_im)), G("dIm", "w", "x"), G("dIm", "w", "y"), G("dIm", "w", "z"))
    ti = [np.zeros(n) for _ in range(ldim)]
    opaddcol3(ti, a_re[0], G("dIm", "u", "x"), G("dIm", "u", "y"), G("dIm", "u", "z"))
    opaddcol3(ti, a_re[1], G("dIm", "v", "x"), G("dIm", "v", "y"), G("dIm", "w", "z"))
    opaddcol3(ti, vz(a_re), G("dIm", "w", "x"), G("dIm", "w", "y"), G("dIm", "w", "z"))
    opaddcol3(ti, -a_im[0], G("dRe", "u", "x"), G("dRe", "u", "y"), G("dRe", "u", "z"))
    opaddcol3(ti, -a_im[1], G("dRe", "v", "x"), G("dRe", "v", "y"), G("dRe", "w", "z"))
    opaddcol3(ti, neg(vz(a_im)), G("dRe", "w", "x"), G("dRe", "w", "y"), G("dRe", "w", "z"))
    pr = [np.zeros(n) for _ in range(ldim)]
    opaddcol3(pr, d_re[0], G("aRe", "u", "x"), G("aRe", "v", "x"), G("aRe", "w", "x"))
    opaddcol3(pr, d_re[1], G("aRe", "u", "y"), G("aRe", "v", "y"), G("aRe", "w", "y"))
    opaddcol3(pr, vz(d_re), G("aRe", "u", "z"), G("aRe", "v", "z"), G("aRe", "w", "z"))
    opaddcol3(pr, d_im[0], G("aIm", "u", "x"), G("aIm", "v", "x"), G("aIm", "w", "x"))
    opaddcol3(pr, d_im[1], G("aIm", "u", "y"), G("aIm", "v", "y"), G("aIm", "w", "y"))
    opaddcol3(pr, vz(d_im), G("aIm", "u", "z"), G("aIm", "v", "z"), G("aIm", "w", "z"))
    pi = [np.zeros(n) for _ in range(ldim)]
    opaddcol3(pi, d_re[0], G("aIm", "u", "x"), G("aIm", "v", "x"), G("aIm", "w", "x"))
    opaddcol3(pi, d_re[1], G("aIm", "u", "y"), G("aIm", "v", "y"), G("aIm", "w", "y"))
    opaddcol3(pi, vz(d_re), G("aIm", "u", "z"), G("aIm", "v", "z"), G("aIm", "w", "z"))
    opaddcol3(pi, -d_im[0], G("aRe", "u", "x"), G("aRe", "v", "x"), G("aRe", "w", "x"))
    opaddcol3(pi, -d_im[1], G("aRe", "u", "y"), G("aRe", "v", "y"), G("aRe", "w", "y"))
    opaddcol3(pi, neg(vz(d_im)), G("aRe", "u", "z"), G("aRe", "v", "z"), G("aRe", "w", "z"))
    sr = [tr[c] + pr[c] for c in range(ldim)]      # opadd2, :258
    si = [ti[c] + pi[c] for c in range(ldim)]      # :259
    return dict(tr=tr, ti=ti, pr=pr, pi=pi, sr=sr, si=si)


def bf_sensitivity(L: OLayout, w, lx1, coords, dRe, dIm, aRe, aIm, average=None):
    """sensitivity.f90:81-269 after the four load_fld calls (``ifto = ifpo = .false.``, :138: ``L``
    is the velocity-only layout): biorthogonalize (:163-166), gradm1 + dsavg of every velocity
    component of the four modes (:170-199; ``average(q)`` is dsavg, default the one-rank
    ``coincident_average``), then the pointwise terms (``bf_sensitivity_terms``).  Reference-order
    vectors.  Returns (terms, the four bi-orthogonalised vectors, the gradients)."""
    if average is None:
        average = lambda q: coincident_average(q, coords)  # noqa: E731
    vecs = biorthogonalize(L, w, dRe, dIm, aRe, aIm)
    nv, ldim = L.nv, L.ldim
    comps = [[v[c * nv:(c + 1) * nv] for c in range(ldim)] for v in vecs]
    g = {}
    for md, vc in zip(("dRe", "dIm", "aRe", "aIm"), comps):
        for c, cn in enumerate("uvw"[:ldim]):
            for d, dn in zip(range(ldim), gradm1(lx1, ldim, coords, vc[c])):
                g[(md, cn, "xyz"[d])] = average(dn)
    return bf_sensitivity_terms(ldim, *comps, g), vecs, g


def _cr(fn):
    """fn rounded correctly to double (mpmath at 160 bits, then round-to-nearest)."""
    import mpmath

    def f(x):
        with mpmath.workprec(160):
            return float(fn(mpmath.mpf(x)))
    return f


def libm(kind="glibc"):
    """(sin, cos): the host's glibc (gfortran's libm, as the reference links it) or correctly rounded."""
    import math

    if kind == "glibc":
        return math.sin, math.cos
    import mpmath
    return _cr(mpmath.sin), _cr(mpmath.cos)


def mth_rand(ix, iy, iz, ieg, xl, fc, if3d, sin=None, cos=None):
    """utils.f90:408-418, one point: left-to-right operand order as written (fc(2)*ix*iy =
    (fc(2)*ix)*iy); sin/cos default to the host's glibc."""
    import math

    sin, cos = sin or math.sin, cos or math.cos
    r = fc[0] * (ieg + xl[0] * sin(xl[1])) + fc[1] * ix * iy + fc[2] * ix
    if if3d:
        r = fc[0] * (ieg + xl[2] * sin(r)) + fc[1] * iz * ix + fc[2] * iz
    return cos(1.0e3 * sin(1.0e3 * sin(r)))


def noise_field(nx, ny, nz, e_first, x, y, z, fc, kind="glibc", points=None):
    """The pointwise noise op_add_noise / add_noise_scal add to one field (utils.f90:274-283,
    318-335): element-major points, il fastest, ieg = e_first + e + 1.  ``kind``: the libm (see
    ``libm``); ``points``: evaluate only these indices (the rest NaN)."""
    sin, cos = libm(kind)
    n = x.size
    out = np.full(n, np.nan)
    ppe = nx * ny * nz
    for p in (range(n) if points is None else points):
        e, r = divmod(int(p), ppe)
        il, jl, kl = r % nx + 1, (r // nx) % ny + 1, r // (nx * ny) + 1
        xl = (x[p], y[p], z[p] if z is not None else 0.0)
        out[p] = mth_rand(float(il), float(jl), float(kl), float(e_first + e + 1), xl, fc, z is not None, sin, cos)
    return out


def add_symmetric_seed(y, z, qy, w, zmin, zmax):
    """utils.f90:361-406 on one rank's points (3-D): the spanwise-periodic perturbation, qy as given,
    scaled by 1e-6 / (0.5 (glsc3(qx,bm1,qx) + glsc3(qy,bm1,qy) + glsc3(qz,bm1,qz))).  Returns
    (qx, qy, qz, qp) — qp is the t(:,1) the in-tree solver passes (eigensolvers.f90:207)."""
    pi = 4.0 * np.arctan(1.0)
    alpha = 2 * pi / (zmax - zmin)
    qx = np.cos(alpha * z) * np.sin(2.0 * pi * y)
    qz = -(2.0 * pi) / alpha * np.cos(alpha * z) * np.cos(2.0 * pi * y)
    qp = np.cos(alpha * z) * np.cos(2.0 * pi * y)
    amp = glsc3_np(qx, w, qx) + glsc3_np(qy, w, qy) + glsc3_np(qz, w, qz)
    amp = 1e-6 / (0.50 * amp)
    return qx * amp, qy * amp, qz * amp, qp * amp


def glsc3_np(a, w, b):
    """Nek5000 glsc3 on one rank: sum of a*w*b in point order."""
    return float(np.sum(a * w * b))


def coincident_average(q, coords, rel_tol=1e-9):
    """dssum followed by vmult on one rank (Nek5000 gs '+', then the inverse multiplicity): every
    point gets the mean of the points with the same coordinates, summed in ascending point order
    and scaled by 1/count.  Independent grouping: a dict on rounded coordinates, then every cell is
    joined with each of its 3^d - 1 neighbour cells holding a point that agrees with one of its own
    to 2e-4 cells in every coordinate (two copies of a point a few ulps apart can round to
    neighbouring cells)."""
    import itertools

    xs = [np.asarray(coords[k]) for k in ("x", "y", "z") if k in coords]
    ext = max(float(np.ptp(a)) for a in xs) or 1.0
    tol = rel_tol * ext
    cells = {}
    for p in range(xs[0].size):
        key = tuple(int(round(float(a[p]) / tol)) for a in xs)
        cells.setdefault(key, []).append(p)
    root = {k: k for k in cells}

    def find(k):
        while root[k] != k:
            k = root[k]
        return k

    for key, pts in cells.items():
        for off in itertools.product((-1, 0, 1), repeat=len(xs)):
            nb = tuple(a + b for a, b in zip(key, off))
            if nb == key or nb not in cells:
                continue
            if any(all(abs(float(a[p]) - float(a[r])) <= 2e-4 * tol for a in xs) for p in pts for r in cells[nb]):
                ra, rb = find(key), find(nb)
                if ra != rb:
                    root[max(ra, rb)] = min(ra, rb)
    groups = {}
    for key, pts in cells.items():
        groups.setdefault(find(key), []).extend(pts)
    out = q.copy()
    for members in groups.values():
        members = sorted(members)
        if len(members) < 2:
            continue
        s = 0.0
        for i in members:
            s = s + q[i]
        v = s * (1.0 / len(members))
        for i in members:
            out[i] = v
    return out


def boostconv_core(state, rb, w, nv_total):
    """fixedp.f90:267-329 in numpy on velocity-only vectors (reference order).  ``state`` is a dict
    created empty by the caller; rb (length nv_total) is corrected in place."""
    n = state.setdefault("n", 10)
    dot = lambda a, b: float(np.sum(a * np.tile(w, a.size // w.size) * b))  # noqa: E731
    if not state.get("init"):
        state.update(X=np.zeros((n, rb.size)), Y=np.zeros((n, rb.size)), Q=np.zeros((n, rb.size)),
                     dd=np.ones((n, n)), rot=0, init=True)
        state["Y"][0] = rb
        state["X"][0] = rb
        return
    X, Y, Q = state["X"], state["Y"], state["Q"]
    r = state["rot"]
    Y[r] = Y[r] - rb
    X[r] = X[r] - Y[r]
    dd = np.zeros((n, n))
    Q[:] = 0.0
    dum = Y[0].copy()
    norma = np.sqrt(dot(dum, dum))
    Q[0] = dum * (1.0 / norma)
    dd[0, 0] = norma
    for j in range(1, n):
        dum = Y[j].copy()
        for i in range(j):
            dd[i, j] = dot(dum, Q[i])
            dum = dum - Q[i] * dd[i, j]
        norma = dot(dum, dum)
        if norma < 1e-60:
            norma = 1.0
            Q[j] = 0.0
        else:
            Q[j] = dum * (1.0 / np.sqrt(norma))
        dd[j, j] = np.sqrt(norma)
    cc = np.array([dot(rb, Q[j]) for j in range(n)])
    ccb = np.zeros(n)
    for j in range(n - 1, -1, -1):
        v = cc[j]
        for k in range(j + 1, n):
            v = v - dd[j, k] * ccb[k]
        ccb[j] = v / dd[j, j]
    state["rot"] = (r + 1) % n
    Y[state["rot"]] = rb
    for j in range(n):
        rb += X[j] * ccb[j]
    X[state["rot"]] = rb
