"""Small dense Hessenberg/Schur steps on the host (mirror of core/lapack_wrapper.f90).

The k x k problems (k <= a few hundred) are latency-bound and tiny next to the HBM-bound basis
work, so — as in the reference, which runs them redundantly on every MPI rank — they run on the
host, redundantly on every GPU process, on bit-identical all-reduced data.  LAPACK comes from
SciPy's bundled OpenBLAS 0.3.28 (the reference links OpenBLAS / system LAPACK or MKL,
bin/mks:44,84-108).  Workspace sizes are the reference's (they select LAPACK's unblocked paths):
dgeev lwork=4n (:152), dgees lwork=3n (:45), dtrsen lwork=n, liwork=1 (:103-104), dgels
lwork=2mn (:283).

Ordering/selection rules that decide a Krylov–Schur restart are restated exactly, including
their quirks:
* ``sort_eigendecomp`` — exchange sort on |lambda|, strict ``<`` (:181-228);
* ``select_eigvals`` — dgees sort predicate sqrt(wr^2+wi^2) > 0.9 (:232-244);
* ``select_eigenvalues`` — |lambda| >= 1-delta, plus the nev+4 largest by ``quicksort2`` order, plus
  one more when the imaginary parts at the boundary are exact negatives — true for two real
  eigenvalues too, since 0 == -0 (core/eigensolvers.f90:688-754, core/utils.f90:29-138).
"""
from __future__ import annotations

import contextlib

import numpy as np
from scipy.linalg import lapack as _lp

_tp = None


def _one_thread():
    """Single-threaded BLAS for the k x k problems: deterministic bits on every rank (the restart
    decisions are taken redundantly per rank and must agree), and no thread fan-out for tiny work."""
    global _tp
    if _tp is None:
        try:
            from threadpoolctl import ThreadpoolController

            _tp = ThreadpoolController()
        except Exception:  # noqa: BLE001  (threadpoolctl missing: run as configured)
            _tp = False
    return _tp.limit(limits=1, user_api="blas") if _tp else contextlib.nullcontext()


def eig(A: np.ndarray):
    """dgeev(jobvl='N', jobvr='V') on a copy; complex vecs from conjugate pairs; sorted by |lambda|
    descending (lapack_wrapper.f90:114-177).  Returns (vals[n] complex, vecs[n,n] complex)."""
    A = np.array(A, dtype=np.float64, order="F", copy=True)
    n = A.shape[0]
    with _one_thread():
        wr, wi, _vl, vr, info = _lp.dgeev(A, compute_vl=0, compute_vr=1, lwork=max(1, 4 * n))
    if info != 0:
        raise np.linalg.LinAlgError(f"dgeev info={info}")
    vals = wr + 1j * wi
    vecs = vr.astype(np.complex128)
    for i in range(n - 1):
        if wi[i] > 0:
            vecs[:, i] = vr[:, i] + 1j * vr[:, i + 1]
            vecs[:, i + 1] = vr[:, i] - 1j * vr[:, i + 1]
        elif wi[i] == 0:
            vecs[:, i] = vr[:, i]
    return sort_eigendecomp(vals, vecs)


def sort_eigendecomp(vals: np.ndarray, vecs: np.ndarray):
    """Exchange sort by decreasing modulus; swaps only on strict ``norm(k) < norm(l)``
    (lapack_wrapper.f90:212-226).  The exchanges run on a permutation of Python floats (the same
    float64 comparisons, so the same permutation, ties included) and are applied to the values
    and vectors once."""
    nrm = np.sqrt(vals.real ** 2 + vals.imag ** 2).tolist()
    n = len(nrm)
    idx = list(range(n))
    for k in range(n - 1):
        nk = nrm[k]
        for l in range(k + 1, n):
            if nk < nrm[l]:
                nrm[k], nrm[l] = nrm[l], nk
                idx[k], idx[l] = idx[l], idx[k]
                nk = nrm[k]
    return vals[idx], vecs[:, idx]


def select_eigvals(wr: float, wi: float) -> bool:
    return bool(np.sqrt(wr * wr + wi * wi) > 0.9)


def schur(A: np.ndarray):
    """dgees(jobvs='V', sort='S', select_eigvals), lwork=3n (lapack_wrapper.f90:3-55).
    Returns (T, Z, vals) with vals in Schur-diagonal order."""
    A = np.array(A, dtype=np.float64, order="F", copy=True)
    n = A.shape[0]
    with _one_thread():
        t, _sdim, wr, wi, vs, _work, info = _lp.dgees(lambda a, b: int(select_eigvals(a, b)), A, compute_v=1,
                                                      sort_t=1, lwork=max(1, 3 * n))
    if info not in (0, n + 1, n + 2):  # the reference ignores info; only hard failures raise here
        raise np.linalg.LinAlgError(f"dgees info={info}")
    return np.asfortranarray(t), np.asfortranarray(vs), wr + 1j * wi


def ordschur(T: np.ndarray, Z: np.ndarray, selected: np.ndarray):
    """dtrsen(job='N', compq='V') moving ``selected`` to the leading block (:59-111)."""
    n = T.shape[0]
    with _one_thread():
        ts, qs, _wr, _wi, m, _s, _sep, info = _lp.dtrsen(np.asarray(selected, dtype=np.int32), T, Z, job="N",
                                                         wantq=1, lwork=max(1, n), liwork=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dtrsen info={info}")
    return np.asfortranarray(ts), np.asfortranarray(qs), int(m)


def lstsq(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    """min ||A x - b||_2 via dgels('N'), lwork=2mn; x = b_tilde(1:n) (:248-300)."""
    A = np.array(A, dtype=np.float64, order="F", copy=True)
    m, n = A.shape
    with _one_thread():
        _lqr, x, info = _lp.dgels(A, np.array(b, dtype=np.float64, copy=True), trans="N",
                                  lwork=max(1, 2 * m * n))
    if info != 0:
        raise np.linalg.LinAlgError(f"dgels info={info}")
    return np.asarray(x[:n], dtype=np.float64)


def quicksort2(arr: np.ndarray) -> np.ndarray:
    """Index order of ``arr`` ascending, exactly as utils.f90:29-138 (median-of-three partition
    with insertion sort below 7 elements, explicit stack).  The tie order matters: conjugate
    pairs have bit-equal moduli.  Simulated 1-based; returns a 0-based index array."""
    n = len(arr)
    a = [0.0] + [float(x) for x in arr]
    idx = list(range(n + 1))  # idx[i] = i (1-based); slot 0 unused
    M = 7
    stack: list[int] = []
    l, ir = 1, n
    while True:
        if ir - l < M:
            for j in range(l + 1, ir + 1):
                av, bv = a[j], idx[j]
                i = j - 1
                while i >= l and a[i] > av:
                    a[i + 1], idx[i + 1] = a[i], idx[i]
                    i -= 1
                a[i + 1], idx[i + 1] = av, bv
            if not stack:
                return np.asarray(idx[1:], dtype=np.int64) - 1
            ir = stack.pop()
            l = stack.pop()
            continue
        k = (l + ir) // 2
        a[k], a[l + 1] = a[l + 1], a[k]
        idx[k], idx[l + 1] = idx[l + 1], idx[k]
        for x, y in ((l, ir), (l + 1, ir), (l, l + 1)):
            if a[x] > a[y]:
                a[x], a[y] = a[y], a[x]
                idx[x], idx[y] = idx[y], idx[x]
        i, j = l + 1, ir
        av, bv = a[l + 1], idx[l + 1]
        while True:
            while a[i] < av:
                i += 1
            while a[j] > av:
                j -= 1
            if i >= j:
                break
            a[i], a[j] = a[j], a[i]
            idx[i], idx[j] = idx[j], idx[i]
            i += 1
            j -= 1
        a[l + 1], a[j] = a[j], av
        idx[l + 1], idx[j] = idx[j], bv
        if ir - i + 1 >= j - l:
            stack += [i, ir]
            ir = j - 1
        else:
            stack += [l, j - 1]
            l = i


def select_eigenvalues(vals: np.ndarray, delta: float, nev: int, faithful: bool = True):
    """(selected[n] bool, cnt) as eigensolvers.f90:688-754.

    ``faithful=True`` orders by the reference's ``quicksort2``, whose partition step overwrites
    the pivot slot and can duplicate/drop indices for n >= 8 ("reference defects"), so
    the "nev+4 largest" may not be the largest.  ``faithful=False`` uses a correct stable argsort."""
    n = vals.shape[0]
    mod = np.abs(vals)
    idx = quicksort2(mod) if faithful else np.argsort(mod, kind="stable")
    selected = mod >= (1.0 - delta)
    top = n - (nev + 4)  # 0-based position of Fortran idx(n-(nev+3))
    if top < 0:
        raise ValueError(f"k_dim={n} too small for schur_tgt={nev} (needs k_dim >= nev+5)")
    selected[idx[top:]] = True
    if top >= 1 and vals[idx[top]].imag == -vals[idx[top - 1]].imag:
        selected[idx[top - 1]] = True
    return selected, int(selected.sum())
