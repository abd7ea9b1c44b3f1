"""The oracle's dense LAPACK: Intel MKL through ctypes.  TEST INFRASTRUCTURE ONLY.

The reference's build links MKL when it finds it (``/root/reference/bin/mks:32-44``: ``-mkl`` /
``-lmkl_rt``), otherwise OpenBLAS or system LAPACK (``bin/mks:84-108``).  The product's host path
(``nekstab_next_amd/lapack.py``) calls SciPy's bundled OpenBLAS.  So that "product vs oracle" never
compares one library with itself, the oracle calls the four routines of
``core/lapack_wrapper.f90`` in MKL (``/opt/conda/lib/libmkl_rt.so``, the image's oneAPI MKL
2021.4), with exactly the reference's arguments and workspace sizes:

* ``dgeev('N', 'V', n, A~, n, wr, wi, vl, 1, vr, n, work, 4n, info)``        lapack_wrapper.f90:152-158
* ``dgees('V', 'S', select_eigvals, n, A, n, sdim, wr, wi, Z, n, work, 3n, bwork, info)``  :45-49
* ``dtrsen('N', 'V', selected, n, T, n, Q, n, wr, wi, m, s, sep, work, n, iwork, 1, info)`` :103-108
* ``dgels('N', m, n, 1, A~, m, b~, m, work, 2mn, info)``                       :281-288

MKL runs in its sequential layer (``MKL_THREADING_LAYER=SEQUENTIAL``) with conditional numerical
reproducibility ``MKL_CBWR=COMPATIBLE``, so its bits do not depend on the host CPU (the build
container's Xeon and the GPU box's EPYC give the same fixtures).  Both variables are set before
the library is first loaded; they only affect MKL.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, byref, c_char, c_double, c_int

import numpy as np

MKL_PATH = os.environ.get("NEKSTAB_ORACLE_MKL", "/opt/conda/lib/libmkl_rt.so")

_mkl = None
_SELECT = ctypes.CFUNCTYPE(c_int, POINTER(c_double), POINTER(c_double))


def available() -> bool:
    return os.path.exists(MKL_PATH)


def lib():
    global _mkl
    if _mkl is None:
        if not os.path.exists(MKL_PATH):
            raise RuntimeError(f"oracle LAPACK: {MKL_PATH} not found (set NEKSTAB_ORACLE_LAPACK=openblas to run "
                               "the oracle on SciPy's OpenBLAS, the product's library)")
        os.environ.setdefault("MKL_THREADING_LAYER", "SEQUENTIAL")
        os.environ.setdefault("MKL_CBWR", "COMPATIBLE")
        os.environ.setdefault("MKL_INTERFACE_LAYER", "LP64")
        L = ctypes.CDLL(MKL_PATH)
        for name in ("dgeev_", "dgees_", "dtrsen_", "dgels_"):
            getattr(L, name).restype = None
        _mkl = L
    return _mkl


def version() -> str:
    buf = ctypes.create_string_buffer(256)
    lib().MKL_Get_Version_String(buf, 256)
    return buf.value.decode()


def _ptr(a):
    return a.ctypes.data_as(POINTER(c_double))


def _ch(s):
    return byref(c_char(s.encode()))


def dgeev(A):
    """(wr, wi, vr) of dgeev('N','V') on a copy of A, lwork = 4n (lapack_wrapper.f90:152-158)."""
    n = A.shape[0]
    a = np.array(A, dtype=np.float64, order="F", copy=True)
    wr, wi = np.zeros(n), np.zeros(n)
    vl = np.zeros((1, n), order="F")
    vr = np.zeros((n, n), order="F")
    work = np.zeros(max(1, 4 * n))
    info = c_int(0)
    lib().dgeev_(_ch("N"), _ch("V"), byref(c_int(n)), _ptr(a), byref(c_int(n)), _ptr(wr), _ptr(wi), _ptr(vl),
                 byref(c_int(1)), _ptr(vr), byref(c_int(n)), _ptr(work), byref(c_int(4 * n)), byref(info))
    return wr, wi, vr, info.value


def _select_eigvals(wr, wi):
    """select_eigvals (lapack_wrapper.f90:232-244): sqrt(wr**2 + wi**2) > 0.9.  Fortran .TRUE. is
    returned as 1 (low bit set and nonzero: true under either LOGICAL convention)."""
    a, b = wr[0], wi[0]
    return 1 if np.sqrt(a * a + b * b) > 0.9 else 0


_select_cb = _SELECT(_select_eigvals)


def dgees(A):
    """(T, Z, wr, wi, sdim, info) of dgees('V','S', select_eigvals), lwork = 3n (:45-49)."""
    n = A.shape[0]
    a = np.array(A, dtype=np.float64, order="F", copy=True)
    wr, wi = np.zeros(n), np.zeros(n)
    vs = np.zeros((n, n), order="F")
    work = np.zeros(max(1, 3 * n))
    bwork = np.zeros(n, dtype=np.int32)
    sdim, info = c_int(0), c_int(0)
    lib().dgees_(_ch("V"), _ch("S"), _select_cb, byref(c_int(n)), _ptr(a), byref(c_int(n)), byref(sdim), _ptr(wr),
                 _ptr(wi), _ptr(vs), byref(c_int(n)), _ptr(work), byref(c_int(max(1, 3 * n))),
                 bwork.ctypes.data_as(POINTER(c_int)), byref(info))
    return a, vs, wr, wi, sdim.value, info.value


def dtrsen(T, Z, selected):
    """(T', Z', m, info) of dtrsen('N','V', selected), lwork = n, liwork = 1 (:103-108)."""
    n = T.shape[0]
    t = np.array(T, dtype=np.float64, order="F", copy=True)
    q = np.array(Z, dtype=np.float64, order="F", copy=True)
    sel = np.ascontiguousarray(np.asarray(selected, dtype=bool).astype(np.int32))
    wr, wi = np.zeros(n), np.zeros(n)
    work = np.zeros(max(1, n))
    iwork = np.zeros(1, dtype=np.int32)
    m, info = c_int(0), c_int(0)
    s, sep = c_double(0.0), c_double(0.0)
    lib().dtrsen_(_ch("N"), _ch("V"), sel.ctypes.data_as(POINTER(c_int)), byref(c_int(n)), _ptr(t), byref(c_int(n)),
                  _ptr(q), byref(c_int(n)), _ptr(wr), _ptr(wi), byref(m), byref(s), byref(sep), _ptr(work),
                  byref(c_int(max(1, n))), iwork.ctypes.data_as(POINTER(c_int)), byref(c_int(1)), byref(info))
    return t, q, m.value, info.value


def dgels(A, b):
    """(x, info) of dgels('N', m, n, 1) on copies, lwork = 2mn; x = b~(1:n) (:281-298)."""
    m, n = A.shape
    a = np.array(A, dtype=np.float64, order="F", copy=True)
    bt = np.array(b, dtype=np.float64, copy=True).reshape(m)
    work = np.zeros(max(1, 2 * m * n))
    info = c_int(0)
    lib().dgels_(_ch("N"), byref(c_int(m)), byref(c_int(n)), byref(c_int(1)), _ptr(a), byref(c_int(m)), _ptr(bt),
                 byref(c_int(m)), _ptr(work), byref(c_int(max(1, 2 * m * n))), byref(info))
    return bt[:n].copy(), info.value
