"""ctypes binding of ``libnekkrylov.so`` (the C ABI declared in ``include/nekkrylov.h``).

The library is built in-tree by ``__graft_entry__.build()`` (``hipcc --offload-arch=gfx950``).
There is no CPU fallback: if the library is missing or no GPU is visible, every entry point
raises.  ``torch`` is imported first on purpose: torch ships its own ``libamdhip64.so.7`` and the
dynamic loader must resolve our ``DT_NEEDED libamdhip64.so.7`` to that same runtime, so device
pointers and streams handed over from torch are valid on our side.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import CFUNCTYPE, POINTER, Structure, c_char_p, c_double, c_int, c_int32, c_int64, c_size_t, c_uint, c_uint64, c_void_p

import torch  # noqa: F401  (must be loaded before the HIP library, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libnekkrylov.so")

NKV_ABI_VERSION = 3
NKV_TILE = 4096
NKV_MAX_COLS = 1024   # most columns per multi-dot (include/nekkrylov.h)
NKV_ROT_MAX_OUT = 256   # most output columns of a basis rotation with more than 16 kept (include/nekkrylov.h)
NKV_OK, NKV_EINVAL, NKV_EHIP, NKV_ENAN, NKV_ESHAPE, NKV_ECALLBACK, NKV_EBREAKDOWN = 0, 1, 2, 3, 4, 5, 6
NKV_TIME = 0x1
NKV_ACCUMULATE = 0x2
NKV_OVERWRITE = 0x4
NKV_NORM2 = 0x8
NKV_TIME_DOT = 0x10
NKV_X_IS_LAST = 0x20
NKV_MGS2 = 0x40
NKV_MGS_ICWY = 0x100
NKV_MGS_LAGGED = 0x200
NKV_CHECK_BREAKDOWN = 0x80


class NkvError(RuntimeError):
    """A non-zero status from the C ABI."""

    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: status {code}: {msg}")
        self.code = code


class NkvNaNError(NkvError, FloatingPointError):
    """NaN detected in a dot product (reference aborts: core/nek_vectors.f90:108-111)."""


class NkvBreakdownError(NkvError):
    """NKV_CHECK_BREAKDOWN: a one-call factorisation reached an invariant subspace (include/nekkrylov.h)."""


class nkv_layout(Structure):
    _fields_ = [
        ("n_v", c_int64),
        ("n_p", c_int64),
        ("sv", c_int64),
        ("sp", c_int64),
        ("ld", c_int64),
        ("n_wf", c_int32),
        ("rank0", c_int32),
    ]


_P = c_void_p  # device pointers and streams travel as plain addresses
_L = POINTER(nkv_layout)
# callbacks of nkv_arnoldi_dcgs2: matvec(user, x, y, stream), allreduce(user, buf, n, stream)
MATVEC_FN = CFUNCTYPE(c_int, c_void_p, c_void_p, c_void_p, c_void_p)
ALLREDUCE_FN = CFUNCTYPE(c_int, c_void_p, c_void_p, c_int, c_void_p)

# name -> (restype, argtypes)
_SIGNATURES = {
    "nkv_abi_version": (c_int, []),
    "nkv_layout_init": (c_int, [_L, c_int, c_int, c_int, c_int64, c_int64, c_int, c_int, c_int]),
    "nkv_last_error": (c_char_p, []),
    "nkv_device_info": (c_int, [POINTER(c_int), POINTER(c_int), POINTER(c_int64), c_char_p, c_int]),
    "nkv_workspace_bytes": (c_size_t, [_L, c_int]),
    "nkv_check_status": (c_int, [_P, _P]),
    "nkv_zero": (c_int, [_L, _P, c_uint, _P]),
    "nkv_copy": (c_int, [_L, _P, _P, c_uint, _P]),
    "nkv_scal": (c_int, [_L, _P, c_double, c_uint, _P]),
    "nkv_axpby": (c_int, [_L, _P, c_double, _P, c_double, c_uint, _P]),
    "nkv_sub3": (c_int, [_L, _P, _P, _P, c_uint, _P]),
    "nkv_axpy_dev": (c_int, [_L, _P, _P, c_double, _P, c_uint, _P]),
    "nkv_normalize_dev": (c_int, [_L, _P, _P, _P, c_uint, _P]),
    "nkv_dot": (c_int, [_L, _P, _P, _P, _P, _P, c_uint, _P]),
    "nkv_block_dot": (c_int, [_L, _P, _P, c_int, _P, _P, _P, c_uint, _P]),
    "nkv_block_update": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, c_uint, _P]),
    "nkv_block_update_dot": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, c_uint, _P]),
    "nkv_arnoldi_finish": (c_int, [_L, _P, _P, _P, c_int, _P, _P, _P, c_uint, _P]),
    "nkv_block_dot2": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, c_uint, _P]),
    "nkv_dcgs2_coef": (c_int, [c_int, _P, _P, _P, _P, c_int64, _P, _P, _P]),
    "nkv_mgs_icwy_solve": (c_int, [c_int, _P, c_int64, _P, _P, _P, _P]),
    "nkv_dcgs2_update": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, _P, _P, c_uint, _P]),
    "nkv_arnoldi_scratch_doubles": (c_size_t, [c_int]),
    "nkv_arnoldi_dcgs2": (c_int, [_L, _P, _P, c_int, c_int, _P, c_int64, _P, _P, _P, MATVEC_FN, _P, ALLREDUCE_FN, _P,
                                  c_uint, _P]),
    "nkv_update_hessenberg": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, _P, ALLREDUCE_FN, _P, c_uint, _P]),
    "nkv_gmres_dcgs2": (c_int, [_L, _P, _P, c_int, c_double, c_double, _P, c_int64, _P, _P, _P, MATVEC_FN, _P,
                                ALLREDUCE_FN, _P, _P, _P, c_uint, _P]),
    "nkv_arnoldi_factorization": (c_int, [_L, _P, _P, c_int, c_int, _P, c_int64, _P, _P, _P, MATVEC_FN, _P,
                                          ALLREDUCE_FN, _P, c_uint, _P]),
    "nkv_combine": (c_int, [_L, _P, c_int, _P, _P, c_uint, _P]),
    "nkv_normalize_store": (c_int, [_L, _P, _P, _P, _P, c_uint, _P]),
    "nkv_mgs2_step": (c_int, [_L, _P, _P, c_int, _P, _P, _P, _P, c_uint, _P]),
    "nkv_axpy_dot": (c_int, [_L, _P, _P, _P, _P, _P, _P, _P, c_uint, _P]),
    "nkv_rotate": (c_int, [_L, _P, c_int, _P, c_int, _P]),
    "nkv_rotate_cols": (c_int, [_L, _P, c_int, _P, c_int, c_int, _P]),
    "nkv_op_diag": (c_int, [_L, _P, _P, _P, c_double, _P]),
    "nkv_op_rot2": (c_int, [_L, _P, _P, _P, _P, _P, c_int, _P]),
    "nkv_op_cdiag": (c_int, [_L, _P, _P, _P, _P, c_int, _P]),
    "nkv_fill_hash": (c_int, [_L, _P, c_uint64, c_int64, c_int64, _P]),
    "nkv_mth_rand_add": (c_int, [_L, c_int, c_int, c_int, c_int64, _P, _P, _P, c_double, c_double, c_double, _P, _P]),
    "nkv_group_average": (c_int, [c_int64, _P, _P, _P, _P]),
    "nkv_symmetric_seed": (c_int, [_L, _P, _P, c_double, _P, _P, _P, _P]),
    "nkv_wavemaker": (c_int, [_L, _P, _P, _P, _P, _P, c_int, _P]),
    "nkv_gradm1": (c_int, [_L, c_int, c_int, _P, _P, _P, _P, _P, c_int, c_int64, _P, c_int64, _P]),
    "nkv_bf_sensitivity": (c_int, [_L, _P, _P, _P, _P, _P, _P, c_int, _P]),
    "nkv_givens_column": (c_double, [c_int, _P, _P, _P, _P]),
    "nkv_lagged_coef": (c_int, [c_int, c_int, _P, _P, c_int64, _P, c_int64, _P]),
    "nkv_gkl_coef": (c_int, [c_int, c_int, _P, _P, _P, c_int64, _P, _P, _P, _P, c_int64, _P, _P, _P]),
}

# Every symbol include/nekkrylov.h declares (tests check the .so exports all of them).
EXPORTED = tuple(_SIGNATURES)

_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load and type the library once.  Raises ImportError with a build hint if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: the MI355X HIP extension is not built. "
            "Run `python -c 'import __graft_entry__ as g; g.build()'` (hipcc --offload-arch=gfx950). "
            "There is no CPU fallback for the Krylov hot path."
        )
    lib = ctypes.CDLL(path)
    for name, (res, args) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.nkv_abi_version() != NKV_ABI_VERSION:
        raise ImportError(f"ABI mismatch: {path} reports {lib.nkv_abi_version()}, expected {NKV_ABI_VERSION}")
    _lib = lib
    return lib


def last_error() -> str:
    return load().nkv_last_error().decode(errors="replace")


def check(code: int, where: str) -> None:
    if code == NKV_OK:
        return
    msg = last_error()
    if code == NKV_ENAN:
        raise NkvNaNError(code, where, msg)
    if code == NKV_EBREAKDOWN:
        raise NkvBreakdownError(code, where, msg)
    raise NkvError(code, where, msg)


def call(name: str, *args) -> None:
    """Call a status-returning entry point and raise on failure."""
    check(getattr(load(), name)(*args), name)


def require_gpu() -> None:
    """Fail loudly when no HIP device is visible: this package has no CPU path."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            "nekstab_next_amd needs an MI355X (HIP device); torch.cuda.is_available() is False. "
            "There is no CPU fallback."
        )
    load()
