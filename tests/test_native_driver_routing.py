"""CPU contract tests of the one-call native drivers' Python wiring.

``arnoldi_factorization`` and ``gmres_cycle_native`` route their ``*-native`` modes to ONE library
call (``nkv_arnoldi_dcgs2`` / ``nkv_arnoldi_factorization`` / ``nkv_gmres_dcgs2``) with the mode's
flags; round 5 shipped a mis-indented call that made ``"mgs2-icwy-native"`` a silent no-op (H all
zeros), first caught on the GPU box.  Here a recording stand-in for libnekkrylov.so checks, on CPU:

* every native mode reaches exactly one entry point, with the flags the C driver dispatches on;
* every argument converts through the entry's ctypes signature in ``_lib._SIGNATURES`` (arity and
  types, including the callback types);
* the driver's callbacks reach the Python operator for every column mstart..mend, and what the
  driver writes into H arrives in the caller's H (the call is not a no-op).

The stand-in plays the C drivers' side of the contract only (callbacks in column order, one H
entry per column); the arithmetic is the GPU suite's (tests/test_gpu_kernels.py).
"""
import ctypes
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from nekstab_next_amd import _lib
from nekstab_next_amd.arnoldi import arnoldi_factorization
from nekstab_next_amd.gmres import gmres_cycle_native
from nekstab_next_amd.krylov_schur import _mgs2_of, _nonorth_of
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.layout import box3d_layout

ONE_CALL = ("nkv_arnoldi_dcgs2", "nkv_arnoldi_factorization", "nkv_gmres_dcgs2")


class RecordingLib:
    """Entry points of libnekkrylov.so with their real ctypes signatures, recording each call."""

    def __init__(self, ld8: int):
        self.calls = []
        self.ld8 = ld8

    def nkv_arnoldi_scratch_doubles(self, m):
        return 8 * (int(m) + 2)

    def __getattr__(self, name):
        if name not in _lib._SIGNATURES:
            raise AttributeError(name)
        _res, argtypes = _lib._SIGNATURES[name]

        def entry(*args):
            assert len(args) == len(argtypes), (name, len(args), len(argtypes))
            for a, t in zip(args, argtypes):
                t.from_param(a)   # raises on a wrong type (as ctypes would)
            self.calls.append((name, args))
            return self._play(name, args)

        return entry

    def _play(self, name, args):
        if name in ("nkv_arnoldi_dcgs2", "nkv_arnoldi_factorization"):
            Qp, mstart, mend, Hp, ldh, fptr, mv = args[2], args[3], args[4], args[5], args[6], args[7], args[10]
            for c in range(mstart - 1, mend):   # matvec on Q(mstep), then H(mstep+1, mstep) = 1 + c
                if mv(None, Qp + c * self.ld8, fptr, None) != 0:
                    return _lib.NKV_ECALLBACK
                ctypes.c_double.from_address(Hp + 8 * (c * ldh + c + 1)).value = 1.0 + c
            return 0
        if name == "nkv_gmres_dcgs2":
            Qp, ks, Hp, ldh, fptr, mv, resp, kp = args[2], args[3], args[6], args[7], args[8], args[11], args[15], args[16]
            for c in range(ks):
                if mv(None, Qp + c * self.ld8, fptr, None) != 0:
                    return _lib.NKV_ECALLBACK
                ctypes.c_double.from_address(Hp + 8 * (c * ldh + c + 1)).value = 1.0 + c
                ctypes.c_double.from_address(resp + 8 * c).value = 0.5 ** c
            ctypes.c_int.from_address(kp).value = ks
            return 0
        return 0


class _Basis:
    def __init__(self, ptr, k, ld8):
        self.ptr, self.k, self.ld8 = ptr, k, ld8

    def __getitem__(self, c):
        return SimpleNamespace(col=c, ptr=self.ptr + c * self.ld8)


class _Op:
    def __init__(self):
        self.cols = []

    def matvec(self, x, y):
        self.cols.append(x.col)

    rmatvec = matvec


def _setup(m=6, max_cols=8):
    lay = box3d_layout(2)
    ld8 = 8 * lay.ld
    lib = RecordingLib(ld8)
    Lc = lay.c_struct()
    ctx = SimpleNamespace(lib=lib, _Lc=Lc, _Lp=ctypes.byref(Lc), layout=lay, max_cols=max_cols,
                          w=torch.zeros(8, dtype=torch.float64), ws=torch.zeros(8, dtype=torch.float64),
                          device=torch.device("cpu"), comm=SimpleNamespace(world=1, force=False),
                          time_in_dot=False, stream=None)
    Q = _Basis(1 << 40, m + 1, ld8)
    Hd = SimpleNamespace(t=torch.zeros((m, m + 1), dtype=torch.float64), k=m)   # column-major (m+1) x m
    f = SimpleNamespace(ptr=(1 << 41))
    return ctx, Q, Hd, f


NATIVE = {
    "dcgs2-native": ("nkv_arnoldi_dcgs2", 0),
    "cgs2-native": ("nkv_arnoldi_factorization", 0),
    "mgs2-native": ("nkv_arnoldi_factorization", _lib.NKV_MGS2),
    "mgs2-icwy-native": ("nkv_arnoldi_factorization", _lib.NKV_MGS_ICWY),
    "mgs2-lagged-native": ("nkv_arnoldi_factorization", _lib.NKV_MGS_LAGGED),
}


@pytest.mark.parametrize("mode", sorted(NATIVE))
@pytest.mark.parametrize("mstart", [1, 3])
def test_native_mode_is_one_real_call(mode, mstart):
    ctx, Q, Hd, f = _setup()
    op = _Op()
    m = 6
    arnoldi_factorization(ctx, op, Q, Hd, mstart, m, f=f, mode=mode)
    entry, flags = NATIVE[mode]
    names = [c[0] for c in ctx.lib.calls]
    assert names == [entry], names               # exactly one library call, the mode's entry point
    args = ctx.lib.calls[0][1]
    assert args[-2] == flags                     # the flags the C driver dispatches on
    assert (args[3], args[4]) == (mstart, m)
    assert op.cols == list(range(mstart - 1, m))   # the operator saw every column (not a no-op)
    H = Hd.t.numpy().T                           # (m+1) x m as the caller reads it
    for c in range(mstart - 1, m):
        assert H[c + 1, c] == 1.0 + c
    assert np.count_nonzero(H) == m - mstart + 1


@pytest.mark.parametrize("mode", sorted(NATIVE))
def test_native_mode_time_in_dot_flag(mode):
    ctx, Q, Hd, f = _setup()
    ctx.time_in_dot = True
    arnoldi_factorization(ctx, _Op(), Q, Hd, 1, 4, f=f, mode=mode)
    assert ctx.lib.calls[0][1][-2] == NATIVE[mode][1] | _lib.NKV_TIME_DOT


def test_native_mode_with_hook_runs_the_python_sequence():
    """A per-step hook (checkpointing) needs the Python-driven sequence: no one-call entry point."""
    ctx, Q, Hd, f = _setup()
    ctx.call = lambda *a, **k: pytest.fail("device path reached")   # noqa: E731 - the Python sequence starts here
    for mode in ("dcgs2-native", "cgs2-native", "mgs2-native"):
        with pytest.raises(BaseException):
            arnoldi_factorization(ctx, _Op(), Q, Hd, 1, 4, f=f, mode=mode, on_step=lambda c: None)
        assert not [c for c in ctx.lib.calls if c[0] in ONE_CALL]


def test_native_mode_bounds_checked():
    ctx, Q, Hd, f = _setup(m=6, max_cols=4)
    with pytest.raises(ValueError):
        arnoldi_factorization(ctx, _Op(), Q, Hd, 1, 6, f=f, mode="mgs2-icwy-native")
    assert ctx.lib.calls == []


def test_gmres_native_cycle_is_one_real_call():
    ctx, Q, Hd, f = _setup()
    op = _Op()
    k, res = gmres_cycle_native(ctx, op.matvec, Q, Hd, f, 6, 2.0, 1e-9)
    assert [c[0] for c in ctx.lib.calls] == ["nkv_gmres_dcgs2"]
    assert k == 6 and op.cols == list(range(6))
    np.testing.assert_array_equal(res, 0.5 ** np.arange(6))
    args = ctx.lib.calls[0][1]
    assert args[3] == 6 and args[4] == 2.0 and args[5] == 1e-9 and args[-2] == 0
    assert Hd.t.numpy().T[6, 5] == 6.0


def test_callback_failure_surfaces():
    """An exception in the operator callback is re-raised after the library call returns."""
    ctx, Q, Hd, f = _setup()

    class Boom(_Op):
        def matvec(self, x, y):
            raise RuntimeError("operator failed")

    with pytest.raises(RuntimeError, match="operator failed"):
        arnoldi_factorization(ctx, Boom(), Q, Hd, 1, 4, f=f, mode="cgs2-native")


def test_krylov_schur_keeps_native_modes_native():
    """A solve configured with a native mode falls back (non-orthonormal seed, time in k_dot) to the
    library-driven twin of the fallback, never silently to the Python one."""
    cfg = KrylovSchurConfig()
    assert _mgs2_of("dcgs2-native") == "mgs2-native" and _mgs2_of("dcgs2") == "mgs2"
    assert _nonorth_of("dcgs2-native", cfg) == "mgs2-lagged-native"
    assert _nonorth_of("dcgs2-native", cfg, time_in_dot=True) == "mgs2-icwy-native"
    assert _nonorth_of("dcgs2", cfg, time_in_dot=True) == "mgs2-icwy"
    for m in _nonorth_of("dcgs2-native", cfg), _nonorth_of("dcgs2-native", cfg, True), _mgs2_of("cgs2-native"):
        assert m in NATIVE
