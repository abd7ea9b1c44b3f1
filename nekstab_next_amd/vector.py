"""Device-resident nekStab state vectors and Krylov bases (host mirror of the vector layer).

Mirrors two reference abstractions over ONE device layout (include/nekkrylov.h):

* LightKrylov's ``real_nek_vector`` with type-bound ``zero / dot / scal / axpby``
  (core/nek_vectors.f90:20-31, 70-139): :class:`NekVector` methods of the same names, with the same
  quirks — ``dot`` always includes ``self%time*vec%time`` (:106) and ``axpby`` leaves ``time``
  untouched (:127-139).
* the legacy free subroutines ``k_dot, k_norm, k_normalize, k_cmult, k_add2, k_sub2, k_sub3,
  k_zero, k_copy, k_matmul`` on ``type(krylov_vector)`` (core/krylov_subspace.f90:26-209): the
  module-level functions below, where ``time`` follows every update and enters the dot only when
  ``uparam(1) == 2.1`` (:52-54) — here the context's ``time_in_dot`` switch.

All arithmetic runs in ``libnekkrylov.so``; this module only owns memory (torch tensors on the
GPU, one process per device), streams and the collective.  There is no CPU path.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import NKV_OVERWRITE, NKV_TIME
from .comm import Comm
from .layout import NekLayout


def _ptr(t: torch.Tensor) -> int:
    return t.data_ptr()


class NekContext:
    """Per-GPU state: layout (this rank's shard), mass-matrix weights ``bm1s``, workspace, comm.

    ``weights`` are the local ``bm1s`` values (length ``layout.n_v``; zeros allowed, e.g. inside
    a sponge, core/forcing.f90:101-104).  ``time_in_dot`` selects ``k_dot``'s uparam(1)==2.1
    behaviour for the legacy ops and the Gram–Schmidt dots.
    """

    def __init__(self, layout: NekLayout, weights=None, comm: Comm | None = None, max_cols: int = 256,
                 device: torch.device | int | None = None, time_in_dot: bool = False):
        if not 1 <= max_cols < _lib.NKV_MAX_COLS:   # the closing multi-dot takes max_cols + 1 columns
            raise ValueError(f"max_cols={max_cols} outside 1..{_lib.NKV_MAX_COLS - 1}")
        _lib.require_gpu()
        self.comm = comm if comm is not None else Comm()
        if layout.world != self.comm.world or layout.rank != self.comm.rank:
            layout = layout.shard(self.comm.rank, self.comm.world)
        self.layout = layout
        if device is None:
            device = torch.cuda.current_device()
        self.device = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
        self.L = layout.c_struct()
        self._Lp = ctypes.byref(self.L)
        self.time_in_dot = time_in_dot
        self.max_cols = max_cols
        self.timer = None  # optional profiling.PhaseTimer (per-phase HIP events)
        self.lib = _lib.load()
        f64 = dict(dtype=torch.float64, device=self.device)
        # at least one tile: an empty shard (rank with no elements) still passes a valid pointer
        self.w = torch.zeros(max(layout.sv, 4096), **f64)
        if weights is None:
            self.w[: layout.n_v] = 1.0
        else:
            wt = torch.as_tensor(np.asarray(weights, dtype=np.float64)).to(self.device)
            if wt.numel() != layout.n_v:
                raise ValueError(f"weights: expected {layout.n_v} local values, got {wt.numel()}")
            self.w[: layout.n_v] = wt
        nbytes = int(self.lib.nkv_workspace_bytes(self._Lp, max_cols))
        self.ws = torch.zeros((nbytes + 7) // 8, **f64)
        # scalar / short-vector scratch for partials that get all-reduced
        self.h1 = torch.zeros(max_cols + 1, **f64)
        self.h2 = torch.zeros(max_cols + 1, **f64)
        self.scal = torch.zeros(8, **f64)
        # DCGS2: [Q^T W q_j ; Q^T W A q_j] (one all-reduce) and the small-step coefficients
        self.hd = torch.zeros(2 * (max_cols + 1), **f64)
        self.coef = torch.zeros(4 * max_cols + 16, **f64)   # DCGS2: [x | c | 4 scalars | a]

    # ---- plumbing ----------------------------------------------------------------------------
    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def call(self, name: str, *args) -> None:
        _lib.check(getattr(self.lib, name)(self._Lp, *args), name)

    def call_nl(self, name: str, *args) -> None:
        """Entry points without a layout argument (small dense device kernels)."""
        _lib.check(getattr(self.lib, name)(*args), name)

    def check_nan(self) -> None:
        """Surface a NaN flagged by any reduction so far (synchronises the stream)."""
        _lib.check(self.lib.nkv_check_status(_ptr(self.ws), self.stream), "nkv_check_status")

    def synchronize(self) -> None:
        torch.cuda.synchronize(self.device)

    # ---- allocation --------------------------------------------------------------------------
    def vector(self) -> "NekVector":
        return NekVector(self, torch.zeros(self.layout.ld, dtype=torch.float64, device=self.device))

    def basis(self, k: int) -> "Basis":
        return Basis(self, k)

    # ---- reductions (collective) ---------------------------------------------------------------
    def dot_dev(self, a: "NekVector", b: "NekVector", out: torch.Tensor, time: bool) -> torch.Tensor:
        """Local weighted dot into ``out[0]`` then all-reduce; stays on the device."""
        self.call("nkv_dot", _ptr(self.w), a.ptr, b.ptr, _ptr(out), _ptr(self.ws), NKV_TIME if time else 0,
                  self.stream)
        return self.comm.allreduce_(out[:1])

    def dot(self, a: "NekVector", b: "NekVector", time: bool) -> float:
        out = self.scal[0:1]
        self.dot_dev(a, b, out, time)
        val = float(out.item())
        if val != val:
            self.check_nan()
        return val


class NekVector:
    """One state vector ``(vx, vy, [vz], [t..], pr, time)`` in HBM (a view of ``storage``)."""

    def __init__(self, ctx: NekContext, storage: torch.Tensor):
        self.ctx = ctx
        self.storage = storage

    @property
    def ptr(self) -> int:
        return self.storage.data_ptr()

    # ---- LightKrylov abstract_vector API (real_nek_vector) -----------------------------------
    def zero(self) -> None:
        """real_zero: all fields and time set to 0 (nek_vectors.f90:70-78)."""
        self.ctx.call("nkv_zero", self.ptr, NKV_TIME, self.ctx.stream)

    def dot(self, vec: "NekVector") -> float:
        """real_dot: weighted dot incl. ``self%time*vec%time`` (nek_vectors.f90:80-114)."""
        return self.ctx.dot(self, vec, time=True)

    def scal(self, alpha: float) -> None:
        """real_scal: all fields and time scaled (nek_vectors.f90:116-125)."""
        self.ctx.call("nkv_scal", self.ptr, float(alpha), NKV_TIME, self.ctx.stream)

    def axpby(self, alpha: float, vec: "NekVector", beta: float) -> None:
        """real_axpby: self <- alpha*self + beta*vec; ``time`` is NOT updated (nek_vectors.f90:127-139)."""
        self.ctx.call("nkv_axpby", self.ptr, float(alpha), vec.ptr, float(beta), 0, self.ctx.stream)

    # ---- conveniences ------------------------------------------------------------------------
    def copy_from(self, src: "NekVector", time: bool = True) -> None:
        self.ctx.call("nkv_copy", self.ptr, src.ptr, NKV_TIME if time else 0, self.ctx.stream)

    def norm(self) -> float:
        return float(np.sqrt(self.ctx.dot(self, self, time=self.ctx.time_in_dot)))

    @property
    def time(self) -> float:
        return float(self.storage[self.ctx.layout.time_offset].item())

    @time.setter
    def time(self, value: float) -> None:
        self.storage[self.ctx.layout.time_offset] = float(value)

    def fill_hash(self, seed: int) -> None:
        """Shard-independent synthetic data in [-1, 1) (include/nekkrylov.h nkv_fill_hash)."""
        lay = self.ctx.layout
        self.ctx.call("nkv_fill_hash", self.ptr, int(seed) & (2**64 - 1), lay.v_offset, lay.p_offset, self.ctx.stream)

    def from_fields(self, fields: dict, time: float = 0.0) -> "NekVector":
        """Upload host arrays ``{'vx':…, 'vy':…, ['vz'], ['t1'…], 'pr'}`` (this rank's shard)."""
        host = torch.zeros(self.ctx.layout.ld, dtype=torch.float64)
        for name, start, n in self.ctx.layout.field_slices():
            if n:
                host[start:start + n] = torch.as_tensor(np.asarray(fields[name], dtype=np.float64).reshape(-1))
        host[self.ctx.layout.time_offset] = time
        self.storage.copy_(host.to(self.ctx.device))
        return self

    def to_fields(self) -> dict:
        host = self.storage.detach().cpu().numpy()
        out = {name: host[s:s + n].copy() for name, s, n in self.ctx.layout.field_slices()}
        out["time"] = float(host[self.ctx.layout.time_offset])
        return out

    def from_packed(self, packed: np.ndarray) -> "NekVector":
        """Upload a padded host vector of length ``ld`` (the device layout verbatim)."""
        self.storage.copy_(torch.as_tensor(np.asarray(packed, dtype=np.float64)).to(self.ctx.device))
        return self

    def to_packed(self) -> np.ndarray:
        return self.storage.detach().cpu().numpy().copy()


class ComplexNekVector:
    """cmplx_nek_vector{re, im}: dot = re.re + im.im (nek_vectors.f90:33-42,143-203)."""

    def __init__(self, re: NekVector, im: NekVector):
        self.re, self.im = re, im

    def zero(self) -> None:
        self.re.zero()
        self.im.zero()

    def dot(self, vec: "ComplexNekVector") -> float:
        return self.re.dot(vec.re) + self.im.dot(vec.im)

    def scal(self, alpha: float) -> None:
        self.re.scal(alpha)
        self.im.scal(alpha)

    def axpby(self, alpha: float, vec: "ComplexNekVector", beta: float) -> None:
        self.re.axpby(alpha, vec.re, beta)
        self.im.axpby(alpha, vec.im, beta)


class Basis:
    """``k`` vectors in ONE contiguous allocation at stride ``ld`` (column c = Q + c*ld)."""

    def __init__(self, ctx: NekContext, k: int):
        self.ctx = ctx
        self.k = k
        self.storage = torch.zeros((k, ctx.layout.ld), dtype=torch.float64, device=ctx.device)
        self._ptr = self.storage.data_ptr()          # the allocation never moves
        self._stride = ctx.layout.ld * 8

    @property
    def ptr(self) -> int:
        return self._ptr

    def __len__(self) -> int:
        return self.k

    def __getitem__(self, i: int) -> NekVector:
        if not -self.k <= i < self.k:
            raise IndexError(i)
        return NekVector(self.ctx, self.storage[i])

    def col_ptr(self, i: int) -> int:
        if not 0 <= i < self.k:
            raise IndexError(i)
        return self._ptr + i * self._stride


# ---------------------------------------------------------------------------------------------
# legacy krylov_vector API (core/krylov_subspace.f90:26-209).  ``time`` always follows updates.
# ---------------------------------------------------------------------------------------------

def k_dot(p: NekVector, q: NekVector) -> float:
    """alpha = <p, q>_W (+ p%time*q%time iff uparam(1)==2.1), NaN -> error (:26-60)."""
    return p.ctx.dot(p, q, time=p.ctx.time_in_dot)


def k_norm(p: NekVector) -> float:
    return float(np.sqrt(k_dot(p, p)))


def k_normalize(p: NekVector) -> float:
    """alpha = ||p||; p <- p * (1/alpha) (all fields + time) (:75-92).  Returns alpha."""
    ctx = p.ctx
    out = ctx.scal[1:2]
    ctx.dot_dev(p, p, out, time=ctx.time_in_dot)
    beta = ctx.scal[2:3]
    ctx.call("nkv_normalize_dev", p.ptr, _ptr(out), _ptr(beta), NKV_TIME, ctx.stream)
    return float(beta.item())


def k_cmult(p: NekVector, c: float) -> None:
    p.ctx.call("nkv_scal", p.ptr, float(c), NKV_TIME, p.ctx.stream)


def k_add2(p: NekVector, q: NekVector) -> None:
    p.ctx.call("nkv_axpby", p.ptr, 1.0, q.ptr, 1.0, NKV_TIME, p.ctx.stream)


def k_sub2(p: NekVector, q: NekVector) -> None:
    p.ctx.call("nkv_axpby", p.ptr, 1.0, q.ptr, -1.0, NKV_TIME, p.ctx.stream)


def k_sub3(p: NekVector, q: NekVector, r: NekVector) -> None:
    """p = q - r (:129-139)."""
    p.ctx.call("nkv_sub3", p.ptr, q.ptr, r.ptr, NKV_TIME, p.ctx.stream)


def k_zero(p: NekVector) -> None:
    p.ctx.call("nkv_zero", p.ptr, NKV_TIME, p.ctx.stream)


def k_copy(p: NekVector, q: NekVector) -> None:
    """p <- q, fields and time (:152-161)."""
    p.ctx.call("nkv_copy", p.ptr, q.ptr, NKV_TIME, p.ctx.stream)


def k_matmul(dq: NekVector, Q: Basis, y, k: int) -> None:
    """dq = sum_i y_i Q(i) over all fields incl. pressure, time = dot(times, y) (:163-209).

    The reference first copies the basis into per-field 2-D temporaries; here the combination
    streams the resident basis once (NKV_OVERWRITE block update)."""
    ctx = dq.ctx
    yd = ctx.h1[:k]
    yd.copy_(torch.as_tensor(np.asarray(y, dtype=np.float64)[:k]).to(ctx.device))
    ctx.call("nkv_block_update", _ptr(ctx.w), Q.ptr, int(k), _ptr(yd), dq.ptr, None, _ptr(ctx.ws),
             NKV_OVERWRITE | NKV_TIME, ctx.stream)


def combine(out: NekVector, Q: Basis, y: torch.Tensor, k: int, with_time: bool = True) -> None:
    """out = Q[:, :k] y with ``y`` already a device tensor (mode reconstruction, a19)."""
    ctx = out.ctx
    ctx.call("nkv_block_update", _ptr(ctx.w), Q.ptr, int(k), _ptr(y), out.ptr, None, _ptr(ctx.ws),
             NKV_OVERWRITE | (NKV_TIME if with_time else 0), ctx.stream)


# ---------------------------------------------------------------------------------------------
# the in-tree solver's own inner product (core/eigensolvers.f90:3-116): weighted fields only —
# pressure and time never enter, whatever uparam(1) says.
# ---------------------------------------------------------------------------------------------

def inner_product(p: NekVector, q: NekVector) -> float:
    """alpha = sum over vx, vy, [vz], scalars of glsc3(p_f, bm1s, q_f) (eigensolvers.f90:3-56)."""
    return p.ctx.dot(p, q, time=False)


def norm(q: NekVector) -> float:
    """sqrt(inner_product(q, q)) (eigensolvers.f90:60-74)."""
    return float(np.sqrt(inner_product(q, q)))


def normalize(q: NekVector) -> float:
    """q <- q / norm(q) by nopcmult: every field incl. pressure, ``time`` untouched
    (eigensolvers.f90:78-116).  Returns the norm; device-side, one host read for the return."""
    ctx = q.ctx
    out = ctx.scal[1:2]
    ctx.dot_dev(q, q, out, time=False)
    beta = ctx.scal[2:3]
    to = ctx.layout.time_offset
    t_keep = ctx.scal[6:7]
    t_keep.copy_(q.storage[to:to + 1])          # nkv_normalize_dev scales every row, time included
    ctx.call("nkv_normalize_dev", q.ptr, _ptr(out), _ptr(beta), 0, ctx.stream)
    q.storage[to:to + 1].copy_(t_keep)
    return float(beta.item())


__all__ = [
    "NekContext", "NekVector", "ComplexNekVector", "Basis", "k_dot", "k_norm", "k_normalize", "k_cmult",
    "k_add2", "k_sub2", "k_sub3", "k_zero", "k_copy", "k_matmul", "combine", "NKV_NORM2",
    "inner_product", "norm", "normalize",
]
