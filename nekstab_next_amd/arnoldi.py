"""Arnoldi factorisation and Gram–Schmidt orthogonalisation on the GPU.

Reference: ``arnoldi_factorization(Q, H, mstart, mend, ksize)`` and
``update_hessenberg_matrix(H, f, q, k)`` (core/krylov_decomposition.f90:2-99, 103-189).  The
reference orthogonalises f against q_1..q_k by modified Gram–Schmidt (copy -> dot -> cmult ->
sub2 per column, :155-168), repeats the pass for full re-orthogonalisation (:171-180) with
H(i,k) = alpha_1 + alpha_2, then normalises f and stores H(k+1,k) = ||f||_W (:183-186);
Q(k+1) <- f (:81).

Two orthogonalisation modes share the rest of the path:

* ``"cgs2"`` (default, the MI355X hot path): block classical Gram–Schmidt applied twice —
  ``h1 = Q^T W f`` (one multi-dot kernel + ONE length-j all-reduce); then ``f -= Q h1`` fused with
  ``h2 = Q^T W f`` in a single read of Q (+ all-reduce); ``f -= Q h2`` with the ||f||_W^2 partial
  fused (+ all-reduce); one kernel writing q_{k+1} = f/||f|| and the H column (h1 + h2, ||f||) on
  the device.  ~3jN streamed doubles per step instead of the reference's ~20jN, and 3
  collectives instead of (2k+2)*n_fields.
* ``"dcgs2"``: classical Gram–Schmidt with DELAYED re-orthogonalisation (low-synchronisation
  CGS2, cf. Świrydowicz et al. 2020, Bielich et al. 2022): step j projects A q_j once against the
  basis while re-orthogonalising the still-provisional q_j in the same pass — one two-vector
  multi-dot over Q (+ one all-reduce of 2j), a small device kernel that corrects the previous H
  column and derives the coefficients, one update pass over Q that finalises q_j and writes the
  projected f straight into the next basis column (+ the ||f||^2 all-reduce; f is normalised one
  step later, inside the same passes).  Two reads of Q per step instead of three, no separate
  normalisation pass; the last vector of a factorisation is re-orthogonalised and normalised once
  at the end, so on return Q and H are exactly an Arnoldi factorisation, as with cgs2.
* ``"dcgs2-native"``: the same DCGS2 sequence orchestrated inside the library by ONE C-ABI call
  (``nkv_arnoldi_dcgs2``), the operator and the all-reduce passed as callbacks — the entry a
  Fortran/C host binds to replace ``arnoldi_factorization`` whole; bit-identical to ``"dcgs2"``.
* ``"cgs2-native"``: the ``"cgs2"`` step as ONE library call per column (``nkv_update_hessenberg``,
  the reference's ``update_hessenberg_matrix`` entry), the all-reduce as a callback.
* ``"mgs2"`` (reference operation order, for parity studies): the reference's two sequential
  MGS passes, one weighted dot + all-reduce + axpy per column.
* ``"mgs2-icwy"``: the same two MGS passes in inverse compact WY form (Świrydowicz et al. 2020):
  each pass's coefficients come from the classical dots b = Q^T W f through alpha = (I + L)^{-1} b,
  L the strictly lower part of the basis's Gram matrix (kept on the device, one row per step from
  the step's own two-vector multi-dot), so a step reads Q three times, like ``"cgs2"``.  Equal to
  MGS in exact arithmetic for ANY basis, which is what the reference's non-orthonormal bases need
  (the unnormalised noise/load seed, eigensolvers.f90:192-223; a restart with time in k_dot), where
  classical Gram–Schmidt gives a different factorisation.  Whole factorisations only
  (``arnoldi_factorization``): the Gram rows of the columns before ``mstart`` are rebuilt first.
  ``"mgs2-icwy-native"``: the same sequence inside the library (``nkv_arnoldi_factorization`` with
  ``NKV_MGS_ICWY``), bit-identical.
* ``"mgs2-lagged"``: the same MGS2 coefficients for ANY basis with TWO reads of Q per step: the
  second pass of a column is lagged into the next step's two-vector multi-dot as in DCGS2, with the
  Gram matrix G = Q^T W Q in the algebra (``lagged_coefficients``: beta = (I+L)^-1 p finishes the
  provisional column, the Arnoldi relation gives A q from A u, alpha = (I+L)^-1 Q^T W A q starts
  the next one) and the DCGS2 dual-update kernel applying it.  G and H are kept on the host, so a
  step synchronises once (one download of the 2j dots); the rows of the columns before ``mstart``
  are rebuilt from the basis at the start of a factorisation, as for ``"mgs2-icwy"``.  Prototype
  and the numerics against column-by-column MGS2: ``tools/proto_nonorth_dcgs2.py``.
  ``"mgs2-lagged-native"``: the same sequence inside the library (``nkv_arnoldi_factorization`` with
  ``NKV_MGS_LAGGED``), bit-identical (the host algebra is the library's ``nkv_lagged_coef`` in both).

No step synchronises the host (except in ``"mgs2-lagged"``): H lives on the device until the
factorisation ends.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from ._lib import NKV_NORM2, NKV_TIME, NKV_TIME_DOT, NKV_X_IS_LAST
from .operators import LinearOperator
from .vector import Basis, NekContext, NekVector


class HessenbergDev:
    """Device copy of the caller-owned (k+1) x k Hessenberg matrix (column-major as the reference).

    Stored as a (k, k+1) row-major tensor, so column c of H is the contiguous row c."""

    def __init__(self, ctx: NekContext, k: int):
        self.ctx, self.k = ctx, k
        self.t = torch.zeros((k, k + 1), dtype=torch.float64, device=ctx.device)

    def col_ptr(self, c: int) -> int:
        return self.t[c].data_ptr()

    def download(self) -> np.ndarray:
        """H as a (k+1, k) Fortran-ordered numpy array."""
        return np.asfortranarray(self.t.detach().cpu().numpy().T)

    def upload(self, H: np.ndarray) -> None:
        self.t.copy_(torch.as_tensor(np.ascontiguousarray(np.asarray(H, dtype=np.float64).T)).to(self.ctx.device))


def update_hessenberg_matrix(ctx: NekContext, Q: Basis, k: int, f: NekVector, Hd: HessenbergDev,
                             mode: str = "cgs2") -> None:
    """Orthonormalise f against Q[0:k], write Q[k] = f/||f|| and H column k-1 (1-based k, as the
    reference's ``update_hessenberg_matrix(H(1:k+1,1:k), f, Q(1:k), k)``)."""
    j = int(k)
    if j + 1 > Q.k or j > ctx.max_cols:
        raise ValueError(f"step {j} exceeds basis size {Q.k} / max_cols {ctx.max_cols}")
    orthonormalize(ctx, Q, j, f, Q.col_ptr(j), Hd.col_ptr(j - 1), mode)


def orthonormalize(ctx: NekContext, Q: Basis, j: int, f: NekVector, out_ptr: int, hcol_ptr: int,
                   mode: str = "cgs2") -> None:
    """Two-pass Gram–Schmidt of f against Q[0:j] (W inner product), then out = f/||f||; the
    projection coefficients h1+h2 go to hcol[0:j] and ||f|| to hcol[j] (device memory).  j = 0
    only normalises."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    if mode == "mgs2-icwy":
        raise ValueError("mode 'mgs2-icwy' keeps the basis's Gram matrix across steps: run it through "
                         "arnoldi_factorization (or use 'mgs2' for a single step)")
    if mode in ("cgs2-native", "mgs2-native"):   # the cgs2 / mgs2 sequence as ONE library call
        scratch = _native_scratch(ctx, j)
        errors = []
        ar_c = _allreduce_callback(ctx, scratch, errors)
        flags = (NKV_TIME_DOT if ctx.time_in_dot else 0) | (_lib.NKV_MGS2 if mode == "mgs2-native" else 0)
        rc = ctx.lib.nkv_update_hessenberg(ctx._Lp, w, Q.ptr, int(j), f.ptr, out_ptr, hcol_ptr, scratch.data_ptr(), ws,
                                           ar_c, None, flags, st)
        if errors:
            raise errors[0]
        _lib.check(rc, "nkv_update_hessenberg")
        return
    if j == 0:
        tf = NKV_TIME if ctx.time_in_dot else 0
        nrm = ctx.scal[3:4]
        ctx.call("nkv_dot", w, f.ptr, f.ptr, nrm.data_ptr(), ws, tf, st)
        ctx.comm.allreduce_(nrm)
        ctx.call("nkv_arnoldi_finish", f.ptr, nrm.data_ptr(), out_ptr, 0, ctx.h1.data_ptr(), None, hcol_ptr, 0, st)
        return
    tf = NKV_TIME if ctx.time_in_dot else 0
    h1, h2, nrm = ctx.h1[:j], ctx.h2[:j], ctx.scal[3:4]
    if mode == "cgs2":
        lay, tm = ctx.layout, ctx.timer
        # algorithmic bytes: a dot reads j weighted columns + f_w + w; an update
        # reads j full columns + f and writes f (+ w for the fused norm)
        b_dot = 8.0 * (j * lay.N_w + lay.N_w + lay.n_v)
        b_upd = 8.0 * (j * lay.N + 2 * lay.N)
        if tm:
            tm.begin("block_dot")
        ctx.call("nkv_block_dot", w, Q.ptr, j, f.ptr, h1.data_ptr(), ws, tf, st)
        if tm:
            tm.end("block_dot", b_dot)
        ctx.comm.allreduce_(h1)
        # f -= Q h1 and h2 = Q^T W f in ONE pass over Q
        if tm:
            tm.begin("update_dot")
        ctx.call("nkv_block_update_dot", w, Q.ptr, j, h1.data_ptr(), f.ptr, h2.data_ptr(), ws,
                 NKV_TIME | (NKV_TIME_DOT if tf else 0), st)
        if tm:
            tm.end("update_dot", b_upd + 8.0 * lay.n_v)
        ctx.comm.allreduce_(h2)
        if tm:
            tm.begin("block_update")
        ctx.call("nkv_block_update", w, Q.ptr, j, h2.data_ptr(), f.ptr, nrm.data_ptr(), ws,
                 NKV_TIME | NKV_NORM2 | (NKV_TIME_DOT if tf else 0), st)
        if tm:
            tm.end("block_update", b_upd + 8.0 * lay.n_v)
        ctx.comm.allreduce_(nrm)
    elif mode == "mgs2":
        # the reference's order (:155-186): alpha_0 by a dot, then per column one fused pass
        # (nkv_axpy_dot: f -= alpha_i q_i and the next coefficient — alpha_{i+1}, the second pass's
        # alpha_0, or finally ||f||^2 — from the same read of f), each coefficient all-reduced
        ctx.call("nkv_dot", w, f.ptr, Q.col_ptr(0), h1[0:1].data_ptr(), ws, tf, st)
        ctx.comm.allreduce_(h1[0:1])
        fl = NKV_TIME | (NKV_TIME_DOT if tf else 0)
        for p, h in enumerate((h1, h2)):
            for i in range(j):
                last = i + 1 == j
                qn = Q.col_ptr(i + 1) if not last else (Q.col_ptr(0) if p == 0 else None)
                out = h[i + 1:i + 2] if not last else (h2[0:1] if p == 0 else nrm)
                ctx.call("nkv_axpy_dot", w, f.ptr, h[i:i + 1].data_ptr(), Q.col_ptr(i), qn, out.data_ptr(), ws, fl,
                         st)
                ctx.comm.allreduce_(out)
    else:
        raise ValueError(f"unknown orthogonalisation mode {mode!r}")
    if ctx.timer:
        ctx.timer.begin("finish")
    ctx.call("nkv_arnoldi_finish", f.ptr, nrm.data_ptr(), out_ptr, j, h1.data_ptr(), h2.data_ptr(),
             hcol_ptr, 0, st)
    if ctx.timer:
        ctx.timer.end("finish", 16.0 * ctx.layout.N)


def _dcgs2_step(ctx: NekContext, Q: Basis, Hd: HessenbergDev, j: int, f: NekVector, first: bool,
                nrm2: torch.Tensor | None = None) -> None:
    """Step j (1-based) of DCGS2 Arnoldi: Q[0:j-1] final, Q[j-1] = u = beta q_j provisional and not
    yet normalised (unless ``first``: then u is normalised), f = A u.  On return Q[j-1] is final,
    Q[j] = the next u, H columns 0..j-2 final and column j-1 provisional, H(j, j-1) pending.
    beta^2 = u^T W u is the last entry of the step's own Q^T W u, so one all-reduce per step.

    ``nrm2`` (a 1-double device tensor): the update also forms ||next u||_W^2, fused, and all-reduces
    it into ``nrm2`` (one more all-reduce); that value is then this step's H(j, j-1) estimate (per-
    column consumers: the GMRES residual test) and the next step's beta^2.  Pass the same tensor
    to every step of the factorisation."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    lay, tm = ctx.layout, ctx.timer
    tf = NKV_TIME if ctx.time_in_dot else 0
    m = j - 1
    h = ctx.hd[: 2 * j]
    hp, cp = h.data_ptr(), ctx.coef.data_ptr()   # raw pointers: few host objects per step
    u = Q.col_ptr(m)
    if tm:
        tm.begin("block_dot2")
    ctx.call("nkv_block_dot2", w, Q.ptr, j, u, f.ptr, hp, ws, tf | NKV_X_IS_LAST, st)
    if tm:
        tm.end("block_dot2", 8.0 * ((j - 1) * lay.N_w + 2 * lay.N_w + lay.n_v))
    ctx.comm.allreduce_(h)
    nprev = None if first else (nrm2.data_ptr() if nrm2 is not None else hp + 8 * m)
    ctx.call_nl("nkv_dcgs2_coef", m, hp, hp + 8 * j, nprev, Hd.t.data_ptr(), Hd.k + 1, cp, ws, st)
    if tm:
        tm.begin("dcgs2_update")
    ctx.call("nkv_dcgs2_update", w, Q.ptr, m, cp, u, f.ptr, Q.col_ptr(j), None if nrm2 is None else nrm2.data_ptr(),
             ws, NKV_TIME | (NKV_TIME_DOT if tf else 0), st)
    if tm:
        tm.end("dcgs2_update", 8.0 * (m * lay.N + 4 * lay.N) + (0.0 if nrm2 is None else 8.0 * lay.n_v))
    if nrm2 is not None:
        ctx.comm.allreduce_(nrm2)


def _dcgs2_close(ctx: NekContext, Q: Basis, Hd: HessenbergDev, m: int) -> None:
    """Re-orthogonalise and normalise the provisional Q[m] = u against Q[0:m], fill in H(m, m-1)
    and correct H row m (end of a DCGS2 factorisation of m steps)."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    lay, tm = ctx.layout, ctx.timer
    tf = NKV_TIME if ctx.time_in_dot else 0
    h, coef = ctx.hd[: m + 1], ctx.coef
    u = Q.col_ptr(m)
    if tm:
        tm.begin("block_dot")
    ctx.call("nkv_block_dot", w, Q.ptr, m + 1, u, h.data_ptr(), ws, tf, st)
    if tm:
        tm.end("block_dot", 8.0 * ((m + 1) * lay.N_w + lay.N_w + lay.n_v))
    ctx.comm.allreduce_(h)
    ctx.call_nl("nkv_dcgs2_coef", m, h.data_ptr(), None, h.data_ptr() + 8 * m, Hd.t.data_ptr(), Hd.k + 1,
                coef.data_ptr(), ws, st)
    if tm:
        tm.begin("block_update")
    ctx.call("nkv_block_update", w, Q.ptr, m, h.data_ptr(), u, None, ws, NKV_TIME, st)
    if tm:
        tm.end("block_update", 8.0 * (m * lay.N + 2 * lay.N))
    ctx.call("nkv_normalize_dev", u, coef[2 * m + 3:].data_ptr(), None, 0, st)


def _icwy_gram(ctx: NekContext, Q: Basis, mstart: int) -> torch.Tensor:
    """The row-major Gram matrix of ``"mgs2-icwy"`` (kept on the context, ld = max_cols + 1), with
    the rows of columns 1..mstart-2 rebuilt from the basis as it stands (after a restart the kept
    columns are new vectors; row mstart-1 comes from the first step's own multi-dot)."""
    ldg = ctx.max_cols + 1
    G = getattr(ctx, "_icwy_G", None)
    if G is None:
        G = ctx._icwy_G = torch.zeros((ldg, ldg), dtype=torch.float64, device=ctx.device)
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    tf = NKV_TIME if ctx.time_in_dot else 0
    for i in range(1, mstart - 1):
        ctx.call("nkv_block_dot", w, Q.ptr, i, Q.col_ptr(i), G[i].data_ptr(), ws, tf, st)
        ctx.comm.allreduce_(G[i, :i])
    return G


def _icwy_step(ctx: NekContext, Q: Basis, Hd: HessenbergDev, j: int, f: NekVector, G: torch.Tensor) -> None:
    """Step j (1-based) of ``"mgs2-icwy"``: f = A q_{j-1} is orthogonalised against Q[0:j] by two MGS
    passes in inverse compact WY form; Q[j] = f/||f||, H column j-1 = alpha_1 + alpha_2, ||f||."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    lay, tm = ctx.layout, ctx.timer
    tf = NKV_TIME if ctx.time_in_dot else 0
    ldg = G.shape[1]
    h = ctx.hd[: 2 * j]
    hp, gp = h.data_ptr(), G.data_ptr()
    h1, h2, nrm = ctx.h1[:j], ctx.h2[:j], ctx.scal[3:4]
    if tm:
        tm.begin("block_dot2")
    # [Q^T W q_{j-1} (the Gram row of the newest column) ; Q^T W f (pass-1 classical dots)]
    ctx.call("nkv_block_dot2", w, Q.ptr, j, Q.col_ptr(j - 1), f.ptr, hp, ws, tf | NKV_X_IS_LAST, st)
    if tm:
        tm.end("block_dot2", 8.0 * ((j - 1) * lay.N_w + 2 * lay.N_w + lay.n_v))
    ctx.comm.allreduce_(h)
    ctx.call_nl("nkv_mgs_icwy_solve", j, gp, ldg, hp, hp + 8 * j, h1.data_ptr(), st)
    b_upd = 8.0 * (j * lay.N + 2 * lay.N)
    if tm:
        tm.begin("update_dot")
    ctx.call("nkv_block_update_dot", w, Q.ptr, j, h1.data_ptr(), f.ptr, h2.data_ptr(), ws,
             NKV_TIME | (NKV_TIME_DOT if tf else 0), st)
    if tm:
        tm.end("update_dot", b_upd + 8.0 * lay.n_v)
    ctx.comm.allreduce_(h2)
    ctx.call_nl("nkv_mgs_icwy_solve", j, gp, ldg, None, h2.data_ptr(), h2.data_ptr(), st)
    if tm:
        tm.begin("block_update")
    ctx.call("nkv_block_update", w, Q.ptr, j, h2.data_ptr(), f.ptr, nrm.data_ptr(), ws, NKV_TIME | NKV_NORM2 | (NKV_TIME_DOT if tf else 0), st)
    if tm:
        tm.end("block_update", b_upd + 8.0 * lay.n_v)
    ctx.comm.allreduce_(nrm)
    if tm:
        tm.begin("finish")
    ctx.call("nkv_arnoldi_finish", f.ptr, nrm.data_ptr(), Q.col_ptr(j), j, h1.data_ptr(), h2.data_ptr(),
             Hd.col_ptr(j - 1), 0, st)
    if tm:
        tm.end("finish", 16.0 * lay.N)



def lagged_coefficients(G: np.ndarray, H: np.ndarray, hv: np.ndarray, c: int, stage: int) -> np.ndarray:
    """Host algebra of one ``"mgs2-lagged"`` step at column c (0-based), ``nkv_lagged_coef`` of the
    library (drivers.hip; the one-call driver runs the same function, so the two paths are
    bit-identical).  G: the Gram matrix (row-major float64, (max_cols+1)^2), H: the Hessenberg
    matrix (Fortran-ordered (k+1, k)), both updated in place.

    ``stage`` 1 — the first step of a factorisation (Q[c] final): ``hv`` = [Q[0:c+1]^T W q_c ;
    Q[0:c+1]^T W A q_c]; G's row c, then one MGS pass alpha = (I+L)^-1 Q^T W A q_c starts column
    c+1 (L the strictly lower part of G).
    ``stage`` 0 — Q[c] holds u, the previous step's first-pass result, which the reference's second
    pass would turn into f2 = u - Q[0:c] beta, beta = (I+L)^-1 p (p = Q[0:c]^T W u); q_c = f2 / r with
    r^2 = u.u - 2 beta.p + beta^T G beta, H(0:c, c-1) += beta, H(c, c-1) = r, G's new row
    (p - G beta) / r; and, from y = A u and the Arnoldi relation of the finished columns,
    A q_c = (y - Q[0:c+1] H[0:c+1, 0:c] beta) / r, so column c+1's first pass is
    alpha = (I+L)^-1 ([t ; (u.y - beta.t)/r] - G H beta) / r (t = Q[0:c]^T W y) and
    u_next = y / r - Q[0:c+1] (H beta / r + alpha).  With G = I this is DCGS2's algebra.
    Returns nkv_dcgs2_update's coefficient vector [x (c) | . (c+1) | 1/r, y, ., 1 | beta (c)].
    ``stage`` 2 — the closing pass of the last column c: ``hv`` = Q[0:c]^T W u; returns beta in
    coef[0:c] (H(0:c, c-1) += beta).  A column with no new direction raises NkvNaNError."""
    if not (G.dtype == H.dtype == np.float64 and G.flags.c_contiguous and H.flags.f_contiguous):
        raise ValueError("lagged_coefficients: G row-major and H column-major float64 arrays")
    hv = np.ascontiguousarray(hv, dtype=np.float64)
    coef = np.zeros(3 * c + 5)
    rc = _lib.load().nkv_lagged_coef(int(c), int(stage), hv.ctypes.data, G.ctypes.data, G.shape[1], H.ctypes.data,
                                     H.shape[0], coef.ctypes.data)
    _lib.check(rc, "nkv_lagged_coef")
    return coef


def _lagged_gram(ctx: NekContext, Q: Basis, mstart: int) -> np.ndarray:
    """Host Gram matrix of ``"mgs2-lagged"`` ((max_cols+1)^2), rows and diagonal of columns
    0..mstart-2 rebuilt from the basis as it stands (row mstart-1 comes from the first step's
    multi-dot)."""
    k1 = ctx.max_cols + 1
    G = np.zeros((k1, k1))
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    tf = NKV_TIME if ctx.time_in_dot else 0
    for i in range(0, mstart - 1):
        h = ctx.h1[: i + 1]
        ctx.call("nkv_block_dot", w, Q.ptr, i + 1, Q.col_ptr(i), h.data_ptr(), ws, tf, st)
        ctx.comm.allreduce_(h)
        row = h.cpu().numpy()
        G[i, : i + 1] = G[: i + 1, i] = row
    return G


def _lagged_step(ctx: NekContext, Q: Basis, H: np.ndarray, G: np.ndarray, j: int, f: NekVector,
                 first: bool) -> None:
    """Step j (1-based; c = j-1) of ``"mgs2-lagged"``: f = A Q[c]; one two-vector multi-dot over
    Q[0:j]; the host algebra (:func:`lagged_coefficients`); one dual update finishing Q[c] and
    writing the next provisional column Q[j]."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    lay, tm = ctx.layout, ctx.timer
    tf = NKV_TIME if ctx.time_in_dot else 0
    c = j - 1
    h = ctx.hd[: 2 * j]
    if tm:
        tm.begin("block_dot2")
    ctx.call("nkv_block_dot2", w, Q.ptr, j, Q.col_ptr(c), f.ptr, h.data_ptr(), ws, tf | NKV_X_IS_LAST, st)
    if tm:
        tm.end("block_dot2", 8.0 * ((j - 1) * lay.N_w + 2 * lay.N_w + lay.n_v))
    ctx.comm.allreduce_(h)
    coef = lagged_coefficients(G, H, h.cpu().numpy(), c, 1 if first else 0)
    cd = ctx.coef[: coef.size]
    cd.copy_(torch.from_numpy(coef))
    if tm:
        tm.begin("dcgs2_update")
    ctx.call("nkv_dcgs2_update", w, Q.ptr, c, cd.data_ptr(), Q.col_ptr(c), f.ptr, Q.col_ptr(j), None, ws,
             NKV_TIME | (NKV_TIME_DOT if tf else 0), st)
    if tm:
        tm.end("dcgs2_update", 8.0 * (c * lay.N + 4 * lay.N))


def _lagged_close(ctx: NekContext, Q: Basis, H: np.ndarray, G: np.ndarray, m: int) -> None:
    """Finish the provisional Q[m] (the reference's second pass and k_normalize of the last column):
    beta = (I+L)^-1 Q[0:m]^T W u, u <- u - Q[0:m] beta, H(0:m, m-1) += beta, H(m, m-1) = ||u||_W,
    Q[m] = u / ||u||_W."""
    w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
    tf = NKV_TIME if ctx.time_in_dot else 0
    h, hb, nrm, bet = ctx.h1[: m + 1], ctx.h2[:m], ctx.scal[3:4], ctx.scal[4:5]
    ctx.call("nkv_block_dot", w, Q.ptr, m + 1, Q.col_ptr(m), h.data_ptr(), ws, tf, st)
    ctx.comm.allreduce_(h)
    beta = lagged_coefficients(G, H, h.cpu().numpy(), m, 2)[:m]
    hb.copy_(torch.from_numpy(beta))
    ctx.call("nkv_block_update", w, Q.ptr, m, hb.data_ptr(), Q.col_ptr(m), nrm.data_ptr(), ws,
             NKV_TIME | NKV_NORM2 | (NKV_TIME_DOT if tf else 0), st)
    ctx.comm.allreduce_(nrm)
    ctx.call("nkv_normalize_dev", Q.col_ptr(m), nrm.data_ptr(), bet.data_ptr(), 0, st)
    H[m, m - 1] = float(bet.item())
    if not (np.isfinite(H[m, m - 1]) and H[m, m - 1] > 0.0):
        raise _lib.NkvNaNError(_lib.NKV_ENAN, "mgs2-lagged",
                               f"the last column has no new direction (||u|| = {H[m, m - 1]!r})")


def _lagged_factorization(ctx: NekContext, op: LinearOperator, Q: Basis, Hd: HessenbergDev, mstart: int,
                          mend: int, f: NekVector, transpose: bool, on_step=None) -> None:
    """``"mgs2-lagged"`` from column ``mstart`` to ``mend`` (1-based): H on the host for the whole
    factorisation (uploaded before each hook and at the end)."""
    G = _lagged_gram(ctx, Q, mstart)
    H = Hd.download()
    for mstep in range(mstart, mend + 1):
        (op.rmatvec if transpose else op.matvec)(Q[mstep - 1], f)
        _lagged_step(ctx, Q, H, G, mstep, f, first=(mstep == mstart))
        if on_step is not None and mstep > mstart:   # column mstep-1 is final after step mstep
            Hd.upload(H)
            on_step(mstep - 1)
    _lagged_close(ctx, Q, H, G, mend)
    Hd.upload(H)
    if on_step is not None:
        on_step(mend)

def _native_scratch(ctx: NekContext, m: int) -> torch.Tensor:
    """Device scratch of the one-call drivers (nkv_arnoldi_scratch_doubles), kept on the context."""
    need = int(ctx.lib.nkv_arnoldi_scratch_doubles(max(int(m), ctx.max_cols)))
    scratch = getattr(ctx, "_arnoldi_scratch", None)
    if scratch is None or scratch.numel() < need:
        scratch = ctx._arnoldi_scratch = torch.zeros(need, dtype=torch.float64, device=ctx.device)
    return scratch


def _allreduce_callback(ctx: NekContext, scratch: torch.Tensor, errors: list):
    """The all-reduce callback of the one-call drivers: in-place SUM of a slice of ``scratch``
    through the context's communicator (a typed NULL on one rank without forced collectives)."""
    if not (ctx.comm.world > 1 or ctx.comm.force):
        return _lib.ALLREDUCE_FN()
    base, size = scratch.data_ptr(), scratch.numel()

    def allreduce(_user, buf, n, _stream):
        try:
            off, r = divmod((buf or 0) - base, 8)
            if r or off < 0 or n <= 0 or off + n > size:
                raise ValueError("one-call driver allreduce callback: buffer outside the scratch")
            ctx.comm.allreduce_(scratch[off:off + n])
            return 0
        except BaseException as e:  # noqa: BLE001 — surfaced after the call returns
            errors.append(e)
            return 1

    return _lib.ALLREDUCE_FN(allreduce)


def _dcgs2_native(ctx: NekContext, op: LinearOperator, Q: Basis, Hd: HessenbergDev, mstart: int, mend: int,
                  f: NekVector, transpose: bool, entry: str = "nkv_arnoldi_dcgs2", flags: int = 0) -> None:
    """The DCGS2 factorisation as ONE library call (``nkv_arnoldi_dcgs2``, include/nekkrylov.h): the
    C++ side runs the step sequence of ``_dcgs2_step`` / ``_dcgs2_close`` (same entry points, same
    order, so the result is bit-identical to ``mode="dcgs2"``) and calls back for the operator and
    the all-reduce — the shape a Fortran host uses to replace ``arnoldi_factorization``.
    ``entry="nkv_arnoldi_factorization"``: the per-column cgs2 (or, with ``NKV_MGS2`` in ``flags``,
    mgs2) factorisation as one call, bit-identical to those modes."""
    lib = ctx.lib
    scratch = _native_scratch(ctx, mend)
    base, ld8, fptr = Q.ptr, 8 * ctx.layout.ld, f.ptr
    apply = op.rmatvec if transpose else op.matvec
    errors = []

    def matvec(_user, x, y, _stream):
        try:
            c, r = divmod((x or 0) - base, ld8)
            if r or not 0 <= c < Q.k or y != fptr:
                raise ValueError(f"{entry} matvec callback: x={x}, y={y} are not a basis column and f")
            apply(Q[c], f)
            return 0
        except BaseException as e:  # noqa: BLE001 — surfaced after the call returns
            errors.append(e)
            return 1

    mv_c = _lib.MATVEC_FN(matvec)
    ar_c = _allreduce_callback(ctx, scratch, errors)
    rc = getattr(lib, entry)(ctx._Lp, ctx.w.data_ptr(), Q.ptr, int(mstart), int(mend), Hd.t.data_ptr(), Hd.k + 1,
                             fptr, scratch.data_ptr(), ctx.ws.data_ptr(), mv_c, None, ar_c, None,
                             (NKV_TIME_DOT if ctx.time_in_dot else 0) | flags, ctx.stream)
    if errors:
        raise errors[0]
    _lib.check(rc, entry)


def arnoldi_factorization(ctx: NekContext, op: LinearOperator, Q: Basis, Hd: HessenbergDev, mstart: int,
                          mend: int, f: NekVector | None = None, mode: str = "cgs2", transpose: bool = False,
                          on_step=None) -> None:
    """k-step Arnoldi from column ``mstart`` to ``mend`` (1-based, inclusive), as
    krylov_decomposition.f90:68-96: f = A q_mstep; orthonormalise; Q(mstep+1) = f.

    ``on_step(mstep)`` is called once column mstep (0-based: Q[mstep], the reference's Q(mstep+1))
    and H columns 0..mstep-1 are final (hook for checkpointing, cf. ifres at :84).  CGS2 and MGS2
    finish each column in its own step.  DCGS2 finishes column j-1 in step j, so its hook for
    mstep = j-1 runs right after step j (one step later than the reference's call at :84, with the
    same content), and the hook for mend after the closing pass; ``"dcgs2-native"`` with a hook
    runs this Python-driven DCGS2."""
    if mend < mstart:
        return
    if Q.k < mend + 1:
        raise ValueError("basis too small")
    if f is None:
        f = ctx.vector()
    if mode == "dcgs2-native":   # the same DCGS2 sequence, orchestrated by the library (one ABI call)
        if on_step is None:
            if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
                raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
            _dcgs2_native(ctx, op, Q, Hd, mstart, mend, f, transpose)
            return
        mode = "dcgs2"
    if mode == "dcgs2" and on_step is not None:   # lagged hooks: column j-1 is final after step j
        if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
            raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
        for mstep in range(mstart, mend + 1):
            (op.rmatvec if transpose else op.matvec)(Q[mstep - 1], f)
            _dcgs2_step(ctx, Q, Hd, mstep, f, first=(mstep == mstart))
            if mstep > mstart:
                on_step(mstep - 1)
        _dcgs2_close(ctx, Q, Hd, mend)
        on_step(mend)
        return
    if mode == "mgs2-lagged-native":   # the "mgs2-lagged" sequence inside the library (one ABI call)
        if on_step is None:
            if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
                raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
            _dcgs2_native(ctx, op, Q, Hd, mstart, mend, f, transpose, entry="nkv_arnoldi_factorization",
                          flags=_lib.NKV_MGS_LAGGED)
            return
        mode = "mgs2-lagged"
    if mode == "mgs2-lagged":
        if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
            raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
        _lagged_factorization(ctx, op, Q, Hd, mstart, mend, f, transpose, on_step)
        return
    if mode == "mgs2-icwy-native":   # the "mgs2-icwy" sequence inside the library (one ABI call)
        if on_step is None:
            if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
                raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
            _dcgs2_native(ctx, op, Q, Hd, mstart, mend, f, transpose, entry="nkv_arnoldi_factorization",
                          flags=_lib.NKV_MGS_ICWY)
            return
        mode = "mgs2-icwy"
    if mode == "mgs2-icwy":
        if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
            raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
        G = _icwy_gram(ctx, Q, mstart)
        for mstep in range(mstart, mend + 1):
            (op.rmatvec if transpose else op.matvec)(Q[mstep - 1], f)
            _icwy_step(ctx, Q, Hd, mstep, f, G)
            if on_step is not None:
                on_step(mstep)
        return
    if mode in ("cgs2-native", "mgs2-native") and on_step is None:   # per-column modes, one ABI call
        if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
            raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
        _dcgs2_native(ctx, op, Q, Hd, mstart, mend, f, transpose, entry="nkv_arnoldi_factorization",
                      flags=_lib.NKV_MGS2 if mode == "mgs2-native" else 0)
        return
    if mode == "dcgs2" and on_step is None:
        if mend > ctx.max_cols or mend + 1 > Hd.k + 1:
            raise ValueError(f"step {mend} exceeds max_cols {ctx.max_cols} / H size {Hd.k}")
        for mstep in range(mstart, mend + 1):
            (op.rmatvec if transpose else op.matvec)(Q[mstep - 1], f)
            _dcgs2_step(ctx, Q, Hd, mstep, f, first=(mstep == mstart))
        _dcgs2_close(ctx, Q, Hd, mend)
        return
    if mode == "dcgs2":
        mode = "cgs2"
    for mstep in range(mstart, mend + 1):
        x = Q[mstep - 1]
        (op.rmatvec if transpose else op.matvec)(x, f)
        update_hessenberg_matrix(ctx, Q, mstep, f, Hd, mode)
        if on_step is not None:
            on_step(mstep)


class FactorizationGraph:
    """HIP-graph replay of ``arnoldi_factorization(mstart..mend)``.

    Every launch of a factorisation (matvec kernels, the Gram–Schmidt kernels, the RCCL all-reduces
    when the process group is ``nccl``) is captured once per (mstart, mend, transpose) into a
    ``torch.cuda.CUDAGraph`` on the compute stream and replayed: no host work and no launch
    latency between kernels.  World size 1 only (see ``usable``).  All buffers (basis, H, f, workspace, partial vectors) are allocated
    before capture and never move.  The operator must be capturable (device kernels only: no host
    synchronisation in ``matvec``); a ``gloo`` group (host all-reduce) cannot be captured, so
    ``usable()`` is False for it and callers fall back to eager launches."""

    def __init__(self, ctx: NekContext, op: LinearOperator, Q: Basis, Hd: HessenbergDev, f: NekVector,
                 mode: str = "cgs2"):
        self.ctx, self.op, self.Q, self.Hd, self.f, self.mode = ctx, op, Q, Hd, f, mode
        self.graphs = {}

    # modes that synchronise with the host inside every step (the lagged MGS coefficients are solved
    # on the host from a downloaded multi-dot; the native twin synchronises its stream per step): a
    # graph capture of them fails, so they always launch eagerly
    HOST_SYNC_MODES = ("mgs2-lagged", "mgs2-lagged-native")

    def usable(self) -> bool:
        """Single rank and a capturable mode only.  Capturing RCCL all-reduces into a replayed graph
        has never run on more than one GPU (round 1 rehearsed world > 1 only as gloo ranks sharing
        one GPU), so a multi-rank factorisation always launches eagerly; ``krylov_schur`` refuses
        ``graphs=True`` at world > 1 instead of silently falling back.  The host-synchronising
        lagged modes (``HOST_SYNC_MODES``) launch eagerly at any world size."""
        return self.ctx.comm.world == 1 and self.mode not in self.HOST_SYNC_MODES

    def run(self, mstart: int, mend: int, transpose: bool = False) -> None:
        if mend < mstart:
            return
        key = (mstart, mend, transpose)
        Q = self.Q
        g = self.graphs.get(key)
        if g is None:
            timer, self.ctx.timer = self.ctx.timer, None
            g = torch.cuda.CUDAGraph()
            torch.cuda.synchronize(self.ctx.device)
            with torch.cuda.graph(g):
                arnoldi_factorization(self.ctx, self.op, Q, self.Hd, mstart, mend, f=self.f, mode=self.mode,
                                      transpose=transpose)
            self.ctx.timer = timer
            self.graphs[key] = g
        g.replay()
