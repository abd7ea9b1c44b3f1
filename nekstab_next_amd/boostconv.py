"""BoostConv residual-subspace acceleration on the device.

Reference: ``BoostConv`` / ``boostconv_core`` / ``qr_dec`` / ``linear_system``
(core/fixedp.f90:218-403).  Every ``bst_skp`` time steps the velocity residual
r_b = v - v_old is replaced by the least-squares-corrected one using two rotating subspaces of
``bst_snp`` columns (differences of residuals Y and of corrected residuals X):

    first call:  Y(:,1) = X(:,1) = r_b;  D = 1 (all ones);  rot = 1                :294-297
    otherwise :  Y(:,rot) -= r_b;  X(:,rot) -= Y(:,rot)                              :301-302
                 (Q, D) = qr_dec(Y)      single-pass MGS, columns with ||.||^2 < 1e-60 set to 0
                                          and D(j,j) = 1                              :331-385
                 c = Q^T W r_b  (W = bm1)                                             :305-308
                 c_b = D^{-1} c (back substitution, linear_system)                   :387-403
                 rot = mod(rot, bst_snp) + 1;  Y(:,rot) = r_b                         :310-311
                 r_b += X c_b;  X(:,rot) = r_b                                        :313-318

The fields are the velocities only (``opcopy`` / ``opsub2`` act on vx, vy, [vz]), so the
accelerator runs in its own velocity-only context (weights ``bm1``).  Dots, updates and the
combination are the library's device kernels; the k x k triangular solve is on the host.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib
from .layout import NekLayout
from .vector import NekContext, NekVector


def velocity_layout(lay: NekLayout) -> NekLayout:
    return NekLayout(lay.ldim, lay.lx1, lay.lx2, lay.nelgv, n_scalars=0, ifpo=False, rank=lay.rank, world=lay.world)


def linear_system(m: np.ndarray, inp: np.ndarray) -> np.ndarray:
    """Back substitution with the upper triangle of m (fixedp.f90:387-403)."""
    n = inp.shape[0]
    out = np.zeros(n)
    for j in range(n - 1, -1, -1):
        v = inp[j]
        for k in range(j + 1, n):
            v = v - m[j, k] * out[k]
        out[j] = v / m[j, j]
    return out


class BoostConv:
    def __init__(self, ctx: NekContext, bst_snp: int = 10):
        if ctx.layout.n_scalars or ctx.layout.n_p:
            raise ValueError("BoostConv works on a velocity-only context (velocity_layout)")
        self.ctx, self.n = ctx, bst_snp
        self.X, self.Y, self.Q = ctx.basis(bst_snp), ctx.basis(bst_snp), ctx.basis(bst_snp)
        self.dd = np.ones((bst_snp, bst_snp))
        self.rot = 0  # 0-based rot
        self.init = False
        self._dum = ctx.vector()
        self._r = torch.zeros(1, dtype=torch.float64, device=ctx.device)
        self._dd_dev = torch.zeros(bst_snp * bst_snp, dtype=torch.float64, device=ctx.device)   # row-major
        self._nrm_dev = torch.zeros(bst_snp, dtype=torch.float64, device=ctx.device)
        self._cc_dev = torch.zeros(bst_snp, dtype=torch.float64, device=ctx.device)

    def _dot(self, a: NekVector, b: NekVector) -> float:
        return self.ctx.dot(a, b, time=False)

    def qr_dec(self) -> None:
        """Single-pass MGS QR of Y into Q and dd, reference operation order (fixedp.f90:331-385).

        The dots and the projections stay on the device (the scalars never visit the host: one
        synchronisation per QR instead of one per dot); the reference's guard on a numerically
        zero column (norm^2 < 1e-60: Q(j) = 0, dd(j,j) = 1) needs the host, so a QR that meets one
        is redone in the host-scalar form below."""
        if not self._qr_dec_device():
            self._qr_dec_host()

    def _qr_dec_device(self) -> bool:
        ctx, n = self.ctx, self.n
        w, ws, st = ctx.w.data_ptr(), ctx.ws.data_ptr(), ctx.stream
        D, nrm = self._dd_dev, self._nrm_dev
        D.zero_()
        dum = self._dum
        for j in range(n):
            dum.copy_from(self.Y[j], time=False)
            for i in range(j):
                r = D[i * n + j: i * n + j + 1]
                ctx.call("nkv_dot", w, dum.ptr, self.Q[i].ptr, r.data_ptr(), ws, 0, st)
                ctx.comm.allreduce_(r)
                ctx.call("nkv_axpy_dev", dum.ptr, r.data_ptr(), -1.0, self.Q[i].ptr, 0, st)
            ctx.call("nkv_dot", w, dum.ptr, dum.ptr, nrm[j:j + 1].data_ptr(), ws, 0, st)
            ctx.comm.allreduce_(nrm[j:j + 1])
            # dd(j,j) = sqrt(norm^2), Q(j) = dum / dd(j,j) (the reference's scal by the reciprocal)
            ctx.call("nkv_normalize_dev", dum.ptr, nrm[j:j + 1].data_ptr(), D[j * n + j:].data_ptr(), 0, st)
            self.Q[j].copy_from(dum, time=False)
        if bool((nrm[1:] < 1e-60).any()):   # the only host synchronisation of the QR
            # the device normalised the zero column (0 * inf = NaN) and the later dots against it
            # raised the workspace NaN flag: clear it, the host form below recomputes every scalar
            # (and its own dots still flag a NaN that is really in Y)
            code = ctx.lib.nkv_check_status(ctx.ws.data_ptr(), ctx.stream)
            if code not in (_lib.NKV_OK, _lib.NKV_ENAN):
                _lib.check(code, "nkv_check_status")
            return False
        self.dd = D.view(n, n).cpu().numpy()
        if np.isnan(self.dd).any():
            ctx.check_nan()
        return True

    def _qr_dec_host(self) -> None:
        ctx, n = self.ctx, self.n
        dd = np.zeros((n, n))
        dum = self._dum
        for j in range(n):
            dum.copy_from(self.Y[j], time=False)
            for i in range(j):
                r = self._dot(dum, self.Q[i])
                dd[i, j] = r
                dum.axpby(1.0, self.Q[i], -r)
            norma = self._dot(dum, dum)
            if j == 0:
                norma = float(np.sqrt(norma))
                dum.scal(1.0 / norma)
                self.Q[0].copy_from(dum, time=False)
                dd[0, 0] = norma
                continue
            if norma < 1e-60:
                norma = 1.0
                self.Q[j].zero()
            else:
                dum.scal(1.0 / np.sqrt(norma))
                self.Q[j].copy_from(dum, time=False)
            dd[j, j] = np.sqrt(norma)
        self.dd = dd

    def core(self, rb: NekVector) -> None:
        """boostconv_core(rbx, rby, rbz): rb is corrected in place."""
        if not self.init:
            for B in (self.X, self.Y, self.Q):
                for i in range(self.n):
                    B[i].zero()
            self.Y[0].copy_from(rb, time=False)
            self.X[0].copy_from(rb, time=False)
            self.dd = np.ones((self.n, self.n))
            self.rot = 0
            self.init = True
            return
        r = self.rot
        self.Y[r].axpby(1.0, rb, -1.0)           # y_rot -= rb
        self.X[r].axpby(1.0, self.Y[r], -1.0)    # x_rot -= y_rot
        self.qr_dec()
        ctx = self.ctx
        for j in range(self.n):   # <rb, Q(j)>, one dot each as the reference; one host read for all
            c = self._cc_dev[j:j + 1]
            ctx.call("nkv_dot", ctx.w.data_ptr(), rb.ptr, self.Q[j].ptr, c.data_ptr(), ctx.ws.data_ptr(), 0, ctx.stream)
            ctx.comm.allreduce_(c)
        cc = self._cc_dev.cpu().numpy()
        if np.isnan(cc).any():
            ctx.check_nan()
        ccb = linear_system(self.dd, cc)
        self.rot = (r + 1) % self.n
        self.Y[self.rot].copy_from(rb, time=False)
        h = torch.as_tensor(-ccb).to(self.ctx.device)  # rb <- rb - X(-ccb) = rb + X ccb
        self.ctx.call("nkv_block_update", self.ctx.w.data_ptr(), self.X.ptr, self.n, h.data_ptr(), rb.ptr, None,
                      self.ctx.ws.data_ptr(), 0, self.ctx.stream)
        self.X[self.rot].copy_from(rb, time=False)
