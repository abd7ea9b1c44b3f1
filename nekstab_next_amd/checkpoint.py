"""Arnoldi checkpoint / restart (``ifres``) — SURVEY.md §8(a) a20 and §8(f) rank 2.

Reference: ``arnoldi_checkpoint`` (core/eigensolvers.f90:758-857), called after every Arnoldi step
when ``ifres`` (krylov_decomposition.f90:84), writes

* the new Krylov vector Q(k+1) as a Nek5000 field file ``KRY<session>0.f<k+1>`` (``outpost2``,
  numbering via ``whereyouwant``, IO.f90:2-10); Q(1) is written when the run starts (:235-236);
* the spectrum of the current H: ``Spectre_H<evop><k>.dat`` (re, im, residual; 3E15.7) and the
  log-transformed ``Spectre_NS<evop><k>.dat`` (divided by the sampling period dt*nsteps);
* the Hessenberg matrix ``HES<session><k>`` (list-directed, row-major over (k+1) x k, :837).

Restart (``uparam(2) = mstart > 0``, eigensolvers.f90:240-285): rank 0 reads ``HES<session><mstart>``
(rows 1..mstart+1, cols 1..mstart), broadcasts it, ``mstart = mstart + 1`` and ``load_files`` reads
KRY 1..mstart (IO.f90:12-73) before the factorisation continues.  Here every rank writes its own
element range as a multi-file set (fid = rank); the HES text is written with 17 significant digits
(the reference's list-directed output is readable by the same reader and vice versa).
"""
from __future__ import annotations

import os

import numpy as np

from . import fld, lapack
from .arnoldi import HessenbergDev
from .vector import Basis, NekContext, NekVector


def log_transform(x: complex) -> complex:
    """log(x); real when aimag(x) == 0 (eigensolvers.f90:860-869)."""
    v = np.log(complex(x))
    return complex(v.real, 0.0) if x.imag == 0 else v


def write_hes(path: str, H: np.ndarray, k: int) -> None:
    d, b = os.path.split(path)
    tmp = os.path.join(d, f".{b}.part{os.getpid()}")   # renamed into place: never read half written
    with open(tmp, "w") as fh:
        for i in range(k + 1):
            for j in range(k):
                fh.write(f"{H[i, j]: .17E}\n")
    os.replace(tmp, path)


def _list_directed_reals(text: str, count: int, path: str) -> np.ndarray:
    """The first ``count`` items of a Fortran list-directed real read: blank / comma / newline
    separators, ``r*c`` repeat counts, D exponents."""
    vals = []
    for tok in text.replace(",", " ").split():
        if "*" in tok:
            r, c = tok.split("*", 1)
            vals.extend([float(c.replace("D", "E").replace("d", "e"))] * int(r))
        else:
            vals.append(float(tok.replace("D", "E").replace("d", "e")))
        if len(vals) >= count:
            break
    if len(vals) < count:
        raise ValueError(f"{path}: {len(vals)} values, {count} expected")
    return np.array(vals[:count], dtype=np.float64)


def read_hes(path: str, mstart: int, k_dim: int) -> np.ndarray:
    """H (k_dim+1, k_dim) with rows 1..mstart+1, cols 1..mstart filled, read row-major as the
    reference's list-directed ``read (67, *) ((H(i, j), j=1, mstart), i=1, mstart+1)``
    (eigensolvers.f90:262).  ``mstart > k_dim`` is refused: the reference's "subsampling" branch
    (:250-256) reads one (1E15.7) field per record, which takes the first value of each line of the
    several-values-per-record file ``arnoldi_checkpoint`` writes (:837) — not a restatable restart."""
    if mstart > k_dim:
        raise ValueError(f"restart from HES at mstart={mstart} > k_dim={k_dim} is not supported "
                         f"(the reference's subsampling read, eigensolvers.f90:250-256)")
    if mstart < 1:
        raise ValueError(f"mstart={mstart} < 1")
    need = (mstart + 1) * mstart
    with open(path) as fh:
        A = _list_directed_reals(fh.read(), need, path).reshape(mstart + 1, mstart)
    H = np.zeros((k_dim + 1, k_dim), order="F")
    H[: mstart + 1, :mstart] = A
    return H


def write_spectra(directory: str, evop: str, k: int, vals, residual, period: float) -> None:
    with open(os.path.join(directory, f"Spectre_H{evop}{k:04d}.dat"), "w") as fh:
        for v, r in zip(vals, residual):
            fh.write(f"{v.real:15.7E}{v.imag:15.7E}{r:15.7E}\n")
    with open(os.path.join(directory, f"Spectre_NS{evop}{k:04d}.dat"), "w") as fh:
        for v, r in zip(vals, residual):
            lt = log_transform(v)
            fh.write(f"{lt.real / period:15.7E}{lt.imag / period:15.7E}{r:15.7E}\n")


class ArnoldiCheckpoint:
    """Per-step hook: ``krylov_schur(..., on_step=ArnoldiCheckpoint(ctx, dir, session))``."""

    def __init__(self, ctx: NekContext, directory: str, session: str = "nek", evop: str = "_",
                 period: float = 1.0, eigen_tol: float = 1e-6, write_spectra: bool = True):
        self.ctx, self.dir, self.session, self.evop = ctx, directory, session, evop
        self.period, self.eigen_tol, self.spectra = period, eigen_tol, write_spectra
        os.makedirs(directory, exist_ok=True)

    def write_vector(self, v: NekVector, num: int, time: float = 0.0) -> None:
        lay = self.ctx.layout
        f = fld.fld_from_vector(lay, v.to_packed(), time=time, istep=num)
        fld.write_fld(os.path.join(self.dir, fld.fld_name("KRY", self.session, lay.rank, num)), f)

    def __call__(self, mstep: int, Q: Basis, Hd: HessenbergDev) -> None:
        k = mstep
        # outpost2 is collective: on return every rank's KRY file and rank 0's HES are in place
        with fld.collective_output(self.ctx.comm):
            if k == 1:  # Q(1) is written when the factorisation starts (eigensolvers.f90:235-236)
                self.write_vector(Q[0], 1, time=0.0)
            self.write_vector(Q[k], k + 1, time=float(k))   # whereyouwant("KRY", k+1)
            if self.ctx.comm.rank == 0:
                H = Hd.download()
                if self.spectra:
                    vals, vecs = lapack.eig(H[:k, :k])
                    res = np.abs(H[k, k - 1] * vecs[k - 1, :])
                    write_spectra(self.dir, self.evop, k, vals, res, self.period)
                write_hes(os.path.join(self.dir, f"HES{self.session}{k:04d}"), H, k)


def read_restart_hes(comm, directory: str, session: str, mstart: int, k_dim: int) -> np.ndarray:
    """H for a restart at ``mstart``: rank 0 parses ``HES<session><mstart>`` and broadcasts the
    (k_dim+1) x k_dim matrix to every rank (eigensolvers.f90:244-266: ``if (nid == 0)`` read, then
    ``bcast(H, (k_dim+1)*k_dim*wdsize)``).  A failure on rank 0 is broadcast in its place, so every
    rank raises the same exception instead of waiting at the broadcast."""
    got = None
    if comm.rank == 0:
        try:
            got = read_hes(os.path.join(directory, f"HES{session}{mstart:04d}"), mstart, k_dim)
        except Exception as e:  # noqa: BLE001 - sent to every rank, raised on all of them
            got = e
    got = comm.bcast_object(got, src=0)
    if isinstance(got, BaseException):
        raise got
    return np.asfortranarray(got)


def restart_vectors(lay, directory: str, session: str, mstart: int, comm=None):
    """KRY 1..mstart+1 of this rank's shard, one padded host vector at a time (``load_files``,
    IO.f90:12-73, after ``mstart = mstart + 1``): each rank opens only the files holding its own
    elements (``fld.read_fld_set`` with the layout), so host memory stays one vector."""
    for i in range(1, mstart + 2):
        yield fld.vector_from_fld(lay, fld.read_fld_set(directory, "KRY", session, i, lay=lay, comm=comm))


def load_restart(ctx: NekContext, directory: str, session: str, mstart: int, k_dim: int):
    """(Q, H) for ``krylov_schur(..., Q=Q, start=(mstart, H))``: Q[0:mstart+1] = KRY 1..mstart+1,
    H read on rank 0 and broadcast."""
    H = read_restart_hes(ctx.comm, directory, session, mstart, k_dim)
    Q = ctx.basis(k_dim + 1)
    for i, v in enumerate(restart_vectors(ctx.layout, directory, session, mstart, ctx.comm)):
        Q[i].from_packed(v)
    return Q, H
