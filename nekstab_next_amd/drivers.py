"""nekStab's user-facing analysis drivers over the device path (the ★ caller layer,
core/linear_stab.f90:12-119, 295-383).

* :func:`linear_stability_analysis` — prepare_seed, eigs (Krylov–Schur), ``Spectrum_H<evop>.dat``,
  eigvals <- log(eigvals)/t, ``Spectrum_NS<evop>.dat``, Re/Im eigenvector export of the first
  ``maxmodes`` Ritz vectors (``<evop>Re``/``<evop>Im`` field files).
* :func:`transient_growth_analysis` — prepare_seed, svds, sigma <- sigma**2,
  ``Spectrum_Sp.dat`` and the optimal initial condition / response export (``pU``/``pV``).

The operator is any :class:`~nekstab_next_amd.operators.LinearOperator` (the exponential
propagator of a Nek5000 run in production; synthetic operators in the tests) with the sampling
time ``t`` (``exponential_prop%t``).
* :func:`resolvent_analysis` — svds of a resolvent operator on complex (re/im pair) vectors,
  sigma <- sigma**2, ``Spectrum_Sr.dat``.  The resolvent's body (forced Nek5000 run + inner GMRES
  on Id - A^T) is the caller's operator.
"""
from __future__ import annotations

import os

import numpy as np

from . import fld
from .config import KrylovSchurConfig
from .krylov_schur import prepare_seed
from .lightkrylov import eigs, get_vec, svds
from .operators import LinearOperator
from .vector import NekContext, NekVector


def _write_spectrum(path: str, vals, res) -> None:
    with open(path, "w") as fh:
        for v, r in zip(vals, res):
            fh.write(f"{v.real:15.7E}{v.imag:15.7E}{r:15.7E}\n")


def _export(ctx: NekContext, vec: NekVector, outdir: str, prefix: str, session: str, num: int, time: float):
    lay = ctx.layout
    f = fld.fld_from_vector(lay, vec.to_packed(), time=time, istep=num)
    fld.write_fld(os.path.join(outdir, fld.fld_name(prefix, session, lay.rank, num)), f)


def linear_stability_analysis(ctx: NekContext, A: LinearOperator, seed: NekVector, t: float,
                              cfg: KrylovSchurConfig | None = None, transpose: bool = False,
                              outdir: str | None = None, session: str = "nek", evop: str | None = None) -> dict:
    cfg = cfg or KrylovSchurConfig()
    evop = evop or ("a" if transpose else "d")
    X = ctx.basis(cfg.k_dim + 1)
    prepare_seed(seed, X[0])
    vecs, vals, res, info = eigs(ctx, A, X, nev=cfg.schur_tgt, tolerance=cfg.eigen_tol, transpose=transpose,
                                 schur_del=cfg.schur_del, mode=cfg.mode)
    vals_ns = np.log(vals.astype(np.complex128)) / t
    if outdir:
        v = ctx.vector()
        # outpost2 is collective: the sets are whole on return; rank 0's spectra are written inside
        # the block too, so a failure there is raised on every rank (collective_output's agreement)
        with fld.collective_output(ctx.comm):
            os.makedirs(outdir, exist_ok=True)
            if ctx.comm.rank == 0:
                _write_spectrum(os.path.join(outdir, f"Spectrum_H{evop}.dat"), vals, res)
                _write_spectrum(os.path.join(outdir, f"Spectrum_NS{evop}.dat"), vals_ns, res)
            for i in range(min(cfg.maxmodes, cfg.k_dim)):
                get_vec(v, X, vecs[:, i].real, cfg.k_dim)
                _export(ctx, v, outdir, f"{evop}Re", session, i + 1, float(i + 1))
                get_vec(v, X, vecs[:, i].imag, cfg.k_dim)
                _export(ctx, v, outdir, f"{evop}Im", session, i + 1, float(i + 1))
    return dict(eigvals=vals, eigvals_ns=vals_ns, residuals=res, eigvecs=vecs, info=info, X=X)


def transient_growth_analysis(ctx: NekContext, A: LinearOperator, seed: NekVector, k_dim: int = 100,
                              nev: int = 2, tolerance: float = 1e-6, outdir: str | None = None,
                              session: str = "nek", maxmodes: int = 20) -> dict:
    U, V = ctx.basis(k_dim + 1), ctx.basis(k_dim + 1)
    prepare_seed(seed, V[0])
    r = svds(ctx, A, U, V, nev=nev, tolerance=tolerance)
    gain = r.sigma ** 2   # energy gain, sigma = sigma**2 (linear_stab.f90:113)
    if outdir:
        v = ctx.vector()
        with fld.collective_output(ctx.comm):   # rank 0's spectrum and every rank's modes, agreed
            os.makedirs(outdir, exist_ok=True)
            if ctx.comm.rank == 0:
                with open(os.path.join(outdir, "Spectrum_Sp.dat"), "w") as fh:
                    for s, res in zip(gain, r.residuals):
                        fh.write(f"{s:15.7E}{res:15.7E}\n")
            for i in range(min(maxmodes, nev)):
                get_vec(v, U, r.uvecs[:, i], k_dim)
                _export(ctx, v, outdir, "pU", session, i + 1, float(i + 1))
                get_vec(v, V, r.vvecs[:, i], k_dim)
                _export(ctx, v, outdir, "pV", session, i + 1, float(i + 1))
    return dict(gain=gain, sigma=r.sigma, residuals=r.residuals, info=r.info, U=U, V=V, svd=r)


def resolvent_analysis(ctx: NekContext, R: LinearOperator, seed: NekVector, k_dim: int = 100, nev: int = 2,
                       tolerance: float = 1e-6, outdir: str | None = None, evop: str = "r") -> dict:
    """``resolvent_analysis`` (core/linear_stab.f90:120-163): svds of the resolvent operator on
    complex vectors, sigma <- sigma**2, ``Spectrum_S<evop>.dat`` (sigma^2, residual; 2E15.7).

    ``ctx`` is a context on a :class:`~nekstab_next_amd.layout.PairLayout` (complex vectors as
    re/im pair vectors, so the cmplx dot re.re + im.im is the layout's weighted dot and svds runs
    unchanged); ``R`` maps complex to complex (``matvec``) with its adjoint (``rmatvec``).  In
    nekStab R's body is a forced Nek5000 integration plus an inner GMRES
    (linear_operators.f90:348-431) — any operator with that interface plugs in;
    :class:`~nekstab_next_amd.operators.ComplexDiagOperator` is the synthetic, exactly known one.
    The reference seeds re and im separately (prepare_seed on U%re, U%im, :147-148); here the
    seed pair is normalised as one vector (the bidiagonalisation only needs its direction).  The
    cmplx dot is real, so x and i x are independent directions and every singular value of the
    complex operator appears twice in ``sigma2`` — as with LightKrylov's svds on
    cmplx_nek_vector."""
    from .layout import PairLayout

    if not isinstance(ctx.layout, PairLayout):
        raise ValueError("resolvent_analysis needs a NekContext on a PairLayout (complex vectors)")
    U, V = ctx.basis(k_dim + 1), ctx.basis(k_dim + 1)
    prepare_seed(seed, V[0])
    r = svds(ctx, R, U, V, nev=nev, tolerance=tolerance)
    gain = r.sigma ** 2   # sigma = sigma**2 (:157)
    if outdir:
        with fld.collective_output(ctx.comm):   # a failure on rank 0 is raised on every rank
            if ctx.comm.rank == 0:
                os.makedirs(outdir, exist_ok=True)
                with open(os.path.join(outdir, f"Spectrum_S{evop}.dat"), "w") as fh:
                    for s, res in zip(gain, r.residuals):
                        fh.write(f"{s:15.7E}{res:15.7E}\n")
    return dict(sigma2=gain, residuals=r.residuals, info=r.info, U=U, V=V, svd=r)
