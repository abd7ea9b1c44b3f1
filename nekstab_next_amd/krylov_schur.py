"""Krylov–Schur eigensolver driver (host control flow, device basis).

Reference: ``krylov_schur`` (core/eigensolvers.f90:120-359) and ``schur_condensation`` (:363-468).
Control flow restated one-for-one:

    repeat
        arnoldi_factorization(Q, H, mstart, k_dim)                          :298
        vals, vecs = eig(H(1:k,1:k))          (dgeev, sorted by |lambda|)      :306
        residual = |H(k+1,k) * vecs(k,:)|;  cnt = #(residual < eigen_tol)      :309-310
        stop if schur_tgt <= 0 or cnt >= schur_tgt, else schur_condensation    :314-331
    until converged

``schur_condensation``: b = H(k+1,k) e_k; (T, Z) = dgees(H_k) sorted |lambda|>0.9; select
(|lambda| >= 1-schur_del) U (nev+4 largest); dtrsen; zero the unwanted blocks; Q(:,1:k) <- Q(:,1:k) Z
(device, in place, only the ms kept columns — the reference copies the whole basis twice and
rotates all k, :421-442); H(ms+1,:) = b^T Z;
mstart = ms+1; Q(mstart) <- Q(k+1).

The dense k x k work runs on the host (lapack.py), identically on every rank.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import lapack
from ._lib import NkvNaNError
from .arnoldi import FactorizationGraph, HessenbergDev, arnoldi_factorization
from .config import KrylovSchurConfig
from .operators import LinearOperator
from .vector import Basis, NekContext, NekVector


@dataclass
class KrylovSchurResult:
    vals: np.ndarray            # Ritz values of H_k, sorted by decreasing modulus (complex)
    vecs: np.ndarray            # corresponding eigenvectors of H_k (k x k complex)
    residual: np.ndarray        # |H(k+1,k) vecs(k,:)| (Ritz residual estimates)
    converged: int              # count(residual < eigen_tol)
    schur_cnt: int              # number of Schur condensations (restarts)
    H: np.ndarray               # final (k+1) x k Hessenberg/Krylov–Schur matrix
    Q: Basis                    # the resident basis (k+1 vectors)
    mstart_history: list = field(default_factory=list)   # mstart after each condensation
    cnt_history: list = field(default_factory=list)      # converged count after each factorisation
    selected_history: list = field(default_factory=list)  # selected masks per condensation
    breakdowns: list = field(default_factory=list)        # mstart of each factorisation redone in MGS2


_MGS2 = ("mgs2", "mgs2-native")


def _mgs2_of(mode: str) -> str:
    """The reference-order mode a solve falls back to: the library-driven one for a native mode."""
    return "mgs2-native" if mode.endswith("-native") else "mgs2"


def _nonorth_of(mode: str, cfg: KrylovSchurConfig, time_in_dot: bool = False) -> str:
    """The mode for a basis that is not orthonormal (``cfg.nonorth_mode``; "mgs2" keeps a native
    mode's library-driven variant).  An explicit reference-order request (``cfg.mode`` "mgs2" /
    "mgs2-native") is kept as it is: its rounding is the reference's, which ICWY only equals in
    exact arithmetic.  "mgs2-lagged" derives A q from the Arnoldi relation of the finished columns,
    which the reference's restart breaks in the `time` slot (it rotates the fields only, defect 6):
    with time in k_dot ICWY is used instead."""
    if mode in _MGS2:
        return mode
    if cfg.nonorth_mode == "mgs2":
        return _mgs2_of(mode)
    if cfg.nonorth_mode == "mgs2-lagged" and not time_in_dot:
        return "mgs2-lagged-native" if mode.endswith("-native") else "mgs2-lagged"
    if cfg.nonorth_mode not in ("mgs2-icwy", "mgs2-lagged"):
        raise ValueError(f"nonorth_mode={cfg.nonorth_mode!r}: 'mgs2-lagged', 'mgs2-icwy' or 'mgs2'")
    return "mgs2-icwy-native" if mode.endswith("-native") else "mgs2-icwy"


def breakdown_column(H: np.ndarray, c0: int, k: int, tol: float, offset: int = 1) -> int:
    """First Arnoldi column c in [c0, k) whose new direction vanished (|H(c+1,c)| < tol ||H(0:c+2,c)||,
    the Krylov space is invariant to rounding), or that holds a non-finite entry; -1 if none.
    ``offset``: row of a column's new-direction norm relative to c (1 for Hessenberg H; 0 for the
    upper-triangular projection C of Golub–Kahan–Lanczos, whose column c ends at alpha = C(c,c)).

    At such a step the reference's MGS2 (eigensolvers.f90:101-112) still produces a unit vector from the
    rounding noise, orthogonalised twice one projection at a time.  The one-pass classical forms cannot:
    CGS2 leaves O(eps/ratio) components in span(Q) (garbage at ratio ~ eps), and DCGS2's Pythagorean
    norm sqrt(||u||^2 - ||Q^T u||^2) cancels to a negative (NaN).  Normal runs sit at ratios >= 0.1."""
    for c in range(max(c0, 0), k):
        col = H[:c + 1 + offset, c]
        if not np.all(np.isfinite(col)):
            return c
        nrm = float(np.linalg.norm(col))
        if nrm == 0.0 or abs(col[c + offset]) < tol * nrm:
            return c
    return -1


def prepare_seed(seed: NekVector, Q0: NekVector) -> float:
    """X(1) = seed / sqrt(<seed, seed>) with real_dot (incl. time) — core/linear_stab.f90:287-291."""
    Q0.copy_from(seed)
    alpha = float(np.sqrt(Q0.dot(Q0)))
    Q0.scal(1.0 / alpha)
    return alpha


def schur_condensation(ctx: NekContext, H: np.ndarray, Q: Basis, k: int, cfg: KrylovSchurConfig):
    """One Krylov–Schur restart.  Mutates H (host) and Q (device); returns (mstart, selected)."""
    b_vec = np.zeros(k)
    b_vec[k - 1] = H[k, k - 1]
    T, Z, vals = lapack.schur(H[:k, :k])
    selected, ms = lapack.select_eigenvalues(vals, cfg.schur_del, cfg.schur_tgt, faithful=cfg.faithful_select)
    T, Z, _m = lapack.ordschur(T, Z, selected)
    H[:k, :k] = T
    H[:ms, ms:k] = 0.0
    H[ms:k + 1, :] = 0.0
    if ms > 0:
        # Only Q(1:ms) survive the restart: Q(ms+1) <- Q(k+1) below and Q(ms+2..k) are rewritten by
        # the next factorisation before any read, so the device rotation writes ms columns
        # (reads k): 8N(k+ms) bytes instead of the reference's full Q(:,1:k) Z.
        Zd = torch.as_tensor(np.asfortranarray(Z[:, :ms]).ravel(order="F")).to(ctx.device)
        if ctx.timer:
            ctx.timer.begin("rotate")
        ctx.call("nkv_rotate_cols", Q.ptr, int(k), Zd.data_ptr(), int(k), int(ms), ctx.stream)
        if ctx.timer:
            ctx.timer.end("rotate", 8.0 * ctx.layout.N * (k + ms))
    H[ms, :] = b_vec @ Z
    mstart = ms + 1
    # Q(mstart) <- Q(k+1): nopcopy moves the fields only, not time (:458-459)
    Q[mstart - 1].copy_from(Q[k], time=False)
    return mstart, selected


def load_seed(ctx: NekContext, directory: str, session: str = "nek", transpose: bool = False) -> NekVector:
    """The ``ifseed_load`` seed (eigensolvers.f90:210-223): the real part of mode 1 of an earlier
    run, ``dRe<session>0.f00001`` for the direct problem (uparam(1) in [3.0, 3.2)) or
    ``aRe<session>0.f00001`` for the adjoint ([3.2, 3.3)), read as ``load_fld`` + ``nopcopy`` do
    (velocity, pressure, scalars; time 0).  Each rank reads its own elements of a multi-file set.
    Pass it to :func:`krylov_schur` with ``seed_mode="load"``: k_normalize, one matvec,
    Q(1) = A seed, not renormalised (:222-223)."""
    from . import fld

    prefix = "aRe" if transpose else "dRe"
    files = fld.read_fld_set(directory, prefix, session, 1, lay=ctx.layout, comm=ctx.comm)
    return ctx.vector().from_packed(fld.vector_from_fld(ctx.layout, files))


def krylov_schur(ctx: NekContext, op: LinearOperator, seed: NekVector, cfg: KrylovSchurConfig | None = None,
                 transpose: bool = False, on_restart=None, Q: Basis | None = None, on_step=None,
                 start=None) -> KrylovSchurResult:
    """Eigenpairs of ``op`` of largest modulus by Krylov–Schur restarts (reference defaults from
    core/main.f90:9-12: k_dim=100, schur_tgt=2, eigen_tol=1e-6, schur_del=0.1).

    ``Q``: caller-owned basis of k_dim+1 vectors (LightKrylov's ``X``), else allocated.
    ``on_step(mstep, Q, Hd)``: per-Arnoldi-step hook (checkpointing, ifres).
    ``start=(mstart, H)``: resume from a checkpoint (Q[0:mstart] already loaded, uparam(2) > 0,
    eigensolvers.f90:240-285); ``seed`` is then ignored."""
    cfg = cfg or KrylovSchurConfig()
    k = cfg.k_dim
    if Q is None:
        Q = ctx.basis(k + 1)
    elif Q.k < k + 1:
        raise ValueError(f"basis has {Q.k} vectors, k_dim+1={k + 1} needed")
    Hd = HessenbergDev(ctx, k)
    H = np.zeros((k + 1, k), order="F")
    f = ctx.vector()
    if start is not None:
        pass
    elif cfg.seed_mode == "normalize":
        prepare_seed(seed, Q[0])
    elif cfg.seed_mode in ("noise", "load"):
        # ifseed_nois / ifseed_load branches of the in-tree driver: Q(1) = A (seed/||seed||), NOT
        # renormalised (eigensolvers.f90:195-203, 210-223; "load" seeds come from load_seed)
        w2 = ctx.vector()
        w2.copy_from(seed)
        from .vector import k_normalize
        k_normalize(w2)
        (op.rmatvec if transpose else op.matvec)(w2, Q[0])
    elif cfg.seed_mode in ("as_is", "symm"):
        # "symm": ifseed_symm (eigensolvers.f90:205-208): Q(1) = the symmetric seed as it stands
        # (seeds.symmetric_seed), neither normalised nor mapped
        Q[0].copy_from(seed)
    else:
        raise ValueError(cfg.seed_mode)

    mstart = 1
    if start is not None:
        mstart, H0 = start
        H[...] = H0
        Hd.upload(H)
        mstart = int(mstart) + 1  # "careful here!" (eigensolvers.f90:281)
    schur_cnt = 0
    res = KrylovSchurResult(None, None, None, 0, 0, H, Q)
    hook = None if on_step is None else (lambda mstep: on_step(mstep, Q, Hd))
    if cfg.graphs and ctx.comm.world > 1:
        raise ValueError("KrylovSchurConfig.graphs=True is refused at world size > 1: HIP-graph capture of "
                         "the RCCL all-reduces has not been validated on more than one GPU; run eagerly")
    graphs = FactorizationGraph(ctx, op, Q, Hd, f, cfg.mode) if (cfg.graphs and hook is None) else None
    if graphs is not None and not graphs.usable():
        graphs = None
    # the "noise" seed leaves Q(1) unnormalised (eigensolvers.f90:195-203); the reference's MGS2
    # then projects against it as it stands, so its basis is not orthonormal (a projection onto an
    # unnormalised vector removes only part of the component) and classical and modified
    # Gram–Schmidt no longer agree.  That mode therefore runs modified Gram–Schmidt: by default in
    # inverse compact WY form (the same coefficients, three reads of Q per step), or in the
    # reference's own operation order (cfg.nonorth_mode = "mgs2").  A resumed run (``start``) keeps
    # it too: its checkpointed basis descends from the same Q(1) (pass the original seed_mode).
    mode = _nonorth_of(cfg.mode, cfg, ctx.time_in_dot) if cfg.seed_mode in ("noise", "load", "symm") else cfg.mode
    if mode != cfg.mode:
        graphs = None
    snap = None   # Q(mstart) before a classical factorisation (DCGS2's restart-row correction rewrites it)
    while True:
        if mode not in _MGS2:
            H_before = H.copy()
            snap = snap if snap is not None else ctx.vector()
            snap.storage.copy_(Q.storage[mstart - 1])
        broken = False
        try:
            if graphs is not None:
                graphs.run(mstart, k, transpose)
            else:
                arnoldi_factorization(ctx, op, Q, Hd, mstart, k, f=f, mode=mode, transpose=transpose,
                                      on_step=hook)
            H[...] = Hd.download()  # columns mstart..k written on the device, the rest as uploaded
            ctx.check_nan()
        except NkvNaNError:
            if mode in _MGS2:
                raise
            broken = True
        if mode not in _MGS2:
            broken = broken or breakdown_column(H, mstart - 1, k, cfg.breakdown_tol) >= 0
            if ctx.comm.world > 1:   # the H test is replicated; the NaN flag is per rank
                flag = torch.tensor([1.0 if broken else 0.0], dtype=torch.float64, device=ctx.device)
                broken = float(ctx.comm.allreduce_(flag).item()) > 0.0
            if broken:
                # invariant subspace reached: redo this factorisation from its starting state in the
                # reference's MGS2 order, and keep that order for the rest of the solve
                res.breakdowns.append(mstart)
                Q.storage[mstart - 1].copy_(snap.storage)
                H[...] = H_before
                Hd.upload(H)
                mode, graphs = _mgs2_of(mode), None
                arnoldi_factorization(ctx, op, Q, Hd, mstart, k, f=f, mode=mode, transpose=transpose,
                                      on_step=hook)
                H[...] = Hd.download()
                ctx.check_nan()
        vals, vecs = lapack.eig(H[:k, :k])
        residual = np.abs(H[k, k - 1] * vecs[k - 1, :])
        cnt = int(np.count_nonzero(residual < cfg.eigen_tol))
        res.cnt_history.append(cnt)
        if cfg.schur_tgt <= 0 or cnt >= cfg.schur_tgt or schur_cnt >= cfg.max_restarts:
            break
        schur_cnt += 1
        mstart, selected = schur_condensation(ctx, H, Q, k, cfg)
        if ctx.time_in_dot and mode not in _MGS2:
            # the restart moves the fields but not `time` (eigensolvers.f90:421-432, 458-459), so
            # with time in k_dot (uparam(1)==2.1) the kept basis is no longer orthonormal: from here
            # on modified Gram–Schmidt is mirrored (CGS2/DCGS2 assume an orthonormal basis)
            mode, graphs = _nonorth_of(mode, cfg, True), None
        res.mstart_history.append(mstart)
        res.selected_history.append(selected)
        Hd.upload(H)
        if on_restart is not None:
            on_restart(schur_cnt, mstart)
    res.vals, res.vecs, res.residual, res.converged, res.schur_cnt = vals, vecs, residual, cnt, schur_cnt
    res.H = H
    return res


def ritz_vector(ctx: NekContext, Q: Basis, vecs: np.ndarray, i: int, out_re: NekVector, out_im: NekVector,
                k: int | None = None, normalize: bool = True) -> tuple[float, float]:
    """Eigenmode i from the basis: fp = Q(:,1:k) vecs(:,i) (complex, as two real combinations),
    normalised so that ||Re||^2 + ||Im||^2 = 1 (outpost_ks, eigensolvers.f90:565-585, 603-613;
    ``normalize=False`` leaves fp as assembled, the vector ``norm_grad`` sees, :587-588).
    Returns (||Re||, ||Im||) before normalisation."""
    from .vector import combine

    k = vecs.shape[0] if k is None else k
    yr = torch.as_tensor(np.ascontiguousarray(vecs[:k, i].real)).to(ctx.device)
    yi = torch.as_tensor(np.ascontiguousarray(vecs[:k, i].imag)).to(ctx.device)
    combine(out_re, Q, yr, k, with_time=False)
    combine(out_im, Q, yi, k, with_time=False)
    a_r = float(np.sqrt(ctx.dot(out_re, out_re, time=False)))
    a_i = float(np.sqrt(ctx.dot(out_im, out_im, time=False)))
    if normalize:
        beta = 1.0 / np.sqrt(a_r ** 2 + a_i ** 2)
        out_re.scal(beta)
        out_im.scal(beta)
    return a_r, a_i


def orthonormality_report(ctx: NekContext, Q: Basis, k: int) -> np.ndarray:
    """Gram matrix G[i, j] = <q_i, q_j>_W (k_dot, no time term) of Q[0:k] — the self-check the
    reference writes to ``orthonormality.dat`` after the solve (eigensolvers.f90:335-345).  One
    multi-dot per column over the columns after it (upper triangle, k(k+1)/2 dots in k launches)."""
    G = np.zeros((k, k))
    h = ctx.h1
    for i in range(k):
        n = k - i
        ctx.call("nkv_block_dot", ctx.w.data_ptr(), Q.col_ptr(i), n, Q.col_ptr(i), h[:n].data_ptr(), ctx.ws.data_ptr(),
                 0, ctx.stream)
        ctx.comm.allreduce_(h[:n])
        row = h[:n].cpu().numpy()
        G[i, i:] = row
        G[i:, i] = row
    ctx.check_nan()
    return G


def outpost_ks(ctx: NekContext, res: KrylovSchurResult, outdir: str, evop: str = "d", period: float = 1.0,
               maxmodes: int = 20, session: str = "nek", k: int | None = None,
               orthonormality: bool = True, coords: dict | None = None, grad_tol: float = 1.1) -> dict:
    """The end of the in-tree ``krylov_schur`` (eigensolvers.f90:335-349) and ``outpost_ks``
    (:472-640): ``orthonormality.dat``; ``Spectre_H<evop>.dat`` (re, im, residual of every Ritz
    value, 3E15.7) and ``Spectre_NS<evop>.dat`` (log-transformed, divided by the sampling period
    dt*nsteps); for the first ``converged`` modes, up to ``maxmodes``: the eigenmode
    Q(:,1:k) vecs(:,i), normalised so ||Re||^2 + ||Im||^2 = 1, written as ``<evop>Re`` /
    ``<evop>Im`` field files numbered 1.. (time = output number), and its log-transformed value
    appended to ``Spectre_NS<evop>_conv.dat`` (2E15.7).

    Spurious-mode filter (:587-595): with ``coords`` (this rank's GLL coordinates {"x","y"[,"z"]},
    e.g. ``seeds.coords_from_fld``) the squared gradient norms of Re and Im of the assembled,
    not yet normalised mode are taken (``norm_grad``, utils.f90:446-486, on the device:
    :class:`~.sensitivity.NormGrad`), and a mode with either above ``grad_tol`` (1.1) is skipped:
    not written, not in ``_conv.dat``, and the following modes take its output number (the
    reference's ``outp`` counter).  Without coords no mode is filtered (the mesh is the case's).
    Returns the written mode indices, the skipped ones and every (Re, Im) gradient norm."""
    from . import fld
    from .checkpoint import log_transform

    k = res.vecs.shape[0] if k is None else k
    lay = ctx.layout
    G = orthonormality_report(ctx, res.Q, k) if orthonormality else None   # collective: before any write
    ng = None
    if coords is not None:
        from .sensitivity import NormGrad

        ng = NormGrad(ctx, coords)

    def text(name, lines):
        with open(os.path.join(outdir, name), "w") as fh:
            fh.writelines(lines)

    written, skipped, grad_norms = [], [], {}
    re_v, im_v = ctx.vector(), ctx.vector()
    conv_lines = []
    # outpost2 is collective: the set is whole on return.  The body's mode assembly and gradient
    # norms are collectives too, so every file write goes through the guard: a rank whose write
    # fails skips its later writes but keeps the ranks in lock-step, and the error is raised on
    # every rank at the end of the block
    with fld.collective_output(ctx.comm) as write:
        write(os.makedirs, outdir, exist_ok=True)
        if ctx.comm.rank == 0:
            if G is not None:
                lines = []
                for i in range(k):
                    lines.append(f"Norm of the {i + 1:4d}th mode = {np.sqrt(G[i, i]):20.14f}\n")
                    lines += [f"Orthogonality between mode {i + 1:4d} and mode {j + 1:4d} = {G[i, j]:15.7E}\n"
                              for j in range(i + 1, k)]
                    lines.append("\n")
                write(text, "orthonormality.dat", lines)
            h_lines, ns_lines = [], []
            for v, r in zip(res.vals[:k], res.residual[:k]):
                h_lines.append(f"{v.real:15.7E}{v.imag:15.7E}{r:15.7E}\n")
                lt = log_transform(v)
                ns_lines.append(f"{lt.real / period:15.7E}{lt.imag / period:15.7E}{r:15.7E}\n")
            write(text, f"Spectre_H{evop}.dat", h_lines)
            write(text, f"Spectre_NS{evop}.dat", ns_lines)
        for i in range(res.converged):
            if len(written) >= maxmodes:
                break
            a_r, a_i = ritz_vector(ctx, res.Q, res.vecs, i, re_v, im_v, k=k, normalize=ng is None)
            if ng is not None:
                g_re, g_im = ng(re_v), ng(im_v)   # on fp before nopcmult (:587-588)
                grad_norms[i] = (g_re, g_im)
                if g_re > grad_tol or g_im > grad_tol:
                    skipped.append(i)   # "Skipping spurious (non-physical) eigenvector" (:592-595)
                    continue
                beta = 1.0 / np.sqrt(a_r ** 2 + a_i ** 2)
                re_v.scal(beta)
                im_v.scal(beta)
            num = len(written) + 1
            for vec, name in ((re_v, f"{evop}Re"), (im_v, f"{evop}Im")):
                f = fld.fld_from_vector(lay, vec.to_packed(), time=float(num), istep=num)
                write(fld.write_fld, os.path.join(outdir, fld.fld_name(name, session, lay.rank, num)), f)
            lt = log_transform(res.vals[i])
            conv_lines.append(f"{lt.real / period:15.7E}{lt.imag / period:15.7E}\n")
            written.append(i)
        if ctx.comm.rank == 0:
            write(text, f"Spectre_NS{evop}_conv.dat", conv_lines)
    return dict(modes=written, skipped=skipped, grad_norms=grad_norms)
