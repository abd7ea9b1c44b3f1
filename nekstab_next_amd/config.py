"""Solver knobs with nekStab's defaults (core/main.f90:9-16, core/NEKSTAB:37-42)."""
from __future__ import annotations

from dataclasses import dataclass


@dataclass
class KrylovSchurConfig:
    k_dim: int = 100          # Krylov subspace dimension (k_dim, main.f90:9)
    schur_tgt: int = 2        # wanted converged eigenvalues; <= 0: plain k-step Arnoldi (:10, :314-317)
    eigen_tol: float = 1e-6   # Ritz residual tolerance (:11)
    schur_del: float = 0.1    # keep |lambda| >= 1 - schur_del at restarts (:12)
    maxmodes: int = 20        # max eigenmodes exported (:13)
    mode: str = "dcgs2"       # "dcgs2" (block CGS2, delayed re-orth.: 2 reads of Q per step, the MI355X
    #                           hot path) | "cgs2" (3 reads) | "mgs2" (reference order);
    #                           | "mgs2-icwy" (MGS in inverse compact WY form, 3 reads);
    #                           "dcgs2-native" | "cgs2-native" | "mgs2-native": the same sequences driven
    #                           by the library's one-call entry points (bit-identical)
    seed_mode: str = "normalize"   # "normalize" (linear_stab.f90:287-291) | "noise" (seeds.noise_seed) | "load"
    #                                (a krylov_schur.load_seed vector; both eigensolvers.f90:192-223) |
    #                                "symm" (seeds.symmetric_seed as Q(1), :205-208) | "as_is"
    faithful_select: bool = True   # reproduce quicksort2's ordering quirk
    max_restarts: int = 1000       # the reference loops until converged; this bounds it
    graphs: bool = False           # replay each factorisation as a captured HIP graph (capturable ops only)
    nonorth_mode: str = "mgs2-lagged"   # Gram–Schmidt where the basis is not orthonormal (noise/load seed,
    #                                time in k_dot after a restart), which must be modified G-S as the
    #                                reference's: "mgs2-lagged" (MGS2's coefficients with the second
    #                                pass lagged into the next multi-dot, 2 reads of Q per step; not with
    #                                time in k_dot, where ICWY is used), "mgs2-icwy" (inverse compact WY
    #                                form, 3 reads) or "mgs2" (the reference's own per-column order)
    breakdown_tol: float = 1e-8    # |H(c+1,c)| < tol * ||H(1:c+2,c)||: the Krylov space became invariant;
    #                                that factorisation is redone in the reference's MGS2 order


@dataclass
class GmresConfig:
    k_dim: int = 100          # inner Krylov dimension (ksize)
    maxiter: int = 100        # restarts (newton_krylov.f90:120: ts_gmres(f, dq, 100, k_dim, calls))
    tol: float = 1e-9         # max(param(21), param(22)) (newton_krylov.f90:236); test on beta**2
    mode: str = "dcgs2-native"  # inner Arnoldi: one continuous DCGS2 factorisation, the column loop in the
    #                             library (nkv_gmres_dcgs2; "dcgs2": the same cycle driven from Python, bit-
    #                             identical, 7 % slower at config 4); "cgs2" / "mgs2" (gmres.py)
    findiff: bool = False     # iffindiff relaxed exits (1e-8 inner, 1e-6 outer; :269, :292)
