#!/usr/bin/env python
"""Time the non-headline BASELINE configs on one MI355X (parity configs; bench.py is config 3).

config 2: cylinder layout scaled to E=22,728 (N=2,000,064), rotation-scaling operator with
          conjugate pairs, Krylov–Schur k_dim=64, schur_tgt=2 — eager launches vs HIP-graph replay.
config 4: Newton–Krylov GMRES on J = D - I, cylinder mesh (N=175,648) and N=2,000,064, k_dim=200,
          tol 1e-9, DCGS2 (default) and CGS2 inner Arnoldi.
config 5: direct + adjoint Krylov–Schur, N=50,007,232, k_dim=96, two bases resident, + bi-orthogonalisation.
Prints one JSON object per measurement.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import GmresConfig, KrylovSchurConfig
    from nekstab_next_amd.gmres import ts_gmres
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.layout import cylinder_layout
    from nekstab_next_amd.operators import DiagOperator, Rot2Operator, ShiftedOperator
    from nekstab_next_amd.vector import NekContext

    lay = cylinder_layout(22728)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=80)
    c, s, dr, exact = syn.rot2_operator(lay)
    op = Rot2Operator(ctx, c, s, dr)
    seed = ctx.vector()
    seed.fill_hash(5)
    for mode, graphs in (("cgs2", False), ("dcgs2", False), ("dcgs2", True), ("cgs2", False), ("dcgs2", False),
                         ("dcgs2", True)):
        cfg = KrylovSchurConfig(k_dim=64, schur_tgt=2, graphs=graphs, mode=mode)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = krylov_schur(ctx, op, seed, cfg)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = 64 + sum(64 - (m - 1) for m in r.mstart_history)
        conv = r.residual < 1e-6
        err = max(float(np.min(np.abs(exact - v))) for v in r.vals[conv])
        print(json.dumps(dict(config="config2", N=lay.N, k_dim=64, mode=mode, graphs=graphs, seconds=round(dt, 4),
                              arnoldi_steps=steps, ms_per_step=round(dt / steps * 1e3, 4),
                              restarts=r.schur_cnt, converged=int(conv.sum()), max_err_vs_exact=err)), flush=True)
    # the rows above time a whole solve; with graphs=True that includes the one-off capture (the
    # solve converges in its first factorisation, so the graph is never replayed).  Here the same
    # 64-step DCGS2 factorisation is timed eager and as a graph replay (captured beforehand)
    from nekstab_next_amd.arnoldi import FactorizationGraph, HessenbergDev, arnoldi_factorization
    from nekstab_next_amd.krylov_schur import prepare_seed

    Q2, Hd2, f2 = ctx.basis(65), HessenbergDev(ctx, 64), ctx.vector()
    fg = FactorizationGraph(ctx, op, Q2, Hd2, f2, "dcgs2")
    for how in ("eager", "graph", "eager", "graph"):
        prepare_seed(seed, Q2[0])
        if how == "graph" and (1, 64, False) not in fg.graphs:
            fg.run(1, 64)   # capture (+ first replay), untimed
            prepare_seed(seed, Q2[0])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(5):
            if how == "graph":
                fg.run(1, 64)
            else:
                arnoldi_factorization(ctx, op, Q2, Hd2, 1, 64, f=f2, mode="dcgs2")
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(json.dumps(dict(config="config2_factorisation", N=lay.N, steps=64, mode="dcgs2", launch=how,
                              ms=round(dt * 1e3, 3), ms_per_step=round(dt / 64 * 1e3, 4))), flush=True)
    del Q2, Hd2, f2, fg

    # config 3's Krylov–Schur leg at BASELINE size (N=100,014,464, k_dim=128, schur_tgt=4): the
    # shift-invert spectrum and the config-1 diagonal spectrum scaled up converge in the first
    # 128-step factorisation; k_dim=24 on the diagonal spectrum forces Schur restarts (kept-column
    # rotations) at full size
    from nekstab_next_amd.layout import box3d_layout as _box

    lay3 = _box(44176)
    ctx3 = NekContext(lay3, weights=syn.mass_weights(lay3), max_cols=129)
    for name, kd in (("shift_invert", 128), ("diag", 128), ("diag", 24)):
        d3, ex3 = syn.laplacian_shift_invert(lay3) if name == "shift_invert" else syn.diag_spectrum(lay3)
        op3 = DiagOperator(ctx3, d3)
        del d3
        seed3 = ctx3.vector()
        seed3.fill_hash(11)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r3 = krylov_schur(ctx3, op3, seed3, KrylovSchurConfig(k_dim=kd, schur_tgt=4))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        conv = r3.residual < 1e-6
        err = max(float(np.min(np.abs(ex3 - v)) / abs(v)) for v in r3.vals[conv])
        steps = kd + sum(kd - (m - 1) for m in r3.mstart_history)
        print(json.dumps(dict(config="config3_krylov_schur", spectrum=name, N=lay3.N, k_dim=kd, schur_tgt=4,
                              mode=KrylovSchurConfig().mode, seconds=round(dt, 3), arnoldi_steps=steps,
                              restarts=r3.schur_cnt, mstart_history=r3.mstart_history,
                              converged=int(conv.sum()), max_rel_err_vs_exact=err)), flush=True)
        del op3, seed3, r3
    del ctx3

    for E4 in (1996, 22728):   # the real cylinder mesh and BASELINE's N=2,000,064
        lay4 = cylinder_layout(E4)
        ctx4 = NekContext(lay4, weights=syn.mass_weights(lay4), max_cols=210)
        d, _ = syn.diag_spectrum(lay4)
        op4 = ShiftedOperator(DiagOperator(ctx4, d), -1.0)
        rhs, sol = ctx4.vector(), ctx4.vector()
        rhs.fill_hash(3)
        for mode in ("dcgs2", "cgs2", "dcgs2", "cgs2"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            info = ts_gmres(ctx4, op4, rhs, sol, GmresConfig(k_dim=200, maxiter=10, tol=1e-9, mode=mode))
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            print(json.dumps(dict(config="config4", N=lay4.N, mode=mode, seconds=round(dt, 4), matvecs=info.matvecs,
                                  restarts=info.restarts, final_beta2=info.outer_residuals[-1])), flush=True)
    del ctx4, op4, rhs, sol

    # config 5 at BASELINE size on ONE GPU (two 97-vector bases = 78 GB resident): direct and
    # adjoint Krylov–Schur on D + rank-2 non-normal term (k_dim=96, schur_tgt=2), then the
    # bi-orthogonalisation of the leading pair
    from nekstab_next_amd.krylov_schur import ritz_vector
    from nekstab_next_amd.layout import box3d_layout
    from nekstab_next_amd.operators import RankTwoPerturbed
    from nekstab_next_amd.sensitivity import biorthogonalize

    lay5 = box3d_layout(22088)
    ctx5 = NekContext(lay5, weights=syn.mass_weights(lay5), max_cols=97)
    d5, _ = syn.diag_spectrum(lay5)
    vs = []
    for s5 in (21, 22, 23, 24):
        v = ctx5.vector()
        v.fill_hash(s5)
        v.scal(1e-3)
        vs.append(v)
    A5 = RankTwoPerturbed(DiagOperator(ctx5, d5), *vs, sigma=50.0)
    del d5
    seed5 = ctx5.vector()
    seed5.fill_hash(11)
    cfg5 = KrylovSchurConfig(k_dim=96, schur_tgt=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rd = krylov_schur(ctx5, A5, seed5, cfg5)
    ra = krylov_schur(ctx5, A5, seed5, cfg5, transpose=True)
    vecs = [ctx5.vector() for _ in range(4)]
    ritz_vector(ctx5, rd.Q, rd.vecs, 0, vecs[0], vecs[1], k=96)
    ritz_vector(ctx5, ra.Q, ra.vecs, 0, vecs[2], vecs[3], k=96)
    biorthogonalize(ctx5, *vecs)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    re = ctx5.dot(vecs[2], vecs[0], False) + ctx5.dot(vecs[3], vecs[1], False)
    im = ctx5.dot(vecs[2], vecs[1], False) - ctx5.dot(vecs[3], vecs[0], False)
    print(json.dumps(dict(config="config5", N=lay5.N, k_dim=96, mode=cfg5.mode, seconds=round(dt, 3),
                          restarts_direct=rd.schur_cnt, restarts_adjoint=ra.schur_cnt,
                          lambda_direct=str(rd.vals[0]), lambda_adjoint=str(ra.vals[0]),
                          biorth_re_minus_1=re - 1.0, biorth_im=im)), flush=True)


if __name__ == "__main__":
    main()
