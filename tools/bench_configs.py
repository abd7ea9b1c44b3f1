#!/usr/bin/env python
"""Time the non-headline BASELINE configs on one MI355X (parity configs; bench.py is config 3).

config 2: cylinder layout scaled to E=22,728 (N=2,000,064), rotation-scaling operator with
          conjugate pairs, Krylov–Schur k_dim=64, schur_tgt=2 — eager launches vs HIP-graph replay.
config 4: Newton–Krylov GMRES on J = D - I, cylinder mesh (N=175,648), k_dim=200, tol 1e-9.
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
    for graphs in (False, True, False, True):
        cfg = KrylovSchurConfig(k_dim=64, schur_tgt=2, graphs=graphs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = krylov_schur(ctx, op, seed, cfg)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = 64 + sum(64 - (m - 1) for m in r.mstart_history)
        conv = r.residual < 1e-6
        err = max(float(np.min(np.abs(exact - v))) for v in r.vals[conv])
        print(json.dumps(dict(config="config2", N=lay.N, k_dim=64, graphs=graphs, seconds=round(dt, 4),
                              arnoldi_steps=steps, ms_per_step=round(dt / steps * 1e3, 4),
                              restarts=r.schur_cnt, converged=int(conv.sum()), max_err_vs_exact=err)), flush=True)

    lay4 = cylinder_layout(1996)
    ctx4 = NekContext(lay4, weights=syn.mass_weights(lay4), max_cols=210)
    d, _ = syn.diag_spectrum(lay4)
    op4 = ShiftedOperator(DiagOperator(ctx4, d), -1.0)
    rhs, sol = ctx4.vector(), ctx4.vector()
    rhs.fill_hash(3)
    for _ in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        info = ts_gmres(ctx4, op4, rhs, sol, GmresConfig(k_dim=200, maxiter=10, tol=1e-9))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps(dict(config="config4", N=lay4.N, seconds=round(dt, 4), matvecs=info.matvecs,
                              restarts=info.restarts, final_beta2=info.outer_residuals[-1])), flush=True)


if __name__ == "__main__":
    main()
