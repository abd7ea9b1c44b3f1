#!/usr/bin/env python
"""Time Krylov–Schur from the reference's default (unnormalised) noise seed with the two
non-orthonormal Gram–Schmidt forms, "mgs2-lagged" (two reads of Q per step, one host
synchronisation per step) and "mgs2-icwy" (three reads, no synchronisation), on the cylinder layout
(config 2's mesh and its 2e6 scaling) and config 3's layout; rotation-scaling / clustered operators.
Prints one JSON object per measurement (median of 3 after a warm-up).

  python tools/bench_nonorth.py        # on the MI355X box
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.layout import box3d_layout, cylinder_layout
    from nekstab_next_amd.operators import DiagOperator
    from nekstab_next_amd.vector import NekContext

    cases = [("cylinder", cylinder_layout(1996), 64), ("cylinder", cylinder_layout(22728), 64),
             ("box3d", box3d_layout(2000), 128), ("box3d", box3d_layout(11044), 128)]
    for name, lay, k in cases:
        ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=k + 1)
        d, _ = syn.clustered_spectrum(lay)
        op = DiagOperator(ctx, d)
        seed = ctx.vector()
        seed.fill_hash(11)
        Q = ctx.basis(k + 1)
        for nonorth in ("mgs2-lagged", "mgs2-icwy"):
            cfg = KrylovSchurConfig(k_dim=k, schur_tgt=4, seed_mode="noise", nonorth_mode=nonorth)
            krylov_schur(ctx, op, seed, cfg, Q=Q)
            ts = []
            for _ in range(3):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                r = krylov_schur(ctx, op, seed, cfg, Q=Q)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            print(json.dumps(dict(layout=name, E=lay.nelgv, N=lay.N, k_dim=k, nonorth=nonorth,
                                  seconds=round(float(np.median(ts)), 4), restarts=r.schur_cnt,
                                  mstart=r.mstart_history, converged=int(r.converged))), flush=True)
        del Q, ctx


if __name__ == "__main__":
    main()
