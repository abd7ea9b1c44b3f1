#!/usr/bin/env python
"""Probe: Krylov–Schur on a rank-deficient operator (an invariant subspace of dimension r < k_dim is
reached: the Krylov vector after step r is rounding noise).  Reports, per orthogonalisation mode,
whether the solve completes and its leading Ritz values, beside the oracle (the reference's MGS2)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import oracle as orc
    from helpers import olayout, oracle_diag_matvec
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.layout import NekLayout
    from nekstab_next_amd.operators import DiagOperator
    from nekstab_next_amd.vector import NekContext

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    w = syn.mass_weights(lay)
    L = olayout(lay)
    rank = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    d = np.zeros(lay.ld)
    idx = [f * lay.sv + 7 * (i + 1) for f in range(lay.n_wf) for i in range(rank)][:rank]
    for i, g in enumerate(idx):
        d[g] = 0.95 - 0.1 * i
    ref = None
    try:
        q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
        ref = orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 16, 2)
        print("oracle:", "vals", np.round(ref["vals"][:rank + 1].real, 12), "mstart", ref["mstart"], flush=True)
    except Exception as e:  # noqa: BLE001
        print("oracle failed:", type(e).__name__, e, flush=True)
    for mode in ("dcgs2", "cgs2", "mgs2"):
        ctx = NekContext(lay, weights=w, max_cols=32)
        seed = ctx.vector()
        seed.fill_hash(11)
        try:
            r = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=16, schur_tgt=2, mode=mode))
            print(mode, "ok: vals", np.round(r.vals[:rank + 1].real, 12), "mstart", r.mstart_history, flush=True)
        except Exception as e:  # noqa: BLE001
            print(mode, "failed:", type(e).__name__, str(e)[:200], flush=True)


if __name__ == "__main__":
    main()
