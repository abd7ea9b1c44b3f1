#!/usr/bin/env python
"""Config 2 (N=2,000,064, k_dim=64) Krylov–Schur, eager launches, run 3x: the last run is the one
to read in a kernel trace (GPU busy time vs wall time = host/launch overhead per Arnoldi step)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.layout import cylinder_layout
    from nekstab_next_amd.operators import Rot2Operator
    from nekstab_next_amd.vector import NekContext

    lay = cylinder_layout(22728)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=80)
    c, s, dr, _ = syn.rot2_operator(lay)
    op = Rot2Operator(ctx, c, s, dr)
    seed = ctx.vector()
    seed.fill_hash(5)
    mode = sys.argv[1] if len(sys.argv) > 1 else "dcgs2"
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=64, schur_tgt=2, mode=mode))
        torch.cuda.synchronize()
        print(f"{mode} wall {1e3 * (time.perf_counter() - t0):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
