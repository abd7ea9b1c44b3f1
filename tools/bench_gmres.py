#!/usr/bin/env python
"""One full restarted-GMRES cycle of 200 columns (ts_gmres, newton_krylov.f90:245-294, k_dim=200 as
examples/cylinder/1cyl.usr:14) at BASELINE config 4's N=2,000,064 on an operator that does not
converge early (diagonal, spectrum spread over [1e-4, 1]: ~1e-2 residual reduction in 200 steps),
with the host and GPU shares of the cycle:

* ``gpu_ms``: HIP events around every kernel family of a column (the matvec and the CGS2
  orthogonalisation kernels, bench.py's PhaseTimer), summed: the GPU's busy time;
* ``host_ms``: the cycle's wall time minus that (per-column H download and residual estimate,
  Python dispatch, the final dgels, the solution update); ``dcgs2-native`` is the same cycle through
  the one-call C driver ``nkv_gmres_dcgs2`` (its busy time is the ``dcgs2`` row's kernels, which it
  runs in the same order);
* ``dgels_every_column_ms``: what the round-2 form cost on the host — ``lstsq`` of the whole
  (k+1) x k system at every k = 1..200 (timed here on the cycle's own H) — against the O(k)
  Givens update now used (``givens_ms``).
Prints one JSON line.
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

    from nekstab_next_amd import lapack
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.config import GmresConfig
    from nekstab_next_amd.gmres import GivensResidual, ts_gmres
    from nekstab_next_amd.layout import cylinder_layout
    from nekstab_next_amd.operators import DiagOperator, LinearOperator
    from nekstab_next_amd.vector import NekContext

    lay = cylinder_layout(22728)
    ks = 200
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=ks + 1)
    d = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        d[f * lay.sv: f * lay.sv + lay.n_v] = 1e-4 + syn.hash_uniform(9, 400 + f, np.arange(lay.n_v, dtype=np.uint64))
    d[lay.n_wf * lay.sv: lay.n_wf * lay.sv + lay.n_p] = 0.5
    base = DiagOperator(ctx, d)

    class Timed(LinearOperator):      # events around the matvec (the GS kernels: ctx.timer)
        def matvec(self, x, y):
            tm = ctx.timer
            if tm:
                tm.begin("matvec")
            base.matvec(x, y)
            if tm:
                tm.end("matvec", 24.0 * lay.N)

    rhs = ctx.vector()
    rhs.fill_hash(3)
    sol = ctx.vector()
    from nekstab_next_amd.profiling import PhaseTimer

    rows = []
    for mode in ("dcgs2", "dcgs2-native", "cgs2"):
        cfg = GmresConfig(k_dim=ks, maxiter=1, tol=1e-300, mode=mode)
        ts_gmres(ctx, Timed(), rhs, sol, cfg)          # warm-up
        torch.cuda.synchronize()
        ctx.timer = PhaseTimer(ctx.device)
        t0 = time.perf_counter()
        info = ts_gmres(ctx, Timed(), rhs, sol, cfg)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) * 1e3
        ph = ctx.timer.summary()
        ctx.timer = None
        gpu_ms = sum(v["total_ms"] for v in ph.values())
        rows.append((mode, wall, gpu_ms, ph, info))
    # both residual forms on a Hessenberg matrix of the cycle's size (host only)
    H = np.asfortranarray(np.triu(np.random.default_rng(0).standard_normal((ks + 1, ks)), -1))
    e = np.zeros(ks + 1)
    e[0] = 1.0
    t0 = time.perf_counter()
    for k in range(1, ks + 1):
        y = lapack.lstsq(H[: k + 1, :k], e[: k + 1])
        np.linalg.norm(e[: k + 1] - H[: k + 1, :k] @ y)
    dgels_ms = (time.perf_counter() - t0) * 1e3
    t0 = time.perf_counter()
    g = GivensResidual(1.0, ks)
    for k in range(1, ks + 1):
        g.add_column(H[: k + 1, k - 1])
    lapack.lstsq(H, e)
    givens_ms = (time.perf_counter() - t0) * 1e3
    busy = {m: g for m, _w, g, _p, _i in rows}
    for mode, wall, gpu_ms, ph, info in rows:
        if mode == "dcgs2-native":
            # the one-call C driver runs the Gram-Schmidt kernels itself (no per-kernel events from
            # Python): the same kernels in the same order as "dcgs2", so its busy time is that row's
            gpu_ms = busy["dcgs2"] - sum(v["total_ms"] for k, v in rows[0][3].items() if k == "matvec") \
                + sum(v["total_ms"] for k, v in ph.items() if k == "matvec")
        print(json.dumps(dict(
            row="config4_gmres_cycle", mode=mode, N=lay.N, k_dim=ks, columns=len(info.inner_residuals),
            wall_ms=round(wall, 2), gpu_ms=round(gpu_ms, 2), host_ms=round(wall - gpu_ms, 2),
            gpu_share=round(gpu_ms / wall, 3),
            phases={k: dict(launches=v["launches"], total_ms=round(v["total_ms"], 2), gbps=round(v["gbps"], 1))
                    for k, v in ph.items()},
            inner_residual_first_last=[info.inner_residuals[0], info.inner_residuals[-1]],
            dgels_every_column_ms=round(dgels_ms, 2), givens_ms=round(givens_ms, 3),
            note="gpu_ms = HIP events around the matvec and every Gram-Schmidt kernel family (busy time); "
                 "host_ms = wall - gpu_ms")), flush=True)


if __name__ == "__main__":
    main()
