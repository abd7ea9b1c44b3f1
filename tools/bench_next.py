#!/usr/bin/env python
"""Measure the §8(f) "next" rows on one MI355X (bench.py measures the hot path itself):

* f1 LightKrylov-style ``svds`` (transient growth: k-step Golub–Kahan–Lanczos, two bases resident,
  full re-orthogonalisation: the default delayed DCGS2 form, two reads of each basis per step, and
  CGS2, three reads) at N=50,007,232, k=32 — wall time and the Gram–Schmidt kernels'
  achieved HBM GB/s (HIP events on the launch stream, algorithmic bytes as in bench.py);
  ``get_vec`` (one combination of k basis vectors, nkv_combine) GB/s.
* f1/a19 mode reconstruction of the in-tree solver (``ritz_vector``: two real combinations).
* f2 checkpoint: one KRY field file (Nek5000 #std, fp64) of an N=50,007,232 vector written and read
  back through the product's writer/reader (host I/O, device<->host copies included) — MB/s.
* f4 BoostConv ``core`` (bst_snp = 10, velocity-only layout of the scaled cylinder, N=1,636,416 per
  vector) — ms per call (its QR is the reference's MGS order, scalars device-resident).
* f3 .fld I/O is host-only; its throughput is the f2 line.
* f5 wave-maker pointwise kernel (``nkv_wavemaker``, sensitivity.f90:69-71) on config 5's velocity
  layout (3 components, n_v = 11,309,056) — GB/s of its 8 (4 ldim + 1) n_v bytes.
Prints one JSON object per measurement.
"""
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.boostconv import BoostConv, velocity_layout
    from nekstab_next_amd.checkpoint import ArnoldiCheckpoint
    from nekstab_next_amd.layout import box3d_layout, cylinder_layout
    from nekstab_next_amd.lightkrylov import get_vec, svds
    from nekstab_next_amd.operators import DiagOperator
    from nekstab_next_amd.profiling import PhaseTimer
    from nekstab_next_amd.vector import NekContext, k_normalize

    dev = torch.device("cuda", 0)
    lay = box3d_layout(22088)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=40)
    d, exact = syn.laplacian_shift_invert(lay)
    op = DiagOperator(ctx, d / np.abs(exact[0]))   # symmetric in W: singular values = |eigenvalues|
    k = 32
    U, V = ctx.basis(k + 1), ctx.basis(k + 1)
    for mode in ("dcgs2", "cgs2"):
        for rep in range(2):                            # warm-up, then timed with phase events
            V[0].fill_hash(11)
            k_normalize(V[0])
            timer = PhaseTimer(dev) if rep else None
            ctx.timer = timer
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            res = svds(ctx, op, U, V, nev=4, tolerance=1e-8, mode=mode)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            ctx.timer = None
        ph = timer.summary()
        gs = {n: ph[n] for n in ("block_dot", "update_dot", "block_update", "finish", "block_dot2", "dcgs2_update")
              if n in ph}
        gs_ms = sum(v["total_ms"] for v in gs.values())
        gs_b = sum(v["avg_bytes"] * v["launches"] for v in gs.values())
        top = np.sort(np.abs(exact / exact[0]))[::-1][:4]
        print(json.dumps(dict(row="f1_svds", mode=mode, N=lay.N, k=k, seconds=round(dt, 4),
                              gram_schmidt_ms=round(gs_ms, 2), gram_schmidt_gb=round(gs_b / 1e9, 2),
                              gram_schmidt_gbs=round(gs_b / (gs_ms * 1e-3) / 1e9, 1),
                              phases={n: dict(launches=v["launches"], gbps=round(v["gbps"], 1)) for n, v in gs.items()},
                              sigma_top4=[float(s) for s in res.sigma[:4]],
                              sigma_top4_rel_err=float(np.max(np.abs(res.sigma[:4] - top) / top)))), flush=True)

    out = ctx.vector()
    coeffs = np.random.default_rng(1).standard_normal(k)
    get_vec(out, V, coeffs, k)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    reps = 5
    for _ in range(reps):
        get_vec(out, V, coeffs, k)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    print(json.dumps(dict(row="f1_get_vec", N=lay.N, k=k, ms=round(ms, 3),
                          gbs=round(8.0 * (k + 1) * lay.N / (ms * 1e-3) / 1e9, 1))), flush=True)

    # f2: one KRY file of this N through the checkpoint writer, and back through the reader
    with tempfile.TemporaryDirectory(dir=os.environ.get("NKV_BENCH_TMP")) as tmp:
        ck = ArnoldiCheckpoint(ctx, tmp, session="bench", write_spectra=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ck.write_vector(V[1], 2, time=1.0)
        tw = time.perf_counter() - t0
        path = os.path.join(tmp, fld.fld_name("KRY", "bench", 0, 2))
        nbytes = os.path.getsize(path)
        t0 = time.perf_counter()
        files = fld.read_fld_set(tmp, "KRY", "bench", 2)
        back = ctx.vector().from_packed(fld.vector_from_fld(lay, files))
        torch.cuda.synchronize()
        tr = time.perf_counter() - t0
        nw = lay.n_wf * lay.sv
        same = bool(torch.equal(back.storage[:nw], V[1].storage[:nw]))
        pa, pb = back.storage[nw: lay.rows], V[1].storage[nw: lay.rows]
        pdiff = float((pa - pb).abs().max() / pb.abs().max())
    print(json.dumps(dict(row="f2_checkpoint_kry", N=lay.N, file_bytes=nbytes, write_s=round(tw, 3),
                          write_mbs=round(nbytes / tw / 1e6, 1), read_s=round(tr, 3), read_mbs=round(nbytes / tr / 1e6, 1),
                          weighted_fields_bit_identical=same, pressure_round_trip_rel_diff=pdiff,
                          note="pressure is written on the velocity (GLL) mesh and mapped back to the lx2 "
                               "Gauss mesh on read, exact to rounding")), flush=True)
    del U, V, out, ctx, op

    # f5: the wave-maker's pointwise kernel on config 5's velocity layout
    from nekstab_next_amd.sensitivity import velocity_layout as sens_velocity_layout, wavemaker_field

    wlay = sens_velocity_layout(lay)
    wctx = NekContext(wlay, weights=syn.mass_weights(wlay), max_cols=4)
    vs = []
    for s_ in range(4):
        v = wctx.vector()
        v.fill_hash(500 + s_)
        vs.append(v)
    wm = wavemaker_field(wctx, *vs)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        wavemaker_field(wctx, *vs, out=wm)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    nb = 8.0 * (4 * wlay.ldim + 1) * wlay.n_v
    print(json.dumps(dict(row="f5_wavemaker", n_v=wlay.n_v, ms=round(ms, 3), gbs=round(nb / (ms * 1e-3) / 1e9, 1),
                          bytes=nb)), flush=True)
    del wctx, vs, wm

    # f4: BoostConv on the scaled cylinder's velocity layout
    vlay = velocity_layout(cylinder_layout(22728))
    vctx = NekContext(vlay, weights=syn.mass_weights(vlay), max_cols=16)
    bc = BoostConv(vctx, bst_snp=10)
    rb = vctx.vector()
    for it in range(14):            # fill the residual subspace, then time calls
        rb.fill_hash(100 + it)
        if it == 11:
            torch.cuda.synchronize()
            t0 = time.perf_counter()
        bc.core(rb)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 3
    print(json.dumps(dict(row="f4_boostconv_core", N=vlay.N, bst_snp=10, ms_per_call=round(per * 1e3, 3),
                          note="QR in the reference's MGS order (fixedp.f90:331-385), dots and projections "
                               "device-resident: one host synchronisation per QR")), flush=True)


if __name__ == "__main__":
    main()
