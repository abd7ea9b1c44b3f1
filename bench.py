#!/usr/bin/env python
"""Benchmark: Arnoldi-step GB/s (achieved HBM) + Ritz-value relative error, N=1e8, m=128.

BASELINE.json config 3: "Synthetic shift-invert Laplacian, N=1e8 dofs, m=128, basis sharded over
MI355X GPUs with RCCL all-reduce" — 3-D spectral-element layout lx1=8, lx2=6, fields
{vx, vy, vz, t} weighted + pressure, E=44,176 elements -> N = 100,014,464 doubles per vector
(SURVEY.md §8(d)).  Total N is fixed for every GPU count (strong scaling): each rank owns an
element-contiguous shard; dots are all-reduced (RCCL) once per Gram–Schmidt pass.

One *step* = one full m-step Arnoldi factorisation from the normalised seed (prepare_seed, then
m x [synthetic matvec + block Gram–Schmidt + normalise], the closing re-orthogonalisation)
followed by the host Ritz extraction (H download, dgeev, residuals) — the work of one
Krylov–Schur cycle before any restart.

``value`` = achieved HBM GB/s of the whole step: the bytes the executed algorithm moves (global N,
all ranks; see ``executed_bytes``) / step time.  The default ``--mode dcgs2`` (CGS2 with delayed
re-orthogonalisation) reads the basis 2x per Arnoldi step (``cgs2``: 3x), so it moves fewer bytes
than SURVEY.md §8(d)'s 4-pass model
  B(j) = 8 [2j(N_w+N) + 2(N_w+n_v) + 4N + n_v + 2N]  (+ 8*3N matvec);
that model divided by the same time is reported separately as ``effective_gbs_survey_model`` (the
work definition the CPU baseline is also measured in; it exceeds the HBM peak because the
executed algorithm does half the model's reads).  ``roofline`` is the dominant kernel family
(two-vector multi-dot, dual update, or the cgs2 kernels) timed live with HIP events on the launch
stream.  ``restart`` (outside the timed region) times one Krylov–Schur condensation of the final
factorisation: the kept-column rotation the solver runs (HBM-bound) and the reference's full
k-column rotation (2Nk^2 flop, priced against the fp64 peak; f64 MFMA).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 spec (vector = matrix on CDNA4); SURVEY.md §8(d) ridge ~10 flop/B


def survey_model_bytes(N, N_w, n_v, m):
    """SURVEY.md §8(d) byte model of a 4-pass CGS2 step, Σ_j B(j), plus the matvec (8*3N per step).
    Used for the CPU baseline and as the *effective* rate of the GPU (same work definition)."""
    tot = 0.0
    for j in range(1, m + 1):
        tot += 8.0 * (2 * j * (N_w + N) + 2 * (N_w + n_v) + 4 * N + n_v + 2 * N)
        tot += 8.0 * 3 * N
    return tot


def executed_bytes(N, N_w, n_v, m, mode, lazy=False):
    """HBM bytes the executed algorithm moves per factorisation (global sizes), per kernel:
    block_dot 8(jN_w + N_w + n_v); fused update_dot 8(jN + 2N + n_v); update+norm 8(jN + 2N + n_v);
    finish 8(2N); diag matvec 8(3N); DCGS2 dual update 8((j-1)N + 4N), over a lazy basis (one
    output vector) 8(jN + 2N).  (PMC FETCH/WRITE_SIZE agree within 1%, profiles/.)"""
    tot = 0.0
    for j in range(1, m + 1):
        dot = 8.0 * (j * N_w + N_w + n_v)
        upd = 8.0 * (j * N + 2 * N)
        if mode == "cgs2":
            tot += dot + (upd + 8.0 * n_v) + (upd + 8.0 * n_v)
        elif mode == "cgs2-unfused":
            tot += 2 * dot + upd + (upd + 8.0 * n_v)
        elif mode == "dcgs2":   # two-vector dot over j-1 streamed columns (+ u, A u); dual update over j-1
            tot += 8.0 * ((j - 1) * N_w + 2 * N_w + n_v)
            tot += 8.0 * (j * N + 2 * N) if lazy else 8.0 * ((j - 1) * N + 4 * N)
        else:
            raise ValueError(mode)
        tot += (0.0 if mode == "dcgs2" else 8.0 * 2 * N) + 8.0 * 3 * N   # normalise pass (not in dcgs2) + matvec
    if mode == "dcgs2":  # closing re-orthogonalisation of q_{m+1}: dot, update, normalise
        tot += 8.0 * ((m + 1) * N_w + N_w + n_v) + 8.0 * (m * N + 2 * N) + 8.0 * 2 * N
    return tot


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(E_sample: int, m: int, threads: int, budget_s: float, variant: str = "mgs2"):
    """The reference algorithm (MGS + full re-orthogonalisation with per-field weighted dots, copy
    -> dot -> cmult -> sub2, krylov_decomposition.f90:155-180) restated in C (oracle/), on the same
    operator family at a bounded sample size, timed on this host.  Steps run until ``budget_s``.
    ``variant="cgs2"``: the optimised CPU line (oracle/cpu_cgs2.c, blocked OpenMP CGS2)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes

    import oracle as orc
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    lay = box3d_layout(E_sample)
    L = orc.OLayout(lay.n_v, lay.n_p, lay.n_wf, False, lay.ldim)
    w = syn.mass_weights(lay)
    d, _ = syn.laplacian_shift_invert(lay)
    dref = syn.to_reference_order(lay, d)
    # the reference-order restatement timed as the reference is deployed (-Ofast, bin/mks:53-55);
    # the strict-order build (liboracle.so) is the parity checker and ~2.5x slower per primitive
    olib = orc.prod_lib()
    olib.orc_set_threads(threads)
    if variant == "cgs2":
        orc.cgs2_lib().cpu_cgs2_set_threads(threads)
        step = orc.cgs2_lib().cpu_cgs2_update_hessenberg
    else:
        step = olib.orc_update_hessenberg
    Q = np.zeros((m + 1, L.len))
    Q[0] = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
    f = L.zeros()
    wrk = L.zeros()
    c = ctypes.byref(L.c)
    done_bytes, t0, steps = 0.0, time.perf_counter(), 0
    for j in range(1, m + 1):
        olib.orc_op_diag(c, dref, Q[j - 1], f, 0.0)
        col = np.zeros(j + 1)
        step(c, w, col, f, Q[:j], j, wrk)  # Q rows are contiguous views
        Q[j] = f
        done_bytes += 8.0 * (2 * j * (lay.N_w + lay.N) + 2 * (lay.N_w + lay.n_v) + 4 * lay.N + lay.n_v + 2 * lay.N)
        done_bytes += 8.0 * 3 * lay.N
        steps = j
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    olib.orc_set_threads(1)
    what = ("reference MGS2 Arnoldi (C restatement oracle/nekstab_oracle.c, built -Ofast like the "
            "reference's bin/mks)" if variant == "mgs2" else
            "optimised CPU: blocked OpenMP CGS2 (oracle/cpu_cgs2.c, AVX2/FMA)")
    return dict(value=done_bytes / dt / 1e9, unit="GB/s", cores=threads, kind="port",
                sample=(f"{what} on the same 3-D lx1=8 layout at E={E_sample} (N={lay.N}), steps j=1..{steps} "
                        f"of m={m}, {dt:.1f} s, {threads} thread(s) on {cpu_model()}; GB/s in SURVEY.md "
                        f"§8(d)'s CGS2 byte model (compare with effective_gbs_survey_model)"),
                seconds=dt)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--E", type=int, default=44176, help="global elements (44,176 -> N=1.0e8)")
    ap.add_argument("--m", type=int, default=128)
    ap.add_argument("--mode", default="dcgs2", help="dcgs2 (default) | cgs2 | cgs2-unfused")
    ap.add_argument("--lazy-basis", action="store_true",
                    help="dcgs2 over a lazy basis Q = S T (one vector write less per step)")
    ap.add_argument("--cpu-E", type=int, default=512)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-restart", action="store_true", help="skip the restart-rotation measurement")
    ap.add_argument("--force-collectives", action="store_true",
                    help="at one GPU, route every partial through a world-1 RCCL group (collective cost)")
    args = ap.parse_args()

    import torch

    from nekstab_next_amd import lapack
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.arnoldi import HessenbergDev, arnoldi_factorization
    from nekstab_next_amd.comm import init_from_env
    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import prepare_seed, schur_condensation
    from nekstab_next_amd.layout import box3d_layout
    from nekstab_next_amd.operators import DiagOperator
    from nekstab_next_amd.profiling import PhaseTimer
    from nekstab_next_amd.vector import NekContext

    comm = init_from_env(os.environ.get("NKV_BACKEND", "nccl"), force_collectives=args.force_collectives)
    rank, world = comm.rank, comm.world
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    glay = box3d_layout(args.E)
    lay = glay.shard(rank, world)
    m = args.m
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, comm=comm, max_cols=m + 1, device=dev)
    d, exact = syn.laplacian_shift_invert(lay)
    op = DiagOperator(ctx, d)
    del d
    seed = ctx.vector()
    seed.fill_hash(11)
    Q = ctx.basis(m + 1)
    Hd = HessenbergDev(ctx, m)
    f = ctx.vector()

    lazy = args.mode == "dcgs2" and args.lazy_basis

    def one_step():
        prepare_seed(seed, Q[0])
        arnoldi_factorization(ctx, op, Q, Hd, 1, m, f=f, mode=args.mode, lazy=lazy)
        H = Hd.download()
        vals, vecs = lapack.eig(H[:m, :m])
        res = np.abs(H[m, m - 1] * vecs[m - 1, :])
        return vals, res

    for _ in range(args.warmup):
        one_step()
    timer = PhaseTimer(dev)
    ctx.timer = timer
    comm.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        vals, res = one_step()
    torch.cuda.synchronize(dev)
    comm.barrier()
    elapsed = time.perf_counter() - t0
    elapsed = comm.max_scalar(elapsed, device=dev)
    ctx.timer = None
    phases = timer.summary()
    last_step_ms = sum(timer.last_ms(k) for k in ("block_dot2", "dcgs2_update")) if args.mode == "dcgs2" else None
    ctx.check_nan()

    # Krylov–Schur restart on the final factorisation (outside the timed region; reported beside
    # the metric): the kept-column rotation the solver runs, and the reference's
    # full k-column rotation priced against the fp64 matrix peak.
    restart = None
    if not args.no_restart:
        rt = PhaseTimer(dev)
        ctx.timer = rt
        # the shift-invert spectrum is not inside the unit disc (every |mu| >= 1 - schur_del would be
        # kept); scale H by its spectral radius as a time-stepper's exp(L dt) spectrum would be —
        # same Schur vectors, the selection rule then keeps the leading cluster + nev + 4
        H = Hd.download()
        H /= np.max(np.abs(vals))
        t1 = time.perf_counter()
        mstart, _sel = schur_condensation(ctx, H, Q, m, KrylovSchurConfig(k_dim=m, schur_tgt=4))
        torch.cuda.synchronize(dev)
        cond_ms = (time.perf_counter() - t1) * 1e3
        V = torch.as_tensor(np.linalg.qr(np.random.default_rng(5).standard_normal((m, m)))[0].ravel(order="F")
                            .copy()).to(dev)
        for _ in range(2):
            rt.begin("rotate_full")
            ctx.call("nkv_rotate", Q.ptr, m, V.data_ptr(), m, ctx.stream)
            rt.end("rotate_full", 16.0 * lay.N * m)
        ctx.timer = None
        rp = rt.summary()
        kept, full = rp["rotate"], rp["rotate_full"]
        full_tf = 2.0 * lay.N * m * m / (full["avg_ms"] * 1e-3) / 1e12
        restart = {
            "mstart": int(mstart), "condensation_wall_ms": round(cond_ms, 2),
            "rotate_kept_ms": round(kept["avg_ms"], 3), "rotate_kept_gbs": round(kept["gbps"], 1),
            "rotate_kept_frac_hbm": round(kept["gbps"] / HBM_PEAK_GBS, 4),
            "rotate_full_ms": round(full["avg_ms"], 3), "rotate_full_tflops": round(full_tf, 2),
            "rotate_full_frac_fp64": round(full_tf / FP64_PEAK_TFLOPS, 4),
        }

    ms_per_step = elapsed / args.steps * 1e3
    nv_g = glay.pts_v * glay.nelgv
    value = executed_bytes(glay.N, glay.N_w, nv_g, m, args.mode, lazy) * args.steps / elapsed / 1e9
    effective = survey_model_bytes(glay.N, glay.N_w, nv_g, m) * args.steps / elapsed / 1e9

    # SURVEY.md §8(d) headline: Gram–Schmidt bytes over Gram–Schmidt time only (matvec, host LAPACK
    # and launch gaps excluded; kernel-bracketed HIP events, this rank), and the last step alone
    gs_fams = ("block_dot", "update_dot", "block_update", "finish", "block_dot2", "dcgs2_update")
    gs_ms = sum(phases[k]["total_ms"] for k in gs_fams if k in phases) / args.steps
    gs_exec = sum(phases[k]["avg_bytes"] * phases[k]["launches"] for k in gs_fams if k in phases) / args.steps
    survey_gs = survey_model_bytes(lay.N, lay.N_w, lay.n_v, m) - m * 8.0 * 3 * lay.N
    b_last = 8.0 * (2 * m * (lay.N_w + lay.N) + 2 * (lay.N_w + lay.n_v) + 4 * lay.N + lay.n_v + 2 * lay.N)
    gs = {"gs_ms_per_factorisation": round(gs_ms, 2),
          "executed_gs_gbs": round(gs_exec / (gs_ms * 1e-3) / 1e9, 1),
          "survey_headline_gbs": round(survey_gs / (gs_ms * 1e-3) / 1e9, 1),
          "last_step_ms": None if last_step_ms is None else round(last_step_ms, 3),
          "last_step_survey_gbs": None if last_step_ms is None else round(b_last / (last_step_ms * 1e-3) / 1e9, 1),
          "note": "per rank; survey_* use SURVEY.md 8(d)'s 4-pass CGS2 byte model B(j) for the same work"}

    # Ritz accuracy vs the exact spectrum of the synthetic operator
    # (exact spectrum: the 4096 largest |mu|; a converged Ritz value is matched to the nearest one)
    conv = res < 1e-6
    errs = [float(np.min(np.abs(exact - v)) / abs(v)) for v in vals[conv]] if conv.any() else []
    ritz_err = max(errs) if errs else None
    top_err = float(np.max(np.abs(vals[:8] - exact[:8]) / np.abs(exact[:8])))

    # dominant kernel family (rank-local launches; bytes are this rank's shard)
    dom = max(("block_dot", "update_dot", "block_update", "block_dot2", "dcgs2_update"),
              key=lambda k: phases.get(k, {}).get("total_ms", 0.0))
    ph = phases[dom]
    achieved = ph["gbps"]
    traffic = None
    tpath = os.path.join(ROOT, "profiles", "traffic_latest.json")
    if os.path.exists(tpath):
        try:
            tj = json.load(open(tpath))
            if tj.get("kernel_family") == dom and tj.get("E") == args.E and tj.get("m") == m and world == 1:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    if rank == 0:
        cpu = cpu1 = cpu_opt = None
        if not args.no_cpu and world == 1:
            threads = min(16, os.cpu_count() or 1)   # the box's CPU share is 16 cores
            cpu = cpu_baseline(args.cpu_E, m, threads, args.cpu_budget)
            cpu1 = cpu_baseline(args.cpu_E, m, 1, args.cpu_budget / 2)
            cpu_opt = cpu_baseline(args.cpu_E, m, threads, args.cpu_budget / 2, variant="cgs2")
        out = {
            "metric": "Arnoldi-step GB/s (achieved HBM) + Ritz-value rel-err, N=1e8 m=128",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "effective_gbs_survey_model": round(effective, 2),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (diagonalised shift-invert Laplacian, hashed seed, GLL x J_e weights)",
            "config": {
                "workload": f"config3: m-step Arnoldi ({args.mode.upper()}) + Ritz extraction, shift-invert Laplacian",
                "N": glay.N, "N_w": glay.N_w, "E": args.E, "layout": "3D lx1=8 lx2=6 {vx,vy,vz,t}+pr",
                "m": m, "mode": args.mode + ("-lazy" if lazy else ""), "parallelism": (f"element-shard x{world} + " + ("RCCL" if comm.backend == "nccl" else str(comm.backend))
                                + " allreduce") if world > 1 else "single GPU",
            },
            "roofline": {
                "bound": "hbm",
                "kernel": dom,
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "avg_launch_ms": round(ph["avg_ms"], 4),
                "avg_bytes_per_launch": ph["avg_bytes"],
                "launches": ph["launches"],
            },
            "phases": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                       for k, v in phases.items()},
            "gram_schmidt": gs,
            "ritz_rel_err": ritz_err,
            "ritz_top8_rel_err": top_err,
            "ritz_converged": int(conv.sum()),
            "cpu_baseline": ({k: v for k, v in cpu.items() if k != "seconds"} if cpu else None),
            "cpu_baseline_1core": ({k: v for k, v in cpu1.items() if k != "seconds"} if cpu1 else None),
            "cpu_optimised": ({k: v for k, v in cpu_opt.items() if k != "seconds"} if cpu_opt else None),
            "restart": restart,
        }
        print(json.dumps(out), flush=True)
    comm.barrier()
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()   # every rank leaves the RCCL group before the process exits


if __name__ == "__main__":
    main()
