#!/usr/bin/env python
"""Benchmark: Arnoldi-step GB/s (achieved HBM) + Ritz-value relative error, N=1e8, m=128.

BASELINE.json config 3: "Synthetic shift-invert Laplacian, N=1e8 dofs, m=128, basis sharded over
MI355X GPUs with RCCL all-reduce" — 3-D spectral-element layout lx1=8, lx2=6, fields
{vx, vy, vz, t} weighted + pressure, E=44,176 elements -> N = 100,014,464 doubles per vector
(SURVEY.md §8(d)).  Total N is fixed for every GPU count (strong scaling): each rank owns an
element-contiguous shard; dots are all-reduced (RCCL) once per Arnoldi step.

Launch.  ``python bench.py --gpus N`` with N > 1 and no ``WORLD_SIZE`` in the environment spawns N
child processes of itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT,
as ``torch.distributed.run`` sets them) before anything touches the GPU, waits for them and exits
with the worst child exit status (no exec).  Under ``torch.distributed.run`` the environment is
already set and ``--gpus`` must equal ``WORLD_SIZE`` (else exit 2).  ``--dry-launch`` stops every
rank before GPU initialisation and prints its rank environment (CPU test of the launcher).

One *step* = one full m-step Arnoldi factorisation from the normalised seed (prepare_seed, then
m x [synthetic matvec + block Gram–Schmidt], the closing re-orthogonalisation) followed by the
host Ritz extraction (H download, dgeev, residuals) — the work of one Krylov–Schur cycle before
any restart.

``value`` = achieved HBM GB/s of the whole step: the bytes the executed algorithm moves (global N,
all ranks; see ``executed_bytes``) / step time (max over ranks).  One byte model per line: every
GB/s field is executed bytes over measured time, so none can exceed the 8 TB/s peak.  The default
``--mode dcgs2`` (CGS2 with delayed re-orthogonalisation) reads the basis 2x per Arnoldi step
(``cgs2``: 3x); SURVEY.md §8(d)'s 4-pass model
  B(j) = 8 [2j(N_w+N) + 2(N_w+n_v) + 4N + n_v + 2N]  (+ 8*3N matvec)
enters only as the dimensionless ``survey_model_time_ratio``: the time that model's bytes take at
the 8 TB/s peak over the measured step time (> 1: the step is faster than a 4-pass CGS2 could be
even at roofline).  ``roofline`` is the dominant kernel family timed live with HIP events on the
launch stream.  Outside the timed region: ``restart`` times one
Krylov–Schur condensation of the final factorisation (H rescaled to unit spectral radius, see
there), ``krylov_schur_leg`` runs config 3's Krylov–Schur (k_dim=m, schur_tgt=4) and
``krylov_schur_restart_leg`` the same on a clustered time-stepper-like spectrum that needs real
m-column restarts.
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

ROT_WIDE_KEPT = 25   # kept columns of the Krylov–Schur restart leg's first restart at m = 128
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)
FP64_PEAK_TFLOPS = 78.6  # MI355X fp64 spec (vector = matrix on CDNA4); SURVEY.md §8(d) ridge ~10 flop/B
N_HEADLINE = 100_014_464  # config 3, E=44,176
# multi-rank wall clocks (seconds; env NKV_RANK_WALL_S / NKV_LAUNCH_WALL_S override, <= 0 disables):
# a rank ends itself first (stack dump, status 124), the launcher is the backstop; both sit below the
# driver's 600 s budget for one bench line
DEFAULT_RANK_WALL_S = "540"
DEFAULT_LAUNCH_WALL_S = "570"


# ---- byte models ---------------------------------------------------------------------------------

def survey_step_bytes(N, N_w, n_v, j):
    """SURVEY.md §8(d) B(j) of a 4-pass CGS2 step plus the matvec (8*3N)."""
    return 8.0 * (2 * j * (N_w + N) + 2 * (N_w + n_v) + 4 * N + n_v + 2 * N) + 8.0 * 3 * N


def survey_model_bytes(N, N_w, n_v, m):
    """Σ_j B(j) (+ matvec): the 4-pass CGS2 of SURVEY.md §8(d) (also the bytes oracle/cpu_cgs2.c,
    the optimised CPU line, executes: two blocked dot + update passes per step)."""
    return sum(survey_step_bytes(N, N_w, n_v, j) for j in range(1, m + 1))


def reference_step_bytes(N, N_w, n_v, j):
    """Bytes the reference's own MGS2 moves at step j (update_hessenberg_matrix,
    krylov_decomposition.f90:152-186), per basis column and pass: k_copy 2N, k_dot 3N_w (p, w, q per
    weighted field), k_cmult 2N, k_sub2 3N; plus the unused k_norm (:152, 3N_w), the closing
    k_normalize (3N_w + 2N) and the matvec (3N).  ≈ 20jN per step."""
    return 8.0 * (2 * j * (7 * N + 3 * N_w) + 6 * N_w + 2 * N + 3 * N)


def executed_bytes(N, N_w, n_v, m, mode):
    """HBM bytes the executed algorithm moves per factorisation (global sizes), per kernel:
    block_dot 8(jN_w + N_w + n_v); fused update_dot 8(jN + 2N + n_v); update+norm 8(jN + 2N + n_v);
    finish 8(2N); diag matvec 8(3N); DCGS2 dual update 8((j-1)N + 4N);
    mgs2-icwy: a two-vector dot 8((j-1)N_w + 2N_w + n_v) then the cgs2 update_dot and
    update+norm; mgs2 (the reference's order) one dot 8(2N_w + n_v), then per column
    and pass one fused axpy + next dot (nkv_axpy_dot) 8(3N + N_w + n_v), the last one's dot the norm.  A "-native" mode moves the bytes of its twin."""
    mode = mode.replace("-native", "")
    tot = 0.0
    for j in range(1, m + 1):
        dot = 8.0 * (j * N_w + N_w + n_v)
        upd = 8.0 * (j * N + 2 * N)
        if mode == "mgs2":   # a dot, then 2j fused column passes (the last one's dot is ||f||^2)
            tot += 8.0 * (2 * N_w + n_v) + 2 * j * 8.0 * (3 * N + N_w + n_v) - 8.0 * N_w
        elif mode == "cgs2":
            tot += dot + (upd + 8.0 * n_v) + (upd + 8.0 * n_v)
        elif mode == "mgs2-icwy":   # two-vector dot (Gram row + pass-1 dots), fused update+dot, update+norm
            tot += 8.0 * ((j - 1) * N_w + 2 * N_w + n_v) + (upd + 8.0 * n_v) + (upd + 8.0 * n_v)
        elif mode in ("dcgs2", "mgs2-lagged"):   # two-vector dot over j-1 streamed columns (+ u, A u); dual
            # update over j-1 (mgs2-lagged: the same two kernels with MGS2's coefficients from the host)
            tot += 8.0 * ((j - 1) * N_w + 2 * N_w + n_v)
            tot += 8.0 * ((j - 1) * N + 4 * N)
        else:
            raise ValueError(mode)
        tot += (0.0 if mode in ("dcgs2", "mgs2-lagged") else 8.0 * 2 * N) + 8.0 * 3 * N   # normalise (not
        # in the delayed forms) + matvec
    if mode in ("dcgs2", "mgs2-lagged"):  # closing re-orthogonalisation of q_{m+1}: dot, update, normalise
        tot += 8.0 * ((m + 1) * N_w + N_w + n_v) + 8.0 * (m * N + 2 * N) + 8.0 * 2 * N
        if mode == "mgs2-lagged":   # its closing update carries the fused norm (the weights once more)
            tot += 8.0 * n_v
    return tot


# ---- host CPU facts ----------------------------------------------------------------------------

def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpus():
    """CPU quota of this process's cgroup in CPUs (v2 cpu.max or v1 cfs quota), None if unlimited."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(p)
    except (OSError, ValueError):
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else q / p
    except (OSError, ValueError):
        return None


def host_threads() -> dict:
    """Threads the CPU baseline uses: every CPU this process may run on (sched_getaffinity),
    capped by the cgroup quota and by the host's declared CPU share (OMP_NUM_THREADS: 16 per GPU
    on the GPU boxes, whose nproc shows the whole machine).  All inputs are recorded."""
    aff = len(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    omp = os.environ.get("OMP_NUM_THREADS")
    n = aff
    if quota is not None:
        n = min(n, max(1, int(quota)))
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return dict(threads=n, affinity_cpus=aff, nproc=os.cpu_count(), cgroup_quota_cpus=quota,
                omp_num_threads=omp, cpu=cpu_model())


# ---- CPU baseline ------------------------------------------------------------------------------

def cpu_baseline(E_sample: int, m: int, threads: int, variant: str = "mgs2", n_full: int = N_HEADLINE,
                 fit_js=(1, 32, 64, 128), progress: bool = False):
    """The reference algorithm timed on this host: ONE complete m-step Arnoldi factorisation (after
    one untimed warm-up step) — the synthetic matvec, then MGS + full re-orthogonalisation with
    per-field weighted dots (copy -> dot -> cmult -> sub2, krylov_decomposition.f90:68-96,
    152-186), restated in C (oracle/nekstab_oracle.c, built -Ofast like the reference's
    bin/mks:53-55) — on the config-3 layout at ``E_sample`` elements, seeded like the GPU run
    (hashed seed normalised with real_dot, prepare_seed).  ``seconds_per_factorisation_sample`` is
    that measured wall time; it is scaled by N to BASELINE's N=1e8 (the steps stream the basis
    from DRAM: linear in N; ``tools/cpu_factorisation.py`` measured the scaling on the GPU box).
    ``fit_check``: the round-3 method (t(j) = a + b j fitted to the steps ``fit_js`` only, summed
    over j = 1..m) evaluated on this run's own step times, with its error against the measured
    total.  ``variant="cgs2"``: the optimised CPU line (oracle/cpu_cgs2.c, blocked OpenMP CGS2).
    ``progress``: a line on stderr every 8 steps (long samples: a silent process looks hung)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ctypes

    import oracle as orc
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    lay = box3d_layout(E_sample)
    L = orc.OLayout(lay.n_v, lay.n_p, lay.n_wf, False, lay.ldim)
    c = ctypes.byref(L.c)
    olib = orc.prod_lib()
    olib.orc_set_threads(threads)
    if variant == "cgs2":
        orc.cgs2_lib().cpu_cgs2_set_threads(threads)
        step = orc.cgs2_lib().cpu_cgs2_update_hessenberg
    else:
        step = olib.orc_update_hessenberg
    w = syn.mass_weights(lay)
    d, _ = syn.laplacian_shift_invert(lay)
    dref = syn.to_reference_order(lay, d)
    del d
    Q = np.empty((m + 1, L.len))
    Q[1:] = 0.0   # k_zero(Q(1:k_dim+1)) before the factorisation (eigensolvers.f90:154): pages touched untimed
    Q[0] = syn.to_reference_order(lay, syn.hash_vector(lay, 11))
    Q[0] /= np.sqrt(float(np.sum(np.concatenate([w] * lay.n_wf) * Q[0][: lay.N_w] ** 2)) + Q[0][-1] ** 2)
    f, wrk = L.zeros(), L.zeros()
    col = np.zeros(m + 1)
    olib.orc_op_diag(c, dref, Q[0], f, 0.0)       # warm-up step (first touch of f / wrk, thread pool)
    step(c, w, col, f, Q[:1], 1, wrk)
    t_step = np.zeros(m)
    t0 = time.perf_counter()
    for j in range(1, m + 1):
        ts = time.perf_counter()
        olib.orc_op_diag(c, dref, Q[j - 1], f, 0.0)      # matvec(f, Q(mstep))
        step(c, w, col, f, Q[:j], j, wrk)                # update_hessenberg_matrix
        Q[j] = f                                         # k_copy(Q(mstep+1), f)
        t_step[j - 1] = time.perf_counter() - ts
        if progress and (j % 8 == 0 or j == m):
            print(f"cpu_baseline E={E_sample}: step {j}/{m}, {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
    sec_fact = time.perf_counter() - t0
    olib.orc_set_threads(1)
    del Q
    js = [j for j in fit_js if j <= m]
    jj = np.array(js, dtype=np.float64)
    tt = t_step[np.array(js) - 1]
    b, a = np.polyfit(jj, tt, 1) if len(jj) > 1 else (tt[0] / jj[0], 0.0)
    fit_total = m * a + b * m * (m + 1) / 2.0
    scale = n_full / lay.N
    surv = survey_model_bytes(lay.N, lay.N_w, lay.n_v, m)
    refb = sum(reference_step_bytes(lay.N, lay.N_w, lay.n_v, j) for j in range(1, m + 1))
    what = ("reference MGS2 Arnoldi (C restatement oracle/nekstab_oracle.c, built -Ofast like the "
            "reference's bin/mks)" if variant == "mgs2" else
            "optimised CPU: blocked OpenMP CGS2 (oracle/cpu_cgs2.c, AVX2/FMA)")
    # executed bytes of the algorithm this CPU line runs (the GPU value's basis: bytes the executed
    # algorithm moves / time): the reference's MGS2 with its copies, or the 4-pass blocked CGS2
    execb = refb if variant == "mgs2" else surv
    return dict(
        value=round(execb / sec_fact / 1e9, 2), unit="GB/s (bytes the timed CPU algorithm executes)", cores=threads,
        kind="port",
        executed_bytes_model=("reference MGS2: per column and pass k_copy 2N + k_dot 3N_w + k_cmult 2N + k_sub2 3N, "
                              "+ unused k_norm, k_normalize, matvec (bench.reference_step_bytes)" if variant == "mgs2"
                              else "4-pass CGS2 with fused norm + matvec (SURVEY.md 8(d) B(j), bench.survey_model_bytes)"),
        seconds_per_factorisation_sample=round(sec_fact, 3),
        seconds_per_factorisation_measured=True,
        E_sample=E_sample,
        seconds_scaled_from_sample_N1e8=round(sec_fact * scale, 2),
        step_seconds={int(j): round(float(t_step[j - 1]), 4) for j in sorted(set(js + [m]))},
        fit_check={"js": js, "fitted_total_s": round(fit_total, 3),
                   "rel_err_vs_measured": round((fit_total - sec_fact) / sec_fact, 4)},
        sample=(f"{what}; config-3 layout (3-D lx1=8, {{vx,vy,vz,t}}+pr) at E={E_sample} (N={lay.N}); one complete "
                f"m={m} factorisation (matvec + update_hessenberg_matrix + k_copy per step) timed after one warm-up "
                f"step; " + (f"seconds scaled by N to N={n_full}" if lay.N != n_full else "full size, unscaled")
                + f"; {threads} thread(s) on {cpu_model()}"))


FULL_SIZE_FILES = {"mgs2": "cpu_full_size_latest.json", "cgs2": "cpu_full_size_cgs2_latest.json"}


def cpu_full_size_run(E: int, m: int, gpu_ms_per_step: float, variant: str = "mgs2", threads: int | None = None):
    """The same CPU factorisation measured ONCE at full size on the GPU box's host, outside this run
    (``tools/cpu_factorisation.py <out> <E> [--variant cgs2]``, minutes at N=1e8, too long for the
    bench's own sample): read from ``profiles/cpu_full_size_latest.json`` (the reference MGS2) or
    ``profiles/cpu_full_size_cgs2_latest.json`` (the optimised CPU CGS2) when it matches this
    workload (E, m) and, if given, this host's thread count; else None.  It is never ``value``."""
    path = os.path.join(ROOT, "profiles", FULL_SIZE_FILES[variant])
    if not os.path.exists(path):
        return None
    try:
        fj = json.load(open(path))
        r = fj["runs"][0]
        if r.get("E") != E or fj.get("m") != m or (threads is not None and int(r["cores"]) != int(threads)):
            return None
        s = float(r["seconds_per_factorisation_sample"])
        return {"seconds_per_factorisation": s, "E": r["E"], "threads": r["cores"], "kind": r["kind"],
                "file": "profiles/" + FULL_SIZE_FILES[variant], "collected": fj.get("tag"), "head": fj.get("head"),
                "cpu": (fj.get("host") or {}).get("cpu"),
                "time_to_solution_ratio_cpu_over_gpu": round(s / (gpu_ms_per_step * 1e-3), 1),
                "note": "measured separately on the GPU box's host (not in this run): one complete "
                        "factorisation of this CPU algorithm at this N"}
    except (OSError, ValueError, KeyError, IndexError, TypeError):
        return None


def lead_with_measured(c: dict, full: dict | None, gpu_ms: float) -> dict:
    """The seconds-to-solution at N=1e8 and the CPU/GPU time ratio come from a measurement: the
    full-size run when one exists for this algorithm, workload and thread count.
    The bounded sample's N-scaled figure stays beside it as ``seconds_scaled_from_sample_N1e8`` with
    its error against the measurement; without a full-size run the ratio is reported only as an
    ``..._estimate`` and ``seconds_per_factorisation_N1e8`` is null."""
    c["gpu_ms_per_factorisation"] = round(gpu_ms, 2)
    c["full_size_run"] = full
    scaled = c["seconds_scaled_from_sample_N1e8"]
    if full is not None:
        s = full["seconds_per_factorisation"]
        c["seconds_per_factorisation_N1e8"] = s
        c["seconds_per_factorisation_N1e8_source"] = (f"measured at full size, E={full['E']}, {full['threads']} "
                                                      f"threads ({full['file']}, {full['collected']})")
        c["time_to_solution_ratio_cpu_over_gpu"] = round(s / (gpu_ms * 1e-3), 1)
        c["sample_scaled_over_measured"] = round(scaled / s, 3)
    else:
        c["seconds_per_factorisation_N1e8"] = None
        c["seconds_per_factorisation_N1e8_source"] = "not measured at full size for this algorithm / thread count"
        c["time_to_solution_ratio_cpu_over_gpu"] = None
        c["time_to_solution_ratio_estimate"] = round(scaled / (gpu_ms * 1e-3), 1)
        c["estimate_note"] = ("the bounded sample scaled linearly in N (an estimate; for the reference MGS2 on 16 "
                              "threads that scaling over-stated the full-size measurement by ~19-30 %)")
    return c


PORT_NOTE = ("the C port runs up to ~1.7x slower than the reference's own Fortran did in the survey's "
             "single-core probe (E=2000, m=16: 7.1 s vs 4.215 s; CHANGELOG.md round 3), so the CPU time "
             "may over-state the reference's by up to that factor")


def host_baselines(args, m: int, gpu_ms: float) -> dict:
    """The three CPU lines timed live on this host (rank 0 only, after every rank has left the
    process group at world > 1, so no peer waits in a collective meanwhile), each led by its
    measured full-size figures where they exist.  The all-threads sample shrinks with the thread
    count (E = cpu_E x threads / 16, at least cpu_E_1core) so that it stays a bounded ~30 s of CPU
    work when a launcher leaves few threads (torch.distributed.run sets OMP_NUM_THREADS=1 unless
    the environment sets it)."""
    host = host_threads()
    e_all = max(args.cpu_E_1core, min(args.cpu_E, args.cpu_E * host["threads"] // 16))
    cpu = cpu_baseline(e_all, m, host["threads"])
    cpu1 = cpu_baseline(args.cpu_E_1core, m, 1)
    cpu_opt = cpu_baseline(e_all, m, host["threads"], variant="cgs2")
    lead_with_measured(cpu, cpu_full_size_run(args.E, m, gpu_ms, "mgs2", host["threads"]), gpu_ms)
    lead_with_measured(cpu1, cpu_full_size_run(args.E, m, gpu_ms, "mgs2", 1), gpu_ms)
    lead_with_measured(cpu_opt, cpu_full_size_run(args.E, m, gpu_ms, "cgs2", host["threads"]), gpu_ms)
    cpu["host"] = host
    for c in (cpu, cpu1):
        c["sample"] += "; " + PORT_NOTE
    return {"cpu_baseline": cpu, "cpu_baseline_1core": cpu1, "cpu_optimised": cpu_opt}


def find_traffic(dom: str, E_shard: int, m: int):
    """PMC HBM bytes per launch of the dominant kernel family for a rank whose shard holds
    ``E_shard`` elements: ``profiles/traffic_latest.json`` (the full one-GPU size) or
    ``profiles/traffic_E<E>.json`` (a shard size measured alone on one GPU: the same per-launch
    bytes a rank of that shard moves at world > 1).  Returns (bytes, provenance) or (None, None)."""
    import glob

    paths = [os.path.join(ROOT, "profiles", "traffic_latest.json")]
    paths += sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_E*.json")))
    for path in paths:
        try:
            tj = json.load(open(path))
        except (OSError, ValueError):
            continue
        if tj.get("kernel_family") == dom and tj.get("E") == E_shard and tj.get("m") == m:
            return tj.get("hbm_bytes_per_launch"), {
                "file": os.path.relpath(path, ROOT), "collected": tj.get("tag") or tj.get("source"),
                "box": tj.get("box"), "head": tj.get("head"), "E_shard": E_shard,
                "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + WRITE_SIZE, separate passes, "
                          "tools/pmc_traffic.py; one GPU running a shard of this size alone; not collected in "
                          "this run"}
    return None, None


# ---- launcher ----------------------------------------------------------------------------------

def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch(n: int, argv, grace_s: float = 60.0, wall_s: float = 0.0) -> int:
    """Spawn ``n`` ranks of this script (torch.distributed.run's environment, no exec) and return
    the worst exit status.  If one rank fails, the others get ``grace_s`` to finish (a rank blocked
    in a collective never does) and are then terminated.  ``wall_s`` > 0 bounds the whole job: a
    hang in which every rank sits in a collective (no rank exits, so no grace period starts) is
    terminated at ``wall_s`` and the launcher exits 124 — before the driver's own limit."""
    port = int(os.environ.get("MASTER_PORT") or _free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NKV_BENCH_LAUNCHER="1")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *argv], env=env))

    def _stop(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)
        raise SystemExit(128 + signum)

    old = {s: signal.signal(s, _stop) for s in (signal.SIGTERM, signal.SIGINT)}
    rcs = [None] * n
    t_fail = None
    t_start = time.monotonic()
    timed_out = False
    try:
        while any(rc is None for rc in rcs):
            if wall_s > 0 and not timed_out and time.monotonic() - t_start > wall_s:
                timed_out = True
                alive = [i for i in range(n) if rcs[i] is None]
                print(f"bench launcher: wall clock of {wall_s:.0f} s exceeded with ranks {alive} still running; "
                      "terminating every rank", file=sys.stderr, flush=True)
                t_fail = time.monotonic() - grace_s - 1.0     # no grace: stop them now

            for i, p in enumerate(procs):
                if rcs[i] is None:
                    rc = p.poll()
                    if rc is not None:
                        rcs[i] = rc
                        if rc != 0 and t_fail is None:
                            t_fail = time.monotonic()
                            print(f"bench launcher: rank {i} exited with {rc}", file=sys.stderr, flush=True)
            if t_fail is not None and time.monotonic() - t_fail > grace_s:
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        p.terminate()
                for i, p in enumerate(procs):
                    if rcs[i] is None:
                        try:
                            rcs[i] = p.wait(timeout=20)
                        except subprocess.TimeoutExpired:
                            p.kill()
                            rcs[i] = p.wait()
            time.sleep(0.05)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
    norm = [rc if rc >= 0 else 128 - rc for rc in rcs]   # killed by signal k -> 128 + k
    worst = max(norm)
    return 124 if timed_out and worst in (0, 128 + signal.SIGTERM, 128 + signal.SIGKILL) else worst


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--E", type=int, default=44176, help="global elements (44,176 -> N=1.0e8)")
    ap.add_argument("--m", type=int, default=128)
    ap.add_argument("--mode", default="dcgs2",
                    help="dcgs2 (default) | cgs2 | mgs2 (reference order) | dcgs2-native | "
                         "cgs2-native | mgs2-native (the one-call C drivers) | mgs2-icwy (MGS in inverse compact WY form) "
                         "| mgs2-lagged[-native] (MGS2's coefficients, second pass lagged: the non-orthonormal-seed "
                         "default)")
    ap.add_argument("--cpu-E", type=int, default=2000,
                    help="CPU baseline sample: one full factorisation on all threads (2,000 -> N=4.5e6, ~20 s)")
    ap.add_argument("--cpu-E-1core", type=int, default=128, help="... with one thread (128 -> N=2.9e5)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-restart", action="store_true", help="skip the restart-rotation measurement")
    ap.add_argument("--no-ks", action="store_true", help="skip the Krylov–Schur restart leg")
    ap.add_argument("--force-collectives", action="store_true",
                    help="at one GPU, route every partial through a world-1 RCCL group (collective cost)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="print each rank's launch environment and stop before GPU initialisation")
    ap.add_argument("--dry-line", action="store_true",
                    help="CPU rehearsal of the JSON line at any world size: gloo ranks, fabricated (labelled) "
                         "measurements, the real line assembly and the real rank-0 CPU baselines")
    ap.add_argument("--collective-probe", action="store_true",
                    help="CPU test of the collective path: init the process group (bounded timeout, rank "
                         "watchdog), gather the ranks' device identities, one all-reduce, print one JSON line")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    ws = os.environ.get("WORLD_SIZE")
    if ws is None and args.gpus > 1:
        sys.exit(launch(args.gpus, sys.argv[1:], grace_s=float(os.environ.get("NKV_LAUNCH_GRACE_S", "60")),
                        wall_s=float(os.environ.get("NKV_LAUNCH_WALL_S", DEFAULT_LAUNCH_WALL_S))))
    world_env = int(ws) if ws is not None else 1
    if world_env != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; refusing to run", file=sys.stderr)
        sys.exit(2)
    if args.dry_launch:
        keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
        print(json.dumps({"dry_launch": True, "pid": os.getpid(), **{k: os.environ.get(k) for k in keys}}),
              flush=True)
        r = os.environ.get("RANK", "0")   # test hooks: a rank that hangs / fails
        time.sleep(float(os.environ.get("NKV_DRY_SLEEP_RANK" + r, "0")))
        sys.exit(int(os.environ.get("NKV_DRY_RC_RANK" + r, "0")))
    if world_env > 1:
        # last-resort per-rank wall clock (also under torch.distributed.run, where no launcher of
        # ours is the parent): ends a rank stuck past NKV_RANK_WALL_S with status 124
        from nekstab_next_amd.comm import start_rank_watchdog

        start_rank_watchdog(float(os.environ.get("NKV_RANK_WALL_S", DEFAULT_RANK_WALL_S)),
                            label=f"bench.py rank {os.environ.get('RANK', '?')}")
    if args.collective_probe:
        sys.exit(collective_probe())
    # the contract's ONE JSON line: keep the real stdout for it and send everything else that
    # writes to fd 1 (gloo's C++ connection banner, library prints) to stderr
    sys.stdout.flush()
    args.json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.dry_line:
        run_dry_line(args)
    else:
        run(args)


# ---- one rank ----------------------------------------------------------------------------------

def collective_probe() -> int:
    """``--collective-probe``: the multi-rank plumbing without the solver (CPU tests: gloo ranks).
    Process-group init with the bounded timeout, the ranks' device identities, one SUM all-reduce;
    ``NKV_PROBE_HANG_RANK=r`` makes rank r never join the all-reduce, so its peers' collective
    times out (NKV_COLLECTIVE_TIMEOUT_S) and every rank must end non-zero within the bounds."""
    import torch

    from nekstab_next_amd.comm import init_from_env

    comm = init_from_env(os.environ.get("NKV_BACKEND", "gloo"))
    devs = comm.devices()
    hang = os.environ.get("NKV_PROBE_HANG_RANK")
    if hang is not None and int(hang) == comm.rank:
        print(f"probe rank {comm.rank}: not joining the all-reduce", file=sys.stderr, flush=True)
        time.sleep(3600)
    t = torch.tensor([float(comm.rank + 1)], dtype=torch.float64)
    t0 = time.monotonic()
    try:
        comm.allreduce_(t)
    except Exception as e:  # noqa: BLE001 - the bounded collective's timeout, reported and fatal
        print(f"probe rank {comm.rank}: all-reduce failed after {time.monotonic() - t0:.1f} s: "
              f"{type(e).__name__}: {str(e).splitlines()[0] if str(e) else ''}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)   # no interpreter teardown under a broken group (c10d's threads can abort it: -6)
    if comm.rank == 0:
        print(json.dumps({"collective_probe": True, "world": comm.world, "backend": comm.backend,
                          "sum": float(t.item()), "devices": devs,
                          "distinct_devices": distinct_devices(devs)}), flush=True)
    _leave_group(comm)
    return 0


def _leave_group(comm, keep_rank0: bool = False) -> None:
    """Every rank leaves the process group together, then the process ends without the
    interpreter's teardown: c10d's background threads, torn down by static destructors at exit, were
    seen to abort a gloo rank ("terminate called without an active exception", status -6) after its
    work was done — which a launcher reports as a failed job.  ``keep_rank0``: rank 0 returns (it
    still has host work to do and ends with ``os._exit`` itself)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return
    comm.barrier()
    dist.destroy_process_group()
    if comm.world > 1 and not (keep_rank0 and comm.rank == 0):
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


def distinct_devices(devs) -> bool | None:
    """True iff every rank drove a different GPU (PCI address + host); None without GPUs."""
    keys = [(d.get("host"), d.get("pci")) for d in devs]
    if any(k[1] is None for k in keys):
        return None
    return len(set(keys)) == len(keys)


def krylov_schur_leg(ctx, lay, Q, d_scaled, exact_scaled, seed, k_dim, schur_tgt, warmup=True,
                     operator="config-3 shift-invert / max|mu|"):
    """BASELINE config 3's Krylov–Schur leg at full N (k_dim=128, schur_tgt=4) on the
    shift-invert operator scaled to unit spectral radius (|mu| / max|mu|, the spectrum a
    time-stepper exp(L dt) would present), the reference defaults eigen_tol=1e-6, schur_del=0.1.
    With schur_tgt=4 the first m=128 factorisation already converges (shift-invert separates the
    wanted end of the spectrum: no restart happens); the restart leg runs the same m and schur_tgt
    on ``syn.clustered_spectrum`` (a time-stepper-like cluster below 1), which restarts.  The oracle
    runs both at reduced N with identical restart / mstart / converged-count histories
    (tests/test_gpu_solvers.py::test_config3_krylov_schur_m128_vs_oracle,
    ::test_krylov_schur_m128_real_restart_vs_oracle)."""
    import torch

    from nekstab_next_amd.config import KrylovSchurConfig
    from nekstab_next_amd.krylov_schur import krylov_schur
    from nekstab_next_amd.operators import DiagOperator

    op = DiagOperator(ctx, d_scaled)
    cfg = KrylovSchurConfig(k_dim=k_dim, schur_tgt=schur_tgt)
    if warmup:
        krylov_schur(ctx, op, seed, cfg, Q=Q)       # warm-up (first-touch of small buffers)
    torch.cuda.synchronize(ctx.device)
    ctx.comm.barrier()
    t0 = time.perf_counter()
    res = krylov_schur(ctx, op, seed, cfg, Q=Q)
    torch.cuda.synchronize(ctx.device)
    dt = ctx.comm.max_scalar(time.perf_counter() - t0, device=ctx.device)
    # eigen_tol is absolute (eigensolvers.f90:309-310): besides the wanted end it counts Ritz values
    # near zero whose residual is small only because they are; the accuracy is reported over the
    # relatively converged ones (residual < 1e-6 |mu|), all of them among the exact 4096 largest
    rel = res.residual < 1e-6 * np.abs(res.vals)
    errs = [float(np.min(np.abs(exact_scaled - v)) / abs(v)) for v in res.vals[rel]]
    top = [float(abs(v - e) / abs(e)) for v, e in zip(res.vals[:4], exact_scaled[:4])]
    return {"k_dim": k_dim, "schur_tgt": schur_tgt, "eigen_tol": cfg.eigen_tol,
            "operator": operator, "seconds": round(dt, 4),
            "schur_cnt": int(res.schur_cnt), "mstart_history": list(map(int, res.mstart_history)),
            "cnt_history": list(map(int, res.cnt_history)), "converged": int(res.converged),
            "relatively_converged": int(rel.sum()),
            "ritz_rel_err_vs_exact": max(errs) if errs else None, "top4_rel_err_vs_exact": max(top)}


def run(args):
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

    backend = os.environ.get("NKV_BACKEND", "nccl")
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world_env > max(1, ndev):
        print(f"bench.py: {world_env} RCCL ranks need {world_env} GPUs, {ndev} visible "
              f"(NKV_BACKEND=gloo shares one GPU between ranks)", file=sys.stderr)
        sys.exit(2)
    comm = init_from_env(backend, force_collectives=args.force_collectives)
    rank, world = comm.rank, comm.world
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, ndev)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    devices = comm.devices(dev)      # per-rank GPU identity (gathered at world > 1)

    glay = box3d_layout(args.E)
    lay = glay.shard(rank, world)
    m = args.m
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, comm=comm, max_cols=m + 1, device=dev)
    d, exact = syn.laplacian_shift_invert(lay)
    op = DiagOperator(ctx, d)
    rho = float(np.abs(exact[0]))
    d_scaled = d / rho
    del d
    seed = ctx.vector()
    seed.fill_hash(11)
    Q = ctx.basis(m + 1)
    Hd = HessenbergDev(ctx, m)
    f = ctx.vector()

    def one_step():
        prepare_seed(seed, Q[0])
        arnoldi_factorization(ctx, op, Q, Hd, 1, m, f=f, mode=args.mode)
        H = Hd.download()
        vals, vecs = lapack.eig(H[:m, :m])
        res = np.abs(H[m, m - 1] * vecs[m - 1, :])
        return vals, res

    for _ in range(args.warmup):
        one_step()
    timer = PhaseTimer(dev)
    ctx.timer = timer
    comm.timer = timer
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
    comm.timer = None
    phases = timer.summary()
    last_step_ms = (sum(timer.last_ms(k) for k in ("block_dot2", "dcgs2_update"))
                    if args.mode in ("dcgs2", "mgs2-lagged") else None)
    ctx.check_nan()

    # Krylov–Schur restart on the final factorisation (outside the timed region; reported beside
    # the metric): the kept-column rotation the solver runs, and the reference's
    # full k-column rotation priced against the fp64 matrix peak.
    restart = None
    if not args.no_restart:
        rt = PhaseTimer(dev)
        ctx.timer = rt
        # the shift-invert spectrum is not inside the unit disc (every |mu| >= 1 - schur_del would be
        # kept); H is divided by its spectral radius as a time-stepper's exp(L dt) spectrum would be —
        # same Schur vectors, the selection rule then keeps the leading cluster + nev + 4
        H = Hd.download()
        H /= np.max(np.abs(vals))
        t1 = time.perf_counter()
        mstart, _sel = schur_condensation(ctx, H, Q, m, KrylovSchurConfig(k_dim=m, schur_tgt=4))
        torch.cuda.synchronize(dev)
        cond_ms = (time.perf_counter() - t1) * 1e3
        V = torch.as_tensor(np.linalg.qr(np.random.default_rng(5).standard_normal((m, m)))[0].ravel(order="F")
                            .copy()).to(dev)
        # the solver's kept-column rotation above is the process's first launch of that kernel
        # (+1.4 ms one-time cost at 6 kept columns, profiles/r05af_probe_rotate.log): the same shape
        # again, on the first mstart-1 columns of the random V, gives the kernel's steady rate
        n_kept = int(mstart) - 1
        for _ in range(2):
            rt.begin("rotate_kept_steady")
            ctx.call("nkv_rotate_cols", Q.ptr, m, V.data_ptr(), m, n_kept, ctx.stream)
            rt.end("rotate_kept_steady", 8.0 * lay.N * (m + n_kept))
        for _ in range(2):
            rt.begin("rotate_full")
            ctx.call("nkv_rotate", Q.ptr, m, V.data_ptr(), m, ctx.stream)
            rt.end("rotate_full", 16.0 * lay.N * m)
        # the restart leg's kept-column count at BASELINE size (25 of 128: mstart_history [26] of
        # krylov_schur_restart_leg, checked below when that leg runs) on the 17-64-kept MFMA rotation
        # (VERDICT r5 item 2); timed here so that the PMC passes (--no-ks) see it too
        n_w = ROT_WIDE_KEPT if m == 128 else min(m, max(17, (m * 25) // 128))
        for _ in range(3):
            rt.begin("rotate_wide")
            ctx.call("nkv_rotate_cols", Q.ptr, m, V.data_ptr(), m, n_w, ctx.stream)
            rt.end("rotate_wide", 8.0 * lay.N * (m + n_w))
        ctx.timer = None
        rp = rt.summary()
        kept, steady, full = rp["rotate"], rp["rotate_kept_steady"], rp["rotate_full"]
        full_tf = 2.0 * lay.N * m * m / (full["avg_ms"] * 1e-3) / 1e12
        restart = {
            "note": ("one condensation of the timed run's final factorisation with H divided by its spectral "
                     "radius (synthetic: the raw shift-invert spectrum lies outside the unit disc, so the "
                     "selection rule would keep every column); rotate_kept is the solver's call (the process's "
                     "first launch of that kernel), rotate_kept_steady the same shape repeated; rotate_full is "
                     "the reference's full k-column Q V on a random orthogonal V"),
            "mstart": int(mstart), "condensation_wall_ms": round(cond_ms, 2),
            "rotate_kept_ms": round(kept["avg_ms"], 3), "rotate_kept_gbs": round(kept["gbps"], 1),
            "rotate_kept_frac_hbm": round(kept["gbps"] / HBM_PEAK_GBS, 4),
            "rotate_kept_steady_ms": round(steady["avg_ms"], 3),
            "rotate_kept_steady_frac_hbm": round(steady["gbps"] / HBM_PEAK_GBS, 4),
            "rotate_full_ms": round(full["avg_ms"], 3), "rotate_full_tflops": round(full_tf, 2),
            "rotate_full_frac_fp64": round(full_tf / FP64_PEAK_TFLOPS, 4),
        }
        wp = rp["rotate_wide"]
        restart.update({"rotate_wide_kept": n_w, "rotate_wide_ms": round(wp["avg_ms"], 3),
                        "rotate_wide_gbs": round(wp["gbps"], 1),
                        "rotate_wide_frac_hbm": round(wp["gbps"] / HBM_PEAK_GBS, 4),
                        "rotate_wide_tflops": round(2.0 * lay.N * m * n_w / (wp["avg_ms"] * 1e-3) / 1e12, 2)})
    ks_leg = ks_restart = None
    if not args.no_ks:
        ks_leg = krylov_schur_leg(ctx, lay, Q, d_scaled, exact / rho, seed, m, 4)
        del d_scaled
        # the same m and schur_tgt on a time-stepper-like clustered spectrum: real m-column restarts
        d_cl, exact_cl = syn.clustered_spectrum(lay)
        ks_restart = krylov_schur_leg(ctx, lay, Q, d_cl, exact_cl, seed, m, 4, warmup=False,
                                      operator="clustered: 1 - 0.002 (k - 1/2), k <= 400, over U[0, 0.2]")
        del d_cl
        if restart is not None and ks_restart["mstart_history"]:
            restart["rotate_wide_kept_is_restart_legs"] = int(ks_restart["mstart_history"][0]) - 1 == restart["rotate_wide_kept"]
    else:
        del d_scaled

    out = bench_line(args, comm, glay, lay, m, elapsed, phases, last_step_ms, vals, res, exact, restart, ks_leg,
                     ks_restart, devices, dev)
    finish(args, comm, out, m)


def bench_line(args, comm, glay, lay, m, elapsed, phases, last_step_ms, vals, res, exact, restart, ks_leg,
               ks_restart, devices, dev):
    """The ONE JSON line from the measurements (rank 0's copy is printed; the *_over_ranks figures are
    collectives, so every rank calls this).  The CPU lines are attached by ``finish`` after every
    rank has left the process group."""
    world = comm.world
    ms_per_step = elapsed / args.steps * 1e3
    nv_g = glay.pts_v * glay.nelgv
    exec_b = executed_bytes(glay.N, glay.N_w, nv_g, m, args.mode)
    value = exec_b * args.steps / elapsed / 1e9
    survey_b = survey_model_bytes(glay.N, glay.N_w, nv_g, m)
    # SURVEY.md 8(d)'s 4-pass model as a dimensionless time ratio (no GB/s from a foreign byte model)
    survey_time_ratio = (survey_b / (HBM_PEAK_GBS * 1e9)) / (elapsed / args.steps)

    # SURVEY.md §8(d) headline: Gram–Schmidt bytes over Gram–Schmidt time only (matvec, host LAPACK
    # and launch gaps excluded; kernel-bracketed HIP events, this rank), and the last step alone
    gs_fams = ("block_dot", "update_dot", "block_update", "finish", "block_dot2", "dcgs2_update")
    gs_ms = sum(phases[k]["total_ms"] for k in gs_fams if k in phases) / args.steps
    ar = phases.get("allreduce")
    ar_ms = (ar["total_ms"] / args.steps) if ar else 0.0
    gs_exec = sum(phases[k]["avg_bytes"] * phases[k]["launches"] for k in gs_fams if k in phases) / args.steps
    survey_gs = survey_model_bytes(lay.N, lay.N_w, lay.n_v, m) - m * 8.0 * 3 * lay.N
    last_b = 8.0 * ((m - 1) * lay.N_w + 2 * lay.N_w + lay.n_v) + 8.0 * ((m - 1) * lay.N + 4 * lay.N)
    gs_min, gs_max = comm.min_scalar(gs_ms, device=dev), comm.max_scalar(gs_ms, device=dev)
    ar_min, ar_max = comm.min_scalar(ar_ms, device=dev), comm.max_scalar(ar_ms, device=dev)
    gs = {"gs_ms_per_factorisation": round(gs_ms, 2),
          "gs_ms_per_factorisation_min_over_ranks": round(gs_min, 2),
          "gs_ms_per_factorisation_max_over_ranks": round(gs_max, 2),
          "allreduce_ms_per_factorisation": round(ar_ms, 3),
          "allreduce_ms_per_factorisation_min_over_ranks": round(ar_min, 3),
          "allreduce_ms_per_factorisation_max_over_ranks": round(ar_max, 3),
          "allreduces_per_factorisation": (ar["launches"] // args.steps) if ar else 0,
          "gs_incl_allreduce_ms": round(gs_ms + ar_ms, 2),
          "executed_gs_gbs": round(gs_exec / (gs_ms * 1e-3) / 1e9, 1) if gs_ms > 0 else None,
          "survey_model_time_ratio": (round((survey_gs / (HBM_PEAK_GBS * 1e9)) / (gs_ms * 1e-3), 3)
                                      if gs_ms > 0 else None),
          "last_step_ms": None if last_step_ms is None else round(last_step_ms, 3),
          "last_step_executed_gbs": (None if last_step_ms is None else
                                     round(last_b / (last_step_ms * 1e-3) / 1e9, 1)),
          "note": ("rank-0 shard unless *_over_ranks; events on the launch stream; allreduce = events around "
                   "torch.distributed.all_reduce of the step's partial vector (0 at world 1); every GB/s is "
                   "executed bytes / measured time; survey_model_time_ratio = (SURVEY.md 8(d) 4-pass CGS2 "
                   "bytes at the 8 TB/s peak) / measured Gram-Schmidt time")}

    # Ritz accuracy vs the exact spectrum of the synthetic operator
    # (exact spectrum: the 4096 largest |mu|; a converged Ritz value is matched to the nearest one)
    conv = res < 1e-6
    errs = [float(np.min(np.abs(exact - v)) / abs(v)) for v in vals[conv]] if conv.any() else []
    ritz_err = max(errs) if errs else None
    top_err = float(np.max(np.abs(vals[:8] - exact[:8]) / np.abs(exact[:8])))

    # dominant kernel family (rank-local launches; bytes are this rank's shard)
    dom = max(("block_dot", "update_dot", "block_update", "block_dot2", "dcgs2_update"),
              key=lambda k: phases.get(k, {}).get("total_ms", 0.0))
    # the native drivers launch inside one library call and mgs2 runs per-column dots: no
    # kernel-family events in those modes (their kernels are in a rocprof trace), only `value`
    ph = phases.get(dom, {"gbps": 0.0, "avg_ms": 0.0, "avg_bytes": 0.0, "launches": 0})
    achieved = ph["gbps"]
    traffic, tsrc = find_traffic(dom, lay.nelv, m)

    out = {
        "metric": "Arnoldi-step GB/s (achieved HBM) + Ritz-value rel-err, N=1e8 m=128",
        "value": round(value, 2),
        "unit": "GB/s",
        "n_gpus": world,
        "world": world,
        "backend": comm.backend if world > 1 or args.force_collectives else None,
        "devices": devices,
        "distinct_devices": distinct_devices(devices),
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "survey_model_time_ratio": round(survey_time_ratio, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (diagonalised shift-invert Laplacian, hashed seed, GLL x J_e weights)",
        "config": {
            "workload": f"config3: m-step Arnoldi ({args.mode.upper()}) + Ritz extraction, shift-invert Laplacian",
            "N": glay.N, "N_w": glay.N_w, "E": args.E, "layout": "3D lx1=8 lx2=6 {vx,vy,vz,t}+pr",
            "m": m, "mode": args.mode,
            "parallelism": (f"element-shard x{world} + " + ("RCCL" if comm.backend == "nccl" else str(comm.backend))
                            + " allreduce") if world > 1 else "single GPU",
        },
        "roofline": None if dom not in phases else {
            "bound": "hbm",
            "kernel": dom,
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": tsrc,
            "launch": ("one entry-point call per Arnoldi step (nkv_dcgs2_update: NKV_DC_ROUNDS row-band "
                       "dispatches; events span all of them)" if dom == "dcgs2_update" else "one entry-point call"),
            "avg_launch_ms": round(ph["avg_ms"], 4),
            "avg_bytes_per_launch": ph["avg_bytes"],
            "launches": ph["launches"],
            "scope": "one GPU (the only rank)" if world == 1 else
                     f"rank 0's shard on its own GPU (1/{world} of N); peak is one GPU's HBM",
            # a rank's vector that fits the 256 MiB Infinity Cache (MALL) is partly re-read from
            # it (the vector one kernel writes is read by the next): not pure HBM traffic
            "infinity_cache": (None if 8.0 * lay.ld >= 256 * 2 ** 20 else
                               f"rank vectors of {8.0 * lay.ld / 2 ** 20:.0f} MiB fit the 256 MiB Infinity "
                               "Cache: part of the achieved rate is MALL hits, not HBM"),
        },
        "phases": {k: {kk: (round(vv, 4) if isinstance(vv, float) else vv) for kk, vv in v.items()}
                   for k, v in phases.items()},
        "gram_schmidt": gs,
        "ritz_rel_err": ritz_err,
        "ritz_top8_rel_err": top_err,
        "ritz_converged": int(conv.sum()),
        "ritz_top8": [[float(v.real), float(v.imag)] for v in vals[:8]],
        "cpu_baseline": None,
        "cpu_baseline_1core": None,
        "cpu_optimised": None,
        "restart": restart,
        "krylov_schur_leg": ks_leg,
        "krylov_schur_restart_leg": ks_restart,
    }
    return out


def finish(args, comm, out, m) -> None:
    """Every rank leaves the process group together; the ranks other than 0 end there.  Rank 0 then
    times the CPU lines (unless --no-cpu) — at every world size, with no peer left waiting in a
    collective — and prints the ONE JSON line."""
    rank, world = comm.rank, comm.world
    _leave_group(comm, keep_rank0=True)
    if rank == 0:
        if not args.no_cpu:
            out.update(host_baselines(args, m, out["ms_per_step"]))
        print(json.dumps(out), file=args.json_out, flush=True)
    args.json_out.flush()
    if world > 1:
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


def run_dry_line(args) -> None:
    """``--dry-line``: the multi-rank line assembly without a GPU (CPU test of the N > 1 contract).
    Every rank joins a gloo group and contributes fabricated, clearly labelled measurements of the
    right shape (phases of the DCGS2 kernel families, step time, Ritz values); the line is built by
    the same ``bench_line`` and finished by the same ``finish`` (CPU lines on rank 0 after the group
    is left) as a real run, so its keys are the real line's keys."""
    from nekstab_next_amd.comm import init_from_env
    from nekstab_next_amd.layout import box3d_layout

    comm = init_from_env("gloo")
    devices = comm.devices()
    glay = box3d_layout(args.E)
    lay = glay.shard(comm.rank, comm.world)
    m = args.m
    n1 = 8.0 * ((m - 1) * lay.N_w + 2 * lay.N_w + lay.n_v)
    n2 = 8.0 * ((m - 1) * lay.N + 4 * lay.N)
    phases = {"block_dot2": dict(launches=m * args.steps, total_ms=1.0 * m * args.steps, avg_ms=1.0, avg_bytes=n1,
                                 gbps=n1 / 1e-3 / 1e9),
              "dcgs2_update": dict(launches=m * args.steps, total_ms=1.1 * m * args.steps, avg_ms=1.1, avg_bytes=n2,
                                   gbps=n2 / 1.1e-3 / 1e9)}
    if comm.world > 1:
        phases["allreduce"] = dict(launches=m * args.steps, total_ms=0.01 * m * args.steps, avg_ms=0.01,
                                   avg_bytes=16.0 * m, gbps=0.0)
    exact = np.linspace(2.0, 1.0, max(m, 8))
    vals = exact.astype(complex)
    res = np.full(vals.shape, 1e-9)
    elapsed = comm.max_scalar(2.5 * m * 1e-3 * args.steps)
    out = bench_line(args, comm, glay, lay, m, elapsed, phases, 2.1, vals, res, exact, None, None, None, devices, None)
    out["dry_line"] = "fabricated measurements (CPU rehearsal of the line's shape); not a result"
    finish(args, comm, out, m)


if __name__ == "__main__":
    main()
