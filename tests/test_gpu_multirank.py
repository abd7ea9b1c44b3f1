"""Sharded (world_size 2) GPU path on ONE MI355X: two ranks share the device and exchange partial
dots through gloo (RCCL cannot place two ranks on one GPU; on an 8-GPU node the same code runs over
RCCL/xGMI).  Sharded Krylov–Schur must reproduce the single-rank result: identical restart
trajectory, Ritz values to 1e-12 (SURVEY.md §8(e) gate) — and the oracle's unsharded Krylov–Schur on
the same problems (restart trajectory identical, Ritz values to 1e-10)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import match_ritz, ritz_compare_set

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ks(world_rank_pair, out, port, E_box=96, E_cyl=400, mode="dcgs2", seed_mode="normalize",
            nonorth="mgs2-icwy"):
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur
        from nekstab_next_amd.layout import box3d_layout, cylinder_layout
        from nekstab_next_amd.operators import DiagOperator, Rot2Operator
        from nekstab_next_amd.vector import NekContext

        res = {}
        comm = Comm()
        lay = box3d_layout(E_box).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=comm, max_cols=48)
        d, exact = syn.laplacian_shift_invert(lay)
        if seed_mode != "normalize":   # Q(1) = A s: scaled so that ||Q(1)|| = O(1) (as bench.py's KS leg)
            d = d / abs(exact[0])
        seed = ctx.vector()
        seed.fill_hash(11)
        kw = dict(seed_mode=seed_mode, nonorth_mode=nonorth)
        r = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=32, schur_tgt=4, mode=mode, **kw))
        res["lap"] = (r.vals, r.residual, r.mstart_history, r.schur_cnt, r.H)
        lay2 = cylinder_layout(E_cyl).shard(rank, world)
        ctx2 = NekContext(lay2, weights=syn.mass_weights(lay2), comm=comm, max_cols=48)
        c, s, dr, _ = syn.rot2_operator(lay2)
        seed2 = ctx2.vector()
        seed2.fill_hash(5)
        r2 = krylov_schur(ctx2, Rot2Operator(ctx2, c, s, dr), seed2,
                          KrylovSchurConfig(k_dim=24, schur_tgt=2, mode=mode, **kw))
        res["rot"] = (r2.vals, r2.residual, r2.mstart_history, r2.schur_cnt, r2.H)
        out[(world, rank)] = res
    finally:
        if world > 1:
            dist.destroy_process_group()



@pytest.mark.parametrize("nonorth", ["mgs2-lagged", "mgs2-icwy"])
def test_noise_seed_ranks_match_one_rank(gpu, nonorth):
    """The in-tree default seed (Q(1) = A s/||s|| unnormalised, a non-orthonormal basis) on 3 gloo
    ranks with ragged shards against one rank: "mgs2-lagged" (host algebra replicated on the
    all-reduced multi-dot, Gram rows rebuilt through all-reduced dots) and "mgs2-icwy" give the same
    restart trajectory on every rank, H identical on every rank, and Ritz values within 1e-10 of the
    one-rank run: MGS on the non-orthonormal basis amplifies the partial-sum grouping's rounding
    beyond the orthonormal path's 1e-12 (measured 8e-12 for "mgs2-lagged", 4e-11 for ICWY)."""
    world, E_box, E_cyl = 3, 97, 401
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    args = (E_box, E_cyl, "dcgs2", "noise", nonorth)
    p = ctx.Process(target=_run_ks, args=((0, 1), out, _free_port(), *args))
    p.start()
    p.join()
    assert p.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_ks, args=((r, world), out, port, *args)) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    for key in ("lap", "rot"):
        v1, r1, m1, c1, H1 = out[(1, 0)][key]
        for rank in range(world):
            v2, r2, m2, c2, H2 = out[(world, rank)][key]
            assert m2 == m1 and c2 == c1, (key, rank)
            sel = sorted(set(np.nonzero(r1 < 1e-6)[0].tolist() + list(range(8))))
            assert np.max(np.abs(v2[sel] - v1[sel]) / np.abs(v1[sel])) < 1e-10
            np.testing.assert_array_equal(out[(world, 0)][key][4], H2)

@pytest.mark.parametrize("world,E_box,E_cyl,mode", [(2, 96, 400, "dcgs2"), (3, 97, 401, "dcgs2"), (8, 101, 403, "dcgs2"),
                                                   (2, 96, 400, "dcgs2-native"), (3, 97, 401, "cgs2-native")])
def test_ranks_match_one_rank(gpu, world, E_box, E_cyl, mode):
    """Krylov–Schur on `world` gloo ranks sharing the GPU (the sharded HIP path, one shard per
    process) reproduces the one-rank run; (3, 97, 401) gives ragged shards (32/32/33 and
    133/134/134 elements); (8, 101, 403) rehearses the 8-way split of the driver's 8-GPU run with
    ragged shards (12/13 and 50/51 elements); the "-native" modes run the one-call library drivers,
    whose all-reduce callback then goes through gloo between the processes."""
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_ks, args=((0, 1), out, _free_port(), E_box, E_cyl, mode))
    p.start()
    p.join()
    assert p.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_ks, args=((r, world), out, port, E_box, E_cyl, mode)) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    for key in ("lap", "rot"):
        v1, r1, m1, c1, H1 = out[(1, 0)][key]
        for rank in range(world):
            v2, r2, m2, c2, H2 = out[(world, rank)][key]
            assert m2 == m1 and c2 == c1
            conv = r1 < 1e-6
            sel = np.nonzero(conv)[0].tolist() + list(range(8))
            sel = sorted(set(sel))
            assert np.max(np.abs(v2[sel] - v1[sel]) / np.abs(v1[sel])) < 1e-12
            np.testing.assert_array_equal(out[(world, 0)][key][4], H2)  # identical H on every rank
    # and against the oracle (the reference's MGS2 Krylov–Schur restated on the CPU, unsharded):
    # restart trajectory identical, Ritz values of the comparison set to 1e-10
    ref = _oracle_ks(E_box, E_cyl)
    for key in ("lap", "rot"):
        v2, _r2, m2, c2, _H2 = out[(world, 0)][key]
        assert m2 == ref[key]["mstart"] and c2 == ref[key]["schur_cnt"], (key, m2, ref[key]["mstart"])
        sel = ritz_compare_set(ref[key]["vals"], ref[key]["residual"], 1e-6)
        got = match_ritz(ref[key]["vals"][sel], v2)
        assert np.max(np.abs(got - ref[key]["vals"][sel]) / np.abs(ref[key]["vals"][sel])) <= 1e-10


_ORACLE = {}


def _oracle_ks(E_box, E_cyl):
    """The oracle's Krylov–Schur on the unsharded problems of _run_ks (same operators, seeds,
    k_dim and schur_tgt)."""
    if (E_box, E_cyl) in _ORACLE:
        return _ORACLE[(E_box, E_cyl)]
    import oracle as orc
    from helpers import olayout, oracle_diag_matvec, oracle_rot2_matvec
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout, cylinder_layout

    res = {}
    orc.set_threads(8)
    try:
        lay = box3d_layout(E_box)
        L, w = olayout(lay), syn.mass_weights(lay)
        d, _ = syn.laplacian_shift_invert(lay)
        q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
        res["lap"] = orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 32, 4)
        lay2 = cylinder_layout(E_cyl)
        L2, w2 = olayout(lay2), syn.mass_weights(lay2)
        c, s_, dr, _ = syn.rot2_operator(lay2)
        q2 = orc.prepare_seed(L2, w2, syn.to_reference_order(lay2, syn.hash_vector(lay2, 5)))
        res["rot"] = orc.krylov_schur(L2, w2, oracle_rot2_matvec(lay2, c, s_, dr), q2, 24, 2)
    finally:
        orc.set_threads(1)
    _ORACLE[(E_box, E_cyl)] = res
    return res


_RCCL_SCRIPT = r'''
import os, sys
sys.path.insert(0, sys.argv[1])
import numpy as np, torch, torch.distributed as dist
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:" + sys.argv[2], rank=0, world_size=1,
                        device_id=torch.device("cuda", 0))
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.comm import Comm
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.krylov_schur import krylov_schur
from nekstab_next_amd.layout import box3d_layout
from nekstab_next_amd.operators import DiagOperator
from nekstab_next_amd.vector import NekContext
out = {}
for forced in (False, True):
    comm = Comm(force_collectives=forced)   # forced: world 1, every partial through RCCL all_reduce
    assert comm.backend == "nccl"
    lay = box3d_layout(96)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=comm, max_cols=48)
    d, _ = syn.laplacian_shift_invert(lay)
    seed = ctx.vector()
    seed.fill_hash(11)
    for mode in ("dcgs2", "cgs2", "dcgs2-native", "cgs2-native"):
        r = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=32, schur_tgt=4, mode=mode))
        out[(forced, mode)] = (r.vals, r.H, r.mstart_history)
    assert comm.max_scalar(3.0, device=ctx.device) == 3.0
for mode in ("dcgs2", "cgs2", "dcgs2-native", "cgs2-native"):
    a, b = out[(False, mode)], out[(True, mode)]
    np.testing.assert_array_equal(a[0], b[0]); np.testing.assert_array_equal(a[1], b[1]); assert a[2] == b[2]
# the library-driven factorisation (all-reduce through the callback when forced) equals the Python-driven one
for forced in (False, True):
    for m1, m2 in (("dcgs2", "dcgs2-native"), ("cgs2", "cgs2-native")):
        a, b = out[(forced, m1)], out[(forced, m2)]
        np.testing.assert_array_equal(a[0], b[0]); np.testing.assert_array_equal(a[1], b[1]); assert a[2] == b[2]
dist.destroy_process_group()
print("RCCL path ok")
'''


def test_rccl_collective_path_single_gpu(gpu, tmp_path):
    """The nccl (= RCCL) backend on the real device: a world-1 process group with the collective
    code path forced on, so every partial dot goes through dist.all_reduce on the compute stream
    between the HIP kernels (the 8-GPU path minus the peers).  Results must be bit-identical to
    the no-collective run.  Runs in a child process so the test process holds no process group."""
    import subprocess

    script = tmp_path / "rccl_path.py"
    script.write_text(_RCCL_SCRIPT)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, str(script), ROOT, str(_free_port())], capture_output=True, text=True,
                       timeout=300, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    assert "RCCL path ok" in p.stdout


def _run_time(world_rank_pair, out, port):
    """Arnoldi (DCGS2 and CGS2, m=20) with the time slot inside k_dot on a sharded layout: the
    replicated scalar enters the dots on rank 0 only and follows every update on every rank."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.arnoldi import HessenbergDev, arnoldi_factorization
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.layout import NekLayout
        from nekstab_next_amd.operators import DiagOperator
        from nekstab_next_amd.vector import NekContext, k_normalize

        lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=101).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=Comm(), max_cols=24, time_in_dot=True)
        d, _ = syn.diag_spectrum(lay)
        op = DiagOperator(ctx, d, time_scale=0.7)
        res = {}
        for mode in ("dcgs2", "cgs2"):
            Q = ctx.basis(21)
            Q[0].fill_hash(5)
            Q[0].time = 0.3
            k_normalize(Q[0])
            Hd = HessenbergDev(ctx, 20)
            arnoldi_factorization(ctx, op, Q, Hd, 1, 20, mode=mode)
            res[mode] = (Hd.download(), Q.storage[:, lay.time_offset].cpu().numpy())
        out[(world, rank)] = res
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_ranks_match_one_rank_with_time_in_dot(gpu):
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_time, args=((0, 1), out, _free_port()))
    p.start()
    p.join()
    assert p.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_time, args=((r, 3), out, port)) for r in range(3)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    for mode in ("dcgs2", "cgs2"):
        H1, t1 = out[(1, 0)][mode]
        for rank in range(3):
            H, t = out[(3, rank)][mode]
            assert np.max(np.abs(H - H1)) <= 1e-12 * np.max(np.abs(H1)), (mode, rank)
            np.testing.assert_allclose(t, t1, rtol=1e-11, atol=1e-15)   # replicated time, identical on every rank
            assert np.any(np.abs(t) > 1e-3)


def _run_ckpt(world_rank_pair, out, port, directory, action, E):
    """One rank of a sharded checkpoint/restart run (config-1 diagonal operator, k_dim=16):
    ``write``: the first factorisation with the ifres hook (one KRY file per rank, HES on rank 0);
    ``resume``: load_restart at mstart=9 and Krylov–Schur to schur_tgt=5; ``full``: uninterrupted."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.checkpoint import ArnoldiCheckpoint, load_restart
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur
        from nekstab_next_amd.layout import NekLayout
        from nekstab_next_amd.operators import DiagOperator
        from nekstab_next_amd.vector import NekContext

        lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=E).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=Comm(), max_cols=32)
        d, _ = syn.diag_spectrum(lay)
        op = DiagOperator(ctx, d)
        cfg = KrylovSchurConfig(k_dim=16, schur_tgt=5)
        if action == "write":
            seed = ctx.vector()
            seed.fill_hash(11)
            krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=16, schur_tgt=0),
                         on_step=ArnoldiCheckpoint(ctx, directory, session="cyl", evop="d"))
        else:
            if action == "resume":
                Q, H = load_restart(ctx, directory, "cyl", 9, 16)
                r = krylov_schur(ctx, op, None, cfg, Q=Q, start=(9, H))
            else:
                seed = ctx.vector()
                seed.fill_hash(11)
                r = krylov_schur(ctx, op, seed, cfg)
            out[(action, world, rank)] = (r.vals, r.residual, r.mstart_history, r.schur_cnt)
    finally:
        if world > 1:
            dist.destroy_process_group()


def _spawn(world, *args):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_run_ckpt, args=((r, world), args[0], port, *args[1:])) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0


@pytest.mark.parametrize("w_write,w_resume", [(3, 1), (1, 2)])
def test_sharded_checkpoint_resumes_at_another_world_size(gpu, tmp_path, w_write, w_resume):
    """ifres checkpoint written by `w_write` ranks (a Nek5000 multi-file KRY set, one file per rank,
    HES on rank 0; ragged shards 100/100/101 of E=301) and resumed by `w_resume` ranks, as a
    Nek5000 restart reads a field-file set written by any number of ranks (the element map places
    every element; core/IO.f90:12-73 through load_fld).  The resumed run follows the uninterrupted
    one-rank run: restart count and mstart sequence identical, Ritz values of the comparison set
    to 1e-10.  The oracle's independent #std reader (oracle/nekio.py) reads the written set into
    the same Krylov vectors as the one-rank checkpoint's (1e-12 of max |q|)."""
    import nekio

    E = 301
    out = mp.Manager().dict()
    ref_dir, dir_w = str(tmp_path / "one"), str(tmp_path / "w")
    _spawn(1, out, ref_dir, "write", E)
    _spawn(1, out, ref_dir, "full", E)
    _spawn(w_write, out, dir_w, "write", E)
    _spawn(w_resume, out, dir_w, "resume", E)
    assert len([f for f in os.listdir(dir_w) if f.startswith("KRYcyl") and f.endswith(".f00005")]) == w_write
    v1, r1, m1, c1 = out[("full", 1, 0)]
    conv = r1 < 1e-6
    sel = sorted(set(np.nonzero(conv)[0].tolist() + list(range(8))))
    for rank in range(w_resume):
        v2, r2, m2, c2 = out[("resume", w_resume, rank)]
        assert m2 == m1 and c2 == c1
        assert np.max(np.abs(v2[sel] - v1[sel]) / np.abs(v1[sel])) < 1e-10
    g = nekio.Geom(2, 6, 4, E)
    H_ref, Q_ref = nekio.load_restart(ref_dir, "cyl", g, 9, 16, nfiles=1)
    H_w, Q_w = nekio.load_restart(dir_w, "cyl", g, 9, 16, nfiles=w_write)
    assert Q_w.shape == Q_ref.shape
    assert np.max(np.abs(Q_w - Q_ref)) < 1e-12 * np.max(np.abs(Q_ref))
    assert np.max(np.abs(H_w - H_ref)) < 1e-12 * np.max(np.abs(H_ref))


def _run_next(world_rank_pair, out, port, tmpdir):
    """Round-3 paths on `world` gloo ranks: svds (delayed re-orthogonalisation of two bases), GMRES
    on one continuous DCGS2 factorisation, and the wave-maker chain through multi-file mode sets."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import fld
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import GmresConfig, KrylovSchurConfig
        from nekstab_next_amd.gmres import ts_gmres
        from nekstab_next_amd.krylov_schur import krylov_schur, outpost_ks, prepare_seed
        from nekstab_next_amd.layout import NekLayout, box3d_layout, cylinder_layout
        from nekstab_next_amd.lightkrylov import svds
        from nekstab_next_amd.operators import DiagOperator, RankTwoPerturbed, ShiftedOperator
        from nekstab_next_amd.sensitivity import velocity_layout, wave_maker
        from nekstab_next_amd.vector import NekContext

        comm = Comm()
        res = {}

        def pert(ctx, base, scale, sigma):
            vs = []
            for s5 in (21, 22, 23, 24):
                v = ctx.vector()
                v.fill_hash(s5)
                v.scal(scale)
                vs.append(v)
            return RankTwoPerturbed(base, *vs, sigma=sigma)

        lay = NekLayout(ldim=2, lx1=4, lx2=2, nelgv=41, ifpo=False).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=comm, max_cols=48)
        d, _ = syn.diag_spectrum(lay)
        A = pert(ctx, DiagOperator(ctx, d), 0.05, 3.0)
        k = 30
        U, V = ctx.basis(k + 1), ctx.basis(k + 1)
        seed = ctx.vector()
        seed.fill_hash(7)
        prepare_seed(seed, V[0])
        r = svds(ctx, A, U, V, nev=3, tolerance=1e-8, mode="dcgs2")
        res["svds"] = (r.sigma, r.C)

        lay2 = cylinder_layout(203).shard(rank, world)
        ctx2 = NekContext(lay2, weights=syn.mass_weights(lay2), comm=comm, max_cols=48)
        d2, _ = syn.diag_spectrum(lay2)
        op = ShiftedOperator(DiagOperator(ctx2, d2), -1.0)
        rhs, sol, probe = ctx2.vector(), ctx2.vector(), ctx2.vector()
        rhs.fill_hash(3)
        probe.fill_hash(4)
        info = ts_gmres(ctx2, op, rhs, sol, GmresConfig(k_dim=12, maxiter=20, tol=1e-14, mode="dcgs2"))
        res["gmres"] = (info.inner_residuals, info.outer_residuals, ctx2.dot(sol, probe, False))
        sol_n = ctx2.vector()   # the one-call library cycle, its all-reduce through the callback
        info_n = ts_gmres(ctx2, op, rhs, sol_n, GmresConfig(k_dim=12, maxiter=20, tol=1e-14, mode="dcgs2-native"))
        res["gmres_native_equal"] = (info_n.inner_residuals == info.inner_residuals
                                     and bool(torch.equal(sol_n.storage, sol.storage)))
        # Newton for a periodic orbit: the legacy dispatcher's bordered mode-2.1 map, time in k_dot
        from nekstab_next_amd.operators import LegacyMatvec

        ctx4 = NekContext(lay2, weights=syn.mass_weights(lay2), comm=comm, max_cols=16, time_in_dot=True)
        b_fc, b_ic, rhs4, sol4, probe4 = (ctx4.vector() for _ in range(5))
        for v, sd in ((b_fc, 31), (b_ic, 32), (rhs4, 3), (probe4, 4)):
            v.fill_hash(sd)
        b_fc.scal(0.5)
        b_ic.scal(0.5)
        rhs4.time = 0.25
        A4 = LegacyMatvec(2.1, DiagOperator(ctx4, d2), b_fc=b_fc, b_ic=b_ic)
        info4 = ts_gmres(ctx4, A4, rhs4, sol4, GmresConfig(k_dim=8, maxiter=12, tol=1e-12))
        res["upo"] = (info4.inner_residuals, info4.outer_residuals, ctx4.dot(sol4, probe4, False), sol4.time)

        lay3 = box3d_layout(23).shard(rank, world)
        ctx3 = NekContext(lay3, weights=syn.mass_weights(lay3), comm=comm, max_cols=32)
        d3, _ = syn.diag_spectrum(lay3)
        A3 = pert(ctx3, DiagOperator(ctx3, d3), 1e-3, 50.0)
        seed3 = ctx3.vector()
        seed3.fill_hash(11)
        cfg = KrylovSchurConfig(k_dim=24, schur_tgt=2)
        rd = krylov_schur(ctx3, A3, seed3, cfg)
        ra = krylov_schur(ctx3, A3, seed3, cfg, transpose=True)
        d_ = os.path.join(tmpdir, f"w{world}")
        outpost_ks(ctx3, rd, d_, evop="d", maxmodes=1, session="mr", orthonormality=False)
        outpost_ks(ctx3, ra, d_, evop="a", maxmodes=1, session="mr", orthonormality=False)
        vlay = velocity_layout(box3d_layout(23)).shard(rank, world)
        vctx = NekContext(vlay, weights=syn.mass_weights(vlay), comm=comm, max_cols=4)
        wm = wave_maker(vctx, d_, session="mr", d_num=1, a_num=1)
        comm.barrier()
        g = np.zeros((23, vlay.pts_v))
        for f in fld.read_fld_set(d_, "wm_", "mr", 1):   # every rank's file: the global field
            g[f.emap - 1] = f.fields["t"]
        res["wm"] = (wm["inner_product"], g)
        out[(world, rank)] = res
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_round3_paths_sharded_match_one_rank(gpu, tmp_path, world):
    """svds on delayed re-orthogonalisation, GMRES on DCGS2 (Python-driven and the one-call
    nkv_gmres_dcgs2, identical bit for bit on every rank), a UPO Newton solve through the legacy
    dispatcher (mode 2.1: period row, time in k_dot) and the wave-maker (multi-file mode sets
    written and read by every rank) on `world` gloo ranks sharing the GPU (4: config 5's split)
    reproduce the one-rank run:
    singular values and C to 1e-12, GMRES histories 1e-8 (the oracle tests' gate) and the solution's projection 1e-12, the
    modulus of <a, d>_W and the assembled wave-maker field to 1e-10 (Ritz vectors converged to ~1e-9)."""
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_next, args=((0, 1), out, _free_port(), str(tmp_path)))
    p.start()
    p.join()
    assert p.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_next, args=((r, world), out, port, str(tmp_path))) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    one = out[(1, 0)]
    for rank in range(world):
        got = out[(world, rank)]
        s1, C1 = one["svds"]
        s2, C2 = got["svds"]
        np.testing.assert_allclose(s2[:6], s1[:6], rtol=1e-12)
        np.testing.assert_allclose(C2, C1, rtol=0, atol=1e-12 * np.abs(C1).max())
        i1, o1, p1 = one["gmres"]
        i2, o2, p2 = got["gmres"]
        assert len(i1) == len(i2) and len(o1) == len(o2)
        np.testing.assert_allclose(i2, i1, rtol=1e-8)   # as the oracle gate: partial-sum grouping only
        np.testing.assert_allclose(o2, o1, rtol=1e-8)
        assert abs(p2 - p1) <= 1e-12 * abs(p1)
        assert got["gmres_native_equal"]   # nkv_gmres_dcgs2 == the Python-driven cycle, bit for bit
        i1, o1, p1, t1 = one["upo"]
        i2, o2, p2, t2 = got["upo"]
        assert len(i1) == len(i2) and len(o1) == len(o2) and len(o1) >= 2
        np.testing.assert_allclose(i2, i1, rtol=1e-8)
        np.testing.assert_allclose(o2, o1, rtol=1e-8)
        assert abs(p2 - p1) <= 1e-10 * abs(p1) and abs(t2 - t1) <= 1e-10 * abs(t1)   # period correction
        ip1, g1 = one["wm"]
        ip2, g2 = got["wm"]
        # the eigenvectors' free phase (dgeev's sign) may differ between world sizes: |<a, d>| and the
        # wave-maker field do not depend on it.  The modes are Ritz vectors converged to residual
        # ~1e-9 (|<a, d>| = 1 - 1.3e-9); the world size changes only the partial-sum grouping, which
        # moves them by up to ~1e-12 relative (1.06e-12 measured at 4 ranks): gate 1e-10
        assert abs(abs(ip2) - abs(ip1)) <= 1e-10 * abs(ip1)
        assert np.max(np.abs(g2 - g1)) <= 1e-10 * np.max(np.abs(g1))


def _run_config5(world_rank_pair, out, port, E):
    """Config 5 on one rank of `world` (BASELINE: 4 GPUs): direct and adjoint Krylov–Schur on
    A = D + rank-2 non-normal term (two bases resident), leading modes, bi-orthogonalisation."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur, ritz_vector
        from nekstab_next_amd.layout import box3d_layout
        from nekstab_next_amd.operators import DiagOperator, RankTwoPerturbed
        from nekstab_next_amd.sensitivity import biorthogonalize
        from nekstab_next_amd.vector import NekContext

        lay = box3d_layout(E).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=Comm(), max_cols=40)
        d, _ = syn.diag_spectrum(lay)
        vs = [ctx.vector().from_packed(syn.hash_vector(lay, s) * 1e-3) for s in (21, 22, 23, 24)]
        A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=50.0)
        seed = ctx.vector()
        seed.fill_hash(11)
        cfg = KrylovSchurConfig(k_dim=30, schur_tgt=2)
        rd = krylov_schur(ctx, A, seed, cfg)
        ra = krylov_schur(ctx, A, seed, cfg, transpose=True)
        dRe, dIm, aRe, aIm = (ctx.vector() for _ in range(4))
        ritz_vector(ctx, rd.Q, rd.vecs, 0, dRe, dIm, k=30)
        ritz_vector(ctx, ra.Q, ra.vecs, 0, aRe, aIm, k=30)
        ip = biorthogonalize(ctx, dRe, dIm, aRe, aIm)
        # norm_grad on the shard (gradm1 element-local, one all-reduced dot): the filter's number
        from seed_helpers import box_mesh_coords

        from nekstab_next_amd.sensitivity import NormGrad

        ng = NormGrad(ctx, box_mesh_coords(lay, (E, 1, 1)))(dRe)
        out[(world, rank)] = dict(
            d=(rd.vals, rd.residual, rd.mstart_history, rd.cnt_history, rd.schur_cnt),
            a=(ra.vals, ra.residual, ra.mstart_history, ra.cnt_history, ra.schur_cnt),
            ip=ip, modes=[x.to_packed() for x in (dRe, dIm, aRe, aIm)], norm_grad=ng)
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_config5_four_ranks_vs_oracle(gpu):
    """Config 5 split as BASELINE names it (4 ranks; gloo ranks sharing this box's GPU) at reduced N
    (3-D lx1=8, E=61: ragged 15/15/15/16-element shards) against the oracle's UNSHARDED run
    (sensitivity.f90:393-469 after two eigensolver runs, eigensolvers.f90:120-359): direct and
    adjoint restart trajectories identical, comparison-set Ritz values 1e-10, and every rank's
    shard of the bi-orthogonalised leading modes equal to the oracle's modes (1e-9 of max, after
    the pair's common sign) with <a, d>_W = 1 + 0i to 1e-12 on both; the spurious-mode filter's
    norm_grad of the direct mode, computed on the shards, equals the oracle's on the whole mesh."""
    import oracle as orc
    from helpers import olayout, oracle_rank2_matvec
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    E, world = 61, 4
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_run_config5, args=((r, world), out, port, E)) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    g = box3d_layout(E)
    L, w = olayout(g), syn.mass_weights(g)
    d, _ = syn.diag_spectrum(g)
    vh = [syn.hash_vector(g, s) * 1e-3 for s in (21, 22, 23, 24)]
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(g, syn.hash_vector(g, 11)))
    orc.set_threads(8)
    try:
        ref = {tr: orc.krylov_schur(L, w, oracle_rank2_matvec(g, d, *vh, 50.0, w, tr), q1, 30, 2)
               for tr in (False, True)}
    finally:
        orc.set_threads(1)
    modes = []
    for tr in (False, True):
        re, im, _, _ = orc.outpost_mode(L, w, ref[tr]["Q"], ref[tr]["vecs"], 0, 30)
        modes += [re, im]
    o = orc.biorthogonalize(L, w, *modes)
    o_pad = [syn.from_reference_order(g, v) for v in o]
    from seed_helpers import box_mesh_coords

    ng_ref = orc.norm_grad(g.lx1, 3, box_mesh_coords(g, (E, 1, 1)), w, [o[0][c * g.n_v:(c + 1) * g.n_v] for c in range(3)])
    for rank in range(world):
        got = out[(world, rank)]
        for key, tr in (("d", False), ("a", True)):
            vals, res_, mh, ch, sc = got[key]
            r = ref[tr]
            assert sc == r["schur_cnt"] and mh == r["mstart"] and ch == r["cnt"], (rank, key)
            sel = ritz_compare_set(r["vals"], r["residual"], 1e-6)
            assert np.max(np.abs(match_ritz(r["vals"][sel], vals) - r["vals"][sel]) / np.abs(r["vals"][sel])) <= 1e-10
        s = g.shard(rank, world)
        sign = None
        for x, y in zip(got["modes"], o_pad):
            pieces = [(x[f * s.sv: f * s.sv + s.n_v], y[f * g.sv + s.v_offset: f * g.sv + s.v_offset + s.n_v])
                      for f in range(g.n_wf)]
            pieces.append((x[s.n_wf * s.sv: s.n_wf * s.sv + s.n_p],
                           y[g.n_wf * g.sv + s.p_offset: g.n_wf * g.sv + s.p_offset + s.n_p]))
            a = np.concatenate([p[0] for p in pieces])
            b = np.concatenate([p[1] for p in pieces])
            if sign is None:   # the leading mode's free sign (dgeev's), common to the bi-orthogonal pair
                sign = 1.0 if np.dot(a, b) >= 0 else -1.0
            scale = max(np.max(np.abs(v)) for v in o)
            assert np.max(np.abs(sign * a - b)) <= 1e-9 * scale, rank
        ip = got["ip"]
        assert abs(abs(ip) - 1.0) < 0.5   # <a, d> before the rescaling: O(1)
        assert abs(got["norm_grad"] - ng_ref) <= 1e-8 * ng_ref, (rank, got["norm_grad"], ng_ref)   # modes agree to 1e-9



def _run_config3_full(world_rank_pair, out, port, E, m, spectrum="shift_invert", tgt=0):
    """Config 3 as BASELINE names it (3-D lx1=8, E=44,176: N=100,014,464, m=128), DCGS2, one m-step
    factorisation + Ritz extraction (krylov_schur with schur_tgt=0) on this rank's element shard;
    ``spectrum="clustered", tgt=4``: bench.py's restart leg (a Krylov–Schur solve with a restart)."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur
        from nekstab_next_amd.layout import box3d_layout
        from nekstab_next_amd.operators import DiagOperator
        from nekstab_next_amd.vector import NekContext

        lay = box3d_layout(E).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=Comm(), max_cols=m + 1)
        d, exact = syn.laplacian_shift_invert(lay) if spectrum == "shift_invert" else syn.clustered_spectrum(lay)
        op = DiagOperator(ctx, d)
        del d
        seed = ctx.vector()
        seed.fill_hash(11)
        r = krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=m, schur_tgt=tgt, mode="dcgs2"))
        out[(world, rank)] = (r.vals, r.residual, r.cnt_history, r.schur_cnt, r.H, exact[:8], lay.nelv,
                              r.mstart_history, [np.asarray(x).tolist() for x in r.selected_history])
        print(f"config-3 rank {rank}/{world}: {lay.nelv} elements, {int((r.residual < 1e-6).sum())} converged",
              flush=True)
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_config3_full_size_eight_ranks_match_one_rank(gpu):
    """SURVEY §8(e)'s cross-world gate at BASELINE size: config 3 at E=44,176
    (N=100,014,464, m=128, DCGS2) on 8 gloo ranks sharing the GPU (5,522 elements, 12.9 GB of basis
    per rank, 103 GB in all; the 8-way split of the driver's 8-GPU run) against one rank holding the
    whole 103 GB basis.  Converged and top-8 Ritz values 1e-12 relative, converged counts identical,
    H identical on every rank (replicated, all-reduced) and within 1e-12 of max|H| of the one-rank H
    (only the partial-sum grouping differs); top 8 equal the exact spectrum to 1e-10."""
    E, m = 44176, 128
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_config3_full, args=((0, 1), out, _free_port(), E, m))
    p.start()
    p.join()
    assert p.exitcode == 0
    world = 8
    port = _free_port()
    procs = [ctx.Process(target=_run_config3_full, args=((r, world), out, port, E, m)) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    v1, r1, cnt1, sc1, H1, exact = out[(1, 0)][:6]
    assert [out[(world, r)][6] for r in range(world)] == [5522] * 8
    conv = r1 < 1e-6
    sel = sorted(set(np.nonzero(conv)[0].tolist()) | set(range(8)))
    np.testing.assert_allclose(v1[:8].real, exact, rtol=1e-10)
    for rank in range(world):
        v2, r2, cnt2, sc2, H2 = out[(world, rank)][:5]
        assert cnt2 == cnt1 and sc2 == sc1 == 0
        assert np.max(np.abs(v2[sel] - v1[sel]) / np.abs(v1[sel])) <= 1e-12
        np.testing.assert_array_equal(H2, out[(world, 0)][4])   # identical H on every rank
    assert np.max(np.abs(out[(world, 0)][4] - H1)) <= 1e-12 * np.max(np.abs(H1))



def test_config3_full_size_restart_eight_ranks_match_one_rank(gpu):
    """The Krylov–Schur leg with a restart that the driver's 8-GPU bench line runs on every rank
    (bench.py's krylov_schur_restart_leg: config 3's layout at E=44,176, clustered spectrum,
    k_dim=128, schur_tgt=4; one condensation keeping 25 columns: host LAPACK replicated on the
    all-reduced H, the kept-column rotation on each shard) on 8 gloo ranks sharing the GPU against
    one rank: identical restart / mstart / converged-count histories and selected masks on every
    rank, comparison-set Ritz values 1e-12 relative, H identical on every rank."""
    E, m = 44176, 128
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_config3_full, args=((0, 1), out, _free_port(), E, m, "clustered", 4))
    p.start()
    p.join()
    assert p.exitcode == 0
    world = 8
    port = _free_port()
    procs = [ctx.Process(target=_run_config3_full, args=((r, world), out, port, E, m, "clustered", 4))
             for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    v1, r1, cnt1, sc1, H1, _exact, _n, mh1, sel1 = out[(1, 0)]
    assert sc1 >= 1 and mh1
    sel = ritz_compare_set(v1, r1, 1e-6)
    for rank in range(world):
        v2, r2, cnt2, sc2, H2, _e, nelv, mh2, sel2 = out[(world, rank)]
        assert nelv == 5522
        assert (cnt2, sc2, mh2, sel2) == (cnt1, sc1, mh1, sel1), rank
        assert np.max(np.abs(match_ritz(v1[sel], v2) - v1[sel]) / np.abs(v1[sel])) <= 1e-12
        np.testing.assert_array_equal(H2, out[(world, 0)][4])

def _run_config5_full(world_rank_pair, out, port, E, m):
    """Config 5 as BASELINE names it (3-D lx1=8, E=22,088: N=50,007,232, k_dim=96, two bases
    resident) on this rank's element shard: direct and adjoint Krylov–Schur, leading modes,
    bi-orthogonalisation; the modes are reported through W-dots with shard-independent hashed probe
    vectors (global all-reduced scalars, identical on every rank)."""
    rank, world = world_rank_pair
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur, ritz_vector
        from nekstab_next_amd.layout import box3d_layout
        from nekstab_next_amd.operators import DiagOperator, RankTwoPerturbed
        from nekstab_next_amd.sensitivity import biorthogonalize
        from nekstab_next_amd.vector import NekContext

        lay = box3d_layout(E).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=Comm(), max_cols=m + 1)
        d, _ = syn.diag_spectrum(lay)
        vs = []
        for s5 in (21, 22, 23, 24):
            v = ctx.vector()
            v.fill_hash(s5)
            v.scal(1e-3)
            vs.append(v)
        A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=50.0)
        del d
        seed = ctx.vector()
        seed.fill_hash(11)
        cfg = KrylovSchurConfig(k_dim=m, schur_tgt=2, mode="dcgs2")
        rd = krylov_schur(ctx, A, seed, cfg)
        ra = krylov_schur(ctx, A, seed, cfg, transpose=True)
        dRe, dIm, aRe, aIm = (ctx.vector() for _ in range(4))
        ritz_vector(ctx, rd.Q, rd.vecs, 0, dRe, dIm, k=m)
        ritz_vector(ctx, ra.Q, ra.vecs, 0, aRe, aIm, k=m)
        biorthogonalize(ctx, dRe, dIm, aRe, aIm)
        bi = (ctx.dot(aRe, dRe, False) + ctx.dot(aIm, dIm, False), ctx.dot(aRe, dIm, False) - ctx.dot(aIm, dRe, False))
        probes = []
        for s5 in (31, 32):
            p = ctx.vector()
            p.fill_hash(s5)
            probes.append([ctx.dot(x, p, False) for x in (dRe, dIm, aRe, aIm)])
        out[(world, rank)] = dict(d=(rd.vals, rd.mstart_history, rd.cnt_history, rd.schur_cnt),
                                  a=(ra.vals, ra.mstart_history, ra.cnt_history, ra.schur_cnt),
                                  bi=bi, probes=probes, nelv=lay.nelv)
        print(f"config-5 rank {rank}/{world}: {lay.nelv} elements, lambda_1 {rd.vals[0]:.12f}", flush=True)
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_config5_full_size_four_ranks_match_one_rank(gpu):
    """Config 5's split as BASELINE names it (4 GPUs) at its full size (E=22,088: N=50,007,232,
    k_dim=96, two bases resident: 77.6 GB in all, 19.4 GB per rank) on 4 gloo ranks sharing the GPU
    (5,522 elements each) against one rank: the same restart / converged-count histories, direct and
    adjoint comparison-set Ritz values 1e-12 relative, <a, d>_W = 1 + 0i to 1e-12 on every rank, and
    the bi-orthogonalised leading modes equal through their W-dots with two hashed probe vectors
    (1e-10 of the largest, up to the pair's common sign)."""
    E, m = 22088, 96
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_config5_full, args=((0, 1), out, _free_port(), E, m))
    p.start()
    p.join()
    assert p.exitcode == 0
    world = 4
    port = _free_port()
    procs = [ctx.Process(target=_run_config5_full, args=((r, world), out, port, E, m)) for r in range(world)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
        assert q.exitcode == 0
    one = out[(1, 0)]
    assert [out[(world, r)]["nelv"] for r in range(world)] == [5522] * 4
    p1 = np.array(one["probes"])
    scale = np.max(np.abs(p1))
    for r in range(world):
        got = out[(world, r)]
        for key in ("d", "a"):
            v1, mh1, ch1, sc1 = one[key]
            v, mh, ch, sc = got[key]
            assert (mh, ch, sc) == (mh1, ch1, sc1), (r, key)
            sel = list(range(8))
            np.testing.assert_allclose(np.asarray(v)[sel], np.asarray(v1)[sel], rtol=1e-12)
        re_, im_ = got["bi"]
        assert abs(re_ - 1.0) < 1e-12 and abs(im_) < 1e-12, (r, got["bi"])
        pr = np.array(got["probes"])
        sign = 1.0 if np.sum(pr * p1) >= 0 else -1.0
        assert np.max(np.abs(sign * pr - p1)) <= 1e-10 * scale, (r, pr, p1)
