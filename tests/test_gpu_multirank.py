"""Sharded (world_size 2) GPU path on ONE MI355X: two ranks share the device and exchange partial
dots through gloo (RCCL cannot place two ranks on one GPU; on an 8-GPU node the same code runs over
RCCL/xGMI).  Sharded Krylov–Schur must reproduce the single-rank result: identical restart
trajectory, Ritz values to 1e-12 (SURVEY.md §8(e) gate)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_ks(world_rank_pair, out, port, E_box=96, E_cyl=400):
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
        d, _ = syn.laplacian_shift_invert(lay)
        seed = ctx.vector()
        seed.fill_hash(11)
        r = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=32, schur_tgt=4))
        res["lap"] = (r.vals, r.residual, r.mstart_history, r.schur_cnt, r.H)
        lay2 = cylinder_layout(E_cyl).shard(rank, world)
        ctx2 = NekContext(lay2, weights=syn.mass_weights(lay2), comm=comm, max_cols=48)
        c, s, dr, _ = syn.rot2_operator(lay2)
        seed2 = ctx2.vector()
        seed2.fill_hash(5)
        r2 = krylov_schur(ctx2, Rot2Operator(ctx2, c, s, dr), seed2, KrylovSchurConfig(k_dim=24, schur_tgt=2))
        res["rot"] = (r2.vals, r2.residual, r2.mstart_history, r2.schur_cnt, r2.H)
        out[(world, rank)] = res
    finally:
        if world > 1:
            dist.destroy_process_group()


@pytest.mark.parametrize("world,E_box,E_cyl", [(2, 96, 400), (3, 97, 401), (8, 101, 403)])
def test_ranks_match_one_rank(gpu, world, E_box, E_cyl):
    """Krylov–Schur on `world` gloo ranks sharing the GPU (the sharded HIP path, one shard per
    process) reproduces the one-rank run; (3, 97, 401) gives ragged shards (32/32/33 and
    133/134/134 elements); (8, 101, 403) rehearses the 8-way split of the driver's 8-GPU run with
    ragged shards (12/13 and 50/51 elements)."""
    mgr = mp.Manager()
    out = mgr.dict()
    ctx = mp.get_context("spawn")
    p = ctx.Process(target=_run_ks, args=((0, 1), out, _free_port(), E_box, E_cyl))
    p.start()
    p.join()
    assert p.exitcode == 0
    port = _free_port()
    procs = [ctx.Process(target=_run_ks, args=((r, world), out, port, E_box, E_cyl)) for r in range(world)]
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
    for mode in ("dcgs2", "cgs2"):
        r = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=32, schur_tgt=4, mode=mode))
        out[(forced, mode)] = (r.vals, r.H, r.mstart_history)
    assert comm.max_scalar(3.0, device=ctx.device) == 3.0
for mode in ("dcgs2", "cgs2"):
    a, b = out[(False, mode)], out[(True, mode)]
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
