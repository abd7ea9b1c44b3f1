"""More ranks than elements on the sharded GPU path (gloo ranks sharing this box's GPU): a rank
that owns no element takes part in every collective step — the Arnoldi all-reduces, the ifres
checkpoint's KRY set (a header-only member) and the restart's H broadcast, outpost_ks's mode files
and the wave-maker chain — and the results equal one rank's (Nek5000 allows lelt-empty ranks)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from test_gpu_multirank import ROOT, _free_port

pytestmark = pytest.mark.gpu


def _run_tiny(world_rank_pair, out, port, tmpdir):
    """More ranks than elements (cylinder layout, E=2, world 3: rank 0 owns no element): the
    ifres checkpoint, a restart from it, outpost_ks's mode files and the wave-maker chain."""
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
        from nekstab_next_amd.checkpoint import ArnoldiCheckpoint, load_restart
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.config import KrylovSchurConfig
        from nekstab_next_amd.krylov_schur import krylov_schur, outpost_ks
        from nekstab_next_amd.layout import cylinder_layout
        from nekstab_next_amd.operators import DiagOperator
        from nekstab_next_amd.sensitivity import velocity_layout, wave_maker
        from nekstab_next_amd.vector import NekContext

        comm = Comm()
        lay = cylinder_layout(2).shard(rank, world)
        ctx = NekContext(lay, weights=syn.mass_weights(lay), comm=comm, max_cols=16)
        d, _ = syn.diag_spectrum(lay)
        op = DiagOperator(ctx, d)
        seed = ctx.vector()
        seed.fill_hash(11)
        cfg = KrylovSchurConfig(k_dim=8, schur_tgt=2, mode="mgs2")
        ck = os.path.join(tmpdir, f"ck{world}")
        krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=8, schur_tgt=0, mode="mgs2"),
                     on_step=ArnoldiCheckpoint(ctx, ck, session="t", evop="d"))
        Q, H = load_restart(ctx, ck, "t", 4, 8)
        rr = krylov_schur(ctx, op, None, cfg, Q=Q, start=(4, H))
        rd = krylov_schur(ctx, op, seed, cfg)
        md = os.path.join(tmpdir, f"m{world}")
        outpost_ks(ctx, rd, md, evop="d", maxmodes=1, session="t", orthonormality=False)
        outpost_ks(ctx, rd, md, evop="a", maxmodes=1, session="t", orthonormality=False)
        vlay = velocity_layout(cylinder_layout(2)).shard(rank, world)
        vctx = NekContext(vlay, weights=syn.mass_weights(vlay), comm=comm, max_cols=4)
        wm = wave_maker(vctx, md, session="t", d_num=1, a_num=1)
        g = np.zeros((2, vlay.pts_v))
        for f in fld.read_fld_set(md, "wm_", "t", 1):
            if f.emap.size:
                g[f.emap - 1] = f.fields["t"]
        out[(world, rank)] = dict(resumed=(rr.vals, rr.mstart_history, rr.schur_cnt), full=(rd.vals, rd.residual),
                                  ip=wm["inner_product"], wm=g)
    finally:
        if world > 1:
            dist.destroy_process_group()


def test_more_ranks_than_elements_file_chain(gpu, tmp_path):
    """A rank with no elements takes part in every collective file operation (header-only members
    of the KRY / mode / wave-maker sets, the HES broadcast) and the results equal one rank's."""
    out = mp.Manager().dict()
    ctx = mp.get_context("spawn")
    for world in (1, 3):
        port = _free_port()
        procs = [ctx.Process(target=_run_tiny, args=((r, world), out, port, str(tmp_path))) for r in range(world)]
        for q in procs:
            q.start()
        for q in procs:
            q.join()
            assert q.exitcode == 0
    one = out[(1, 0)]
    for rank in range(3):
        got = out[(3, rank)]
        v1, m1, c1 = one["resumed"]
        v2, m2, c2 = got["resumed"]
        assert m1 == m2 and c1 == c2
        np.testing.assert_allclose(v2[:2], v1[:2], rtol=1e-10)
        np.testing.assert_allclose(got["full"][0][:2], one["full"][0][:2], rtol=1e-10)
        assert abs(abs(got["ip"]) - abs(one["ip"])) <= 1e-10 * abs(one["ip"])
        np.testing.assert_allclose(got["wm"], one["wm"], rtol=0, atol=1e-10 * np.abs(one["wm"]).max())
