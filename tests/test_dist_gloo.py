"""World-size-2 gloo tests of the sharded path on CPU.

The device kernels need a GPU, so here the per-rank local work is done by the CPU oracle / numpy
on each rank's element-contiguous shard, and the cross-rank step goes through the product's
``Comm`` wrapper (torch.distributed all-reduce of the partial vector) exactly as
``arnoldi.update_hessenberg_matrix`` uses it: one length-j all-reduce per Gram–Schmidt pass plus one
for the norm.  The sharded factorisation must equal the unsharded one.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cgs2_arnoldi(lay, w, d, q0, m, comm):
    """Sharded CGS2 Arnoldi in numpy on one rank: local partials + comm.allreduce_."""
    from nekstab_next_amd import synthetic as syn

    wf = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        wf[f * lay.sv: f * lay.sv + lay.n_v] = w
    Q = np.zeros((m + 1, lay.ld))
    H = np.zeros((m + 1, m))
    Q[0] = q0
    for k in range(1, m + 1):
        f = d * Q[k - 1]
        hs = []
        for _ in range(2):
            h = torch.as_tensor(Q[:k] @ (wf * f))
            comm.allreduce_(h)
            h = h.numpy()
            f = f - h @ Q[:k]
            hs.append(h)
        nrm = torch.as_tensor([np.sum(wf * f * f)])
        comm.allreduce_(nrm)
        beta = float(np.sqrt(nrm.item()))
        H[:k, k - 1] = hs[0] + hs[1]
        H[k, k - 1] = beta
        Q[k] = f / beta
    return H


def _dcgs2_arnoldi(lay, w, d, q0, m, comm):
    """Sharded DCGS2 Arnoldi in numpy on one rank, the algebra of nkv_block_dot2 /
    nkv_dcgs2_coef / nkv_dcgs2_update with deferred normalisation: ONE all-reduce per step, of
    [Q^T W u ; Q^T W A u] (2j values); column j holds u = beta q_j until step j+1 takes
    beta^2 = u^T W u from that dot, divides the raw dots by beta, corrects H and finalises it; a
    closing pass at the end."""
    wf = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        wf[f * lay.sv: f * lay.sv + lay.n_v] = w
    Q = np.zeros((m + 1, lay.ld))
    H = np.zeros((m + 1, m))
    Q[0] = q0
    beta = None

    def correct(mm, hq, beta):   # pending H(mm, mm-1) = beta, row mm corrected for q = r qbar + Q a
        s = 1.0 if beta is None else 1.0 / beta
        if beta is not None and mm > 0:
            H[mm, mm - 1] = beta
        a = hq[:mm] * s
        r = np.sqrt(hq[mm] * s * s - a @ a)
        row = H[mm, :mm].copy()
        Hold = H[:mm, :mm].copy()
        H[:mm, :mm] += np.outer(a, row)
        H[mm, :mm] = row * r
        return a, r, row, Hold, s

    for j in range(1, m + 1):
        mm = j - 1
        f = d * Q[mm]                                   # A u
        h = torch.as_tensor(np.concatenate([Q[:j] @ (wf * Q[mm]), Q[:j] @ (wf * f)]))
        comm.allreduce_(h)
        h = h.numpy()
        beta = None if j == 1 else float(np.sqrt(h[mm]))
        a, r, row, Hold, s = correct(mm, h[:j], beta)
        b, bj = h[j: j + mm] * s, h[j + mm] * s * s
        t = row @ a
        g = np.concatenate([Hold @ a + a * t, [r * t]])
        c = np.concatenate([(b - g[:mm]) / r, [((bj - a @ b) / r - g[mm]) / r]])
        x, y = g[:mm] / r + c[:mm], g[mm] / r + c[mm]
        qbar = (Q[mm] * s - a @ Q[:mm]) / r
        Q[mm] = qbar
        u = f * s / r - x @ Q[:mm] - qbar * y
        H[:j, j - 1] = c
        Q[j] = u
    hq = torch.as_tensor(Q[: m + 1] @ (wf * Q[m]))
    comm.allreduce_(hq)
    hq = hq.numpy()
    beta = float(np.sqrt(hq[m]))
    correct(m, hq, beta)
    r2s = hq[m] - (hq[:m] / beta) @ (hq[:m] / beta) * beta * beta
    Q[m] = (Q[m] - hq[:m] @ Q[:m]) / np.sqrt(r2s)
    return H


def _worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.layout import NekLayout

        comm = Comm()
        assert comm.rank == rank and comm.world == world
        g = NekLayout(ldim=3, lx1=4, lx2=2, nelgv=11, n_scalars=1)
        lay = g.shard(rank, world)
        w = syn.mass_weights(lay)
        d, _ = syn.laplacian_shift_invert(lay)
        q0 = syn.hash_vector(lay, 3)
        # normalise with a global dot
        wf = np.zeros(lay.ld)
        for f in range(lay.n_wf):
            wf[f * lay.sv: f * lay.sv + lay.n_v] = w
        n2 = torch.as_tensor([np.sum(wf * q0 * q0)])
        comm.allreduce_(n2)
        q0 = q0 / np.sqrt(n2.item())
        H = _cgs2_arnoldi(lay, w, d, q0, 12, comm)
        Hd = _dcgs2_arnoldi(lay, w, d, q0, 12, comm)
        mx = comm.max_scalar(float(rank))
        out[rank] = (H, mx, Hd)
    finally:
        dist.destroy_process_group()


def test_sharded_cgs2_equals_unsharded():
    world = 2
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, port, out), nprocs=world, join=True)
    H0, mx0, Hd0 = out[0]
    H1, mx1, Hd1 = out[1]
    np.testing.assert_array_equal(H0, H1)  # every rank holds identical (all-reduced) H
    np.testing.assert_array_equal(Hd0, Hd1)
    assert mx0 == mx1 == 1.0

    sys.path.insert(0, ROOT)
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.comm import Comm
    from nekstab_next_amd.layout import NekLayout

    g = NekLayout(ldim=3, lx1=4, lx2=2, nelgv=11, n_scalars=1)
    w = syn.mass_weights(g)
    d, _ = syn.laplacian_shift_invert(g)
    q0 = syn.hash_vector(g, 3)
    wf = np.zeros(g.ld)
    for f in range(g.n_wf):
        wf[f * g.sv: f * g.sv + g.n_v] = w
    q0 = q0 / np.sqrt(np.sum(wf * q0 * q0))
    Href = _cgs2_arnoldi(g, w, d, q0, 12, Comm())
    assert np.max(np.abs(H0 - Href)) <= 1e-12 * np.max(np.abs(Href))
    # DCGS2 (sharded, 1 all-reduce per step) builds the same Arnoldi factorisation as CGS2
    assert np.max(np.abs(Hd0 - Href)) <= 1e-12 * np.max(np.abs(Href))


def _dot_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle as orc
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.layout import box3d_layout

        lay = box3d_layout(9).shard(rank, world)
        L = orc.OLayout(lay.n_v, lay.n_p, lay.n_wf, False, 3)
        w = syn.mass_weights(lay)
        a = syn.to_reference_order(lay, syn.hash_vector(lay, 1))
        b = syn.to_reference_order(lay, syn.hash_vector(lay, 2))
        part = torch.tensor([orc.k_dot(L, w, a, b)], dtype=torch.float64)
        Comm().allreduce_(part)
        out[rank] = part.item()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_partial_dot_allreduce_equals_full(world):
    port = _free_port()
    out = mp.Manager().dict()
    mp.spawn(_dot_worker, args=(world, port, out), nprocs=world, join=True)
    import oracle as orc
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    g = box3d_layout(9)
    L = orc.OLayout(g.n_v, g.n_p, g.n_wf, False, 3)
    w = syn.mass_weights(g)
    full = orc.k_dot(L, w, syn.to_reference_order(g, syn.hash_vector(g, 1)),
                     syn.to_reference_order(g, syn.hash_vector(g, 2)))
    vals = [out[r] for r in range(world)]
    assert len(set(vals)) == 1
    assert abs(vals[0] - full) <= 1e-13 * abs(full)
