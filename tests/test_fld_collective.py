"""Collective semantics of the per-rank field-file I/O (CPU, gloo ranks).

Nek5000's ``outpost2`` / ``load_fld`` are collective (eigensolvers.f90:607-615 writes the mode set
that sensitivity.f90:40-60 reads back; the restart reads HES on rank 0 and broadcasts it,
eigensolvers.f90:244-266, then ``load_files`` reads KRY 1..mstart, IO.f90:12-73).  The product's
writers end in ``fld.collective_output`` (a barrier once this rank's files are in place); these
tests run the same context manager and readers with no GPU:

* the race that turned the round-3 GPU run red: one rank writes its member of a set late; with
  the barrier every rank reads the whole set, without it the other ranks find the member missing
  and ``read_fld_set`` raises (it never returns a partial set);
* a restart on 8 ranks opens each KRY file in exactly one rank when the set was written at the
  same world size, only the files intersecting its elements otherwise, and HES only on rank 0
  (the other ranks get H by broadcast).
"""
import os
import socket
import sys
import time

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _race_worker(rank, world, port, directory, barrier, late, reader_comm, out):
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld   # imports and data before the rendezvous: the ranks leave it together
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.comm import Comm
    from nekstab_next_amd.layout import box3d_layout

    lay = box3d_layout(23).shard(rank, world)
    f = fld.fld_from_vector(lay, syn.hash_vector(lay, 4), time=1.0, istep=1)
    _init(rank, world, port)
    try:
        comm = Comm()
        comm.barrier()
        with fld.collective_output(comm, barrier=barrier):
            if rank == late:
                time.sleep(3.0)   # the slowest writer (rank 0 also writes the Spectre_* text)
            fld.write_fld(os.path.join(directory, fld.fld_name("aRe", "mr", rank, 1)), f)
        try:
            # as wave_maker's _load_modes: this rank's elements of the set (reader_comm: the
            # product's collective read, rank 0 broadcasting the set header; without: each rank alone)
            files = fld.read_fld_set(directory, "aRe", "mr", 1, lay=lay, comm=comm if reader_comm else None)
            got = fld.vector_from_fld(lay, files)
            out[rank] = ("ok", float(np.max(np.abs(got - syn.hash_vector(lay, 4)))))
        except FileNotFoundError as e:
            out[rank] = ("missing", str(e))
        comm.barrier()   # keep every rank alive until all have read
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("barrier,late,reader_comm", [(True, 0, True), (True, 3, False), (False, 0, False),
                                                      (False, 3, False)])
def test_delayed_writer_needs_the_barrier(tmp_path, barrier, late, reader_comm):
    """Rank `late` writes its member 3 s after the others.  Late rank 0 is the round-3 failure
    (the readers race rank 0's file); late rank 3 is the same race on a member other than the
    header's.  Without the barrier the independent readers fail (the product's collective read
    broadcasts the set header from rank 0; whether that broadcast also waits for the late rank is
    backend behaviour, so the writers' barrier is what the product relies on)."""
    world = 4
    out = mp.Manager().dict()
    mp.spawn(_race_worker, args=(world, _free_port(), str(tmp_path), barrier, late, reader_comm, out),
             nprocs=world, join=True)
    if barrier:
        for r in range(world):
            assert out[r][0] == "ok", out[r]
            assert out[r][1] < 1e-13   # pressure goes through the lx2 <-> lx1 mapping
    else:
        # without the barrier the ranks that finish first read before the late member exists:
        # an error, not the partial set the round-3 reader returned
        assert out[late][0] == "ok"
        for r in range(world):
            if r != late:
                assert out[r][0] == "missing", out[r]
    # atomic writes leave no temporary files behind
    assert not [f for f in os.listdir(tmp_path) if ".part" in f]


def _write_ckpt(directory, E, world, mstart, k_dim):
    """A KRY/HES checkpoint as `world` ranks write it (fid = rank), with known contents."""
    from nekstab_next_amd import checkpoint as ck
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import NekLayout

    g = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=E)
    for r in range(world):
        lay = g.shard(r, world)
        for i in range(1, mstart + 2):
            f = fld.fld_from_vector(lay, syn.hash_vector(lay, 100 + i), time=float(i - 1), istep=i)
            fld.write_fld(os.path.join(directory, fld.fld_name("KRY", "cyl", r, i)), f)
    H = np.zeros((k_dim + 1, k_dim))
    rng = np.random.default_rng(5)
    for j in range(mstart):
        H[: j + 2, j] = rng.standard_normal(j + 2)
    ck.write_hes(os.path.join(directory, f"HEScyl{mstart:04d}"), H, mstart)
    return H


def _restart_worker(rank, world, port, directory, E, mstart, k_dim, out):
    _init(rank, world, port)
    try:
        from nekstab_next_amd import checkpoint as ck
        from nekstab_next_amd import fld
        from nekstab_next_amd import synthetic as syn
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.layout import NekLayout

        opened, hes = [], []
        real_read, real_header, real_hes = fld.read_fld, fld.read_fld_header, ck.read_hes
        fld.read_fld = lambda p: (opened.append(os.path.basename(p)), real_read(p))[1]
        fld.read_fld_header = lambda p: (opened.append("hdr:" + os.path.basename(p)), real_header(p))[1]
        ck.read_hes = lambda p, *a: (hes.append(os.path.basename(p)), real_hes(p, *a))[1]
        comm = Comm()
        lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=E).shard(rank, world)
        H = ck.read_restart_hes(comm, directory, "cyl", mstart, k_dim)
        err = 0.0
        for i, v in enumerate(ck.restart_vectors(lay, directory, "cyl", mstart, comm)):
            err = max(err, float(np.max(np.abs(v - syn.hash_vector(lay, 101 + i)))))
        out[rank] = (opened, hes, H, err, i + 1)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("w_write", [8, 3])
def test_restart_reads_own_files_and_broadcasts_hes(tmp_path, w_write):
    world, E, mstart, k_dim = 8, 301, 5, 8
    H_ref = _write_ckpt(str(tmp_path), E, w_write, mstart, k_dim)
    out = mp.Manager().dict()
    mp.spawn(_restart_worker, args=(world, _free_port(), str(tmp_path), E, mstart, k_dim, out), nprocs=world,
             join=True)
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld
    from nekstab_next_amd.layout import NekLayout

    g = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=E)
    per_file = {}
    for r in range(world):
        opened, hes, H, err, nvec = out[r]
        assert nvec == mstart + 1 and err < 1e-13
        np.testing.assert_array_equal(H[: mstart + 1, :mstart], H_ref[: mstart + 1, :mstart])
        assert hes == ([f"HEScyl{mstart:04d}"] if r == 0 else [])   # rank 0 parses, the rest receive
        # the set header: fid 0's, read by rank 0 only and broadcast; no fallback header scan
        assert [p for p in opened if p.startswith("hdr:")] == (
            [f"hdr:{fld.fld_name('KRY', 'cyl', 0, i)}" for i in range(1, mstart + 2)] if r == 0 else [])
        data = [p for p in opened if not p.startswith("hdr:")]
        e0, e1 = g.shard(r, world).elem_range()
        mine = [fid for fid in range(w_write) if g.shard(fid, w_write).elem_range()[0] < e1
                and g.shard(fid, w_write).elem_range()[1] > e0]
        expect = sorted(fld.fld_name("KRY", "cyl", fid, i) for i in range(1, mstart + 2) for fid in mine)
        assert sorted(data) == expect, (r, opened)
        for p in opened:
            per_file.setdefault(p.removeprefix("hdr:"), set()).add(r)
    if w_write == world:   # every file opened by exactly one rank (fid r by rank r)
        assert len(per_file) == world * (mstart + 1)
        assert all(len(ranks) == 1 for ranks in per_file.values())
    else:
        assert len(per_file) == w_write * (mstart + 1)


def test_read_fld_set_refuses_incomplete_and_foreign_sets(tmp_path):
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import cylinder_layout

    g = cylinder_layout(40)
    d = str(tmp_path)
    for r in (0, 1, 3):   # fid 2 of a 4-file set missing
        lay = g.shard(r, 4)
        fld.write_fld(os.path.join(d, fld.fld_name("KRY", "s", r, 1)), fld.fld_from_vector(lay, syn.hash_vector(lay, 1)))
    with pytest.raises(FileNotFoundError, match="missing fids \\[2\\]"):
        fld.read_fld_set(d, "KRY", "s", 1)
    for r in range(4):   # every rank of any world size refuses the incomplete set, even if its fid exists
        with pytest.raises(FileNotFoundError):
            fld.read_fld_set(d, "KRY", "s", 1, lay=g.shard(r, 4))
    # a stale larger set beside a complete 2-file set: the header's nfileo decides
    for r in range(2):
        lay = g.shard(r, 2)
        fld.write_fld(os.path.join(d, fld.fld_name("KRY", "s", r, 2)), fld.fld_from_vector(lay, syn.hash_vector(lay, 2)))
    for r in range(5):   # a leftover fid 2..4 from an older run
        fld.write_fld(os.path.join(d, fld.fld_name("KRY", "s", 2 + r, 2)),
                      fld.fld_from_vector(g.shard(4, 5), syn.hash_vector(g.shard(4, 5), 9)))
    for r, w in ((0, 1), (0, 2), (1, 2), (2, 3)):
        lay = g.shard(r, w)
        got = fld.vector_from_fld(lay, fld.read_fld_set(d, "KRY", "s", 2, lay=lay))
        np.testing.assert_allclose(got, syn.hash_vector(lay, 2), rtol=0, atol=1e-13)
    # a set with another element distribution (e.g. a foreign writer): header scan, same result
    import shutil

    d3 = str(tmp_path / "foreign")
    os.makedirs(d3)
    full = fld.fld_from_vector(g, syn.hash_vector(g, 3))
    order = np.random.default_rng(0).permutation(40)
    for fid, part in enumerate(np.array_split(order, 3)):
        f = fld.FldFile(full.nx, full.ny, full.nz, 40, 0.0, 0, fid, 3, full.rdcode, (part + 1).astype(np.int32),
                        {k: v[part] for k, v in full.fields.items()})
        fld.write_fld(os.path.join(d3, fld.fld_name("KRY", "s", fid, 1)), f)
    for r in range(4):
        lay = g.shard(r, 4)
        got = fld.vector_from_fld(lay, fld.read_fld_set(d3, "KRY", "s", 1, lay=lay))
        np.testing.assert_allclose(got, syn.hash_vector(lay, 3), rtol=0, atol=1e-13)
    # a set that does not cover the shard's elements is refused, not zero-filled
    shutil.rmtree(d3)
    os.makedirs(d3)
    f = fld.FldFile(full.nx, full.ny, full.nz, 40, 0.0, 0, 0, 1, full.rdcode, np.arange(1, 39, dtype=np.int32),
                    {k: v[:38] for k, v in full.fields.items()})
    fld.write_fld(os.path.join(d3, fld.fld_name("KRY", "s", 0, 1)), f)
    with pytest.raises(ValueError, match="in no file"):
        fld.read_fld_set(d3, "KRY", "s", 1, lay=g.shard(1, 2))


def test_sets_with_empty_shards(tmp_path):
    """More ranks than elements: the writers of empty shards write element-less members (Nek5000
    would too), and readers of any world size, empty shards included, get their elements back."""
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import cylinder_layout

    g = cylinder_layout(3)
    d = str(tmp_path)
    for r in range(5):
        lay = g.shard(r, 5)
        fld.write_fld(os.path.join(d, fld.fld_name("KRY", "s", r, 1)), fld.fld_from_vector(lay, syn.hash_vector(lay, 7)))
    for w in (1, 2, 5, 7):
        for r in range(w):
            lay = g.shard(r, w)
            files = fld.read_fld_set(d, "KRY", "s", 1, lay=lay)
            if lay.nelv:
                assert all(f.emap.size for f in files)
            else:   # the set's header only: time / istep as on the other ranks
                assert len(files) == 1 and files[0].emap.size == 0 and files[0].nfileo == 5
            np.testing.assert_allclose(fld.vector_from_fld(lay, files), syn.hash_vector(lay, 7), rtol=0, atol=1e-13)


def test_rank_local_reads_any_world_pair(tmp_path):
    """Sets written by W ranks read by R ranks (random E, W, R, including W > E and R > E): every
    reader gets exactly its elements and opens only the files whose element range meets its own."""
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import cylinder_layout

    rng = np.random.default_rng(11)
    for case in range(12):
        E, W, R = int(rng.integers(1, 30)), int(rng.integers(1, 9)), int(rng.integers(1, 9))
        g = cylinder_layout(E)
        d = str(tmp_path / f"c{case}")
        os.makedirs(d)
        for r in range(W):
            lay = g.shard(r, W)
            fld.write_fld(os.path.join(d, fld.fld_name("KRY", "s", r, 3)),
                          fld.fld_from_vector(lay, syn.hash_vector(lay, case)))
        opened = []
        real = fld.read_fld
        fld.read_fld = lambda p: (opened.append(p), real(p))[1]
        try:
            for r in range(R):
                lay = g.shard(r, R)
                opened.clear()
                got = fld.vector_from_fld(lay, fld.read_fld_set(d, "KRY", "s", 3, lay=lay))
                np.testing.assert_allclose(got, syn.hash_vector(lay, case), rtol=0, atol=1e-13)
                e0, e1 = lay.elem_range()
                need = {fid for fid in range(W) if g.shard(fid, W).elem_range()[0] < e1
                        and g.shard(fid, W).elem_range()[1] > e0}
                assert {int(os.path.basename(p).split(".")[0][len("KRYs"):]) for p in opened} == need, (E, W, R, r)
        finally:
            fld.read_fld = real


def _missing_worker(rank, world, port, directory, out):
    _init(rank, world, port)
    try:
        from nekstab_next_amd import checkpoint as ck
        from nekstab_next_amd import fld
        from nekstab_next_amd.comm import Comm
        from nekstab_next_amd.layout import cylinder_layout

        comm = Comm()
        res = []
        try:
            ck.read_restart_hes(comm, directory, "none", 3, 8)
            res.append("read")
        except FileNotFoundError:
            res.append("hes missing")
        try:
            fld.read_fld_set(directory, "KRY", "none", 1, lay=cylinder_layout(9).shard(rank, world), comm=comm)
            res.append("read")
        except FileNotFoundError:
            res.append("set missing")
        comm.barrier()
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_missing_files_raise_on_every_rank(tmp_path):
    """A restart from files that are not there: rank 0's failure to parse HES, and the missing set
    header, are broadcast, so every rank raises FileNotFoundError instead of waiting for rank 0."""
    world = 3
    out = mp.Manager().dict()
    mp.spawn(_missing_worker, args=(world, _free_port(), str(tmp_path), out), nprocs=world, join=True)
    for r in range(world):
        assert out[r] == ["hes missing", "set missing"], out[r]


def _one_rank_fails_worker(rank, world, port, directory, out):
    sys.path.insert(0, ROOT)
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.comm import Comm
    from nekstab_next_amd.layout import box3d_layout

    _init(rank, world, port)
    try:
        comm = Comm()
        res = []
        # (1) a 3-file set whose last member holds only the first half of its elements: rank 2's shard
        #     (E=24 on 3 ranks: elements 16..23) is partly uncovered, ranks 0 and 1 read fine alone
        g = box3d_layout(24)
        if rank == 0:
            for fid in range(world):
                sh = g.shard(fid, world)
                f = fld.fld_from_vector(sh, syn.hash_vector(sh, 4), time=1.0, istep=1)
                if fid == world - 1:
                    f.emap = f.emap[:4]
                    for k in list(f.fields):
                        f.fields[k] = f.fields[k][:4]
                fld.write_fld(os.path.join(directory, fld.fld_name("cov", "x", fid, 1)), f)
        comm.barrier()
        try:
            fld.read_fld_set(directory, "cov", "x", 1, lay=g.shard(rank, world), comm=comm)
            res.append("read")
        except ValueError as e:
            res.append(("ValueError", "rank 2" in str(e) or rank == 2))
        # (2) a truncated member on rank 1 only (its own fid): every rank raises
        if rank == 0:
            for fid in range(world):
                sh = g.shard(fid, world)
                fld.write_fld(os.path.join(directory, fld.fld_name("trc", "x", fid, 1)),
                              fld.fld_from_vector(sh, syn.hash_vector(sh, 5), time=1.0, istep=1))
            p1 = os.path.join(directory, fld.fld_name("trc", "x", 1, 1))
            with open(p1, "r+b") as fh:
                fh.truncate(os.path.getsize(p1) // 2)
        comm.barrier()
        try:
            fld.read_fld_set(directory, "trc", "x", 1, lay=g.shard(rank, world), comm=comm)
            res.append("read")
        except Exception as e:  # noqa: BLE001
            res.append(("raised", "rank 1" in str(e) or rank == 1))
        # (3) a writer that fails on rank 0 only (HES on a full disk): every rank raises at the end of
        #     collective_output instead of waiting at a barrier rank 0 never reaches
        try:
            with fld.collective_output(comm):
                if rank == 0:
                    raise OSError("No space left on device (HES)")
            res.append("written")
        except OSError as e:
            res.append(("OSError", "No space left" in str(e)))
        # (4) a body that interleaves collectives with its writes (outpost_ks assembles each mode with
        #     all-reduced norms before writing it): rank 1's first write fails; the guard skips its
        #     later writes while the all-reduces stay in lock-step, and every rank raises at the end
        import torch

        calls = []

        def wr(tag):
            if rank == 1 and tag == 0:
                raise OSError("disk full on rank 1")
            calls.append(tag)

        try:
            with fld.collective_output(comm) as write:
                for tag in range(3):
                    t = torch.ones(1, dtype=torch.float64)
                    dist.all_reduce(t)   # the body's collective
                    write(wr, tag)
            res.append("written")
        except OSError as e:
            res.append(("OSError", "rank 1" in str(e), list(calls)))
        comm.barrier()
        out[rank] = res
    finally:
        dist.destroy_process_group()


def test_one_rank_failures_raise_on_every_rank(tmp_path):
    """a read failure that only one rank sees (its elements in no file of the set, or its
    own member truncated) and a writer failure on rank 0 alone are raised on EVERY rank (error
    agreement after the reads / at the end of collective_output), so no peer walks into the next
    collective and hangs until the process-group timeout; a write that fails inside a body which
    also makes collective calls (outpost_ks) is deferred by the WriteGuard, so the ranks stay in
    lock-step until that agreement."""
    world = 3
    out = mp.Manager().dict()
    mp.spawn(_one_rank_fails_worker, args=(world, _free_port(), str(tmp_path), out), nprocs=world, join=True)
    for r in range(world):
        assert out[r][:3] == [("ValueError", True), ("raised", True), ("OSError", True)], (r, out[r])
        assert out[r][3] == ("OSError", True, [] if r == 1 else [0, 1, 2]), (r, out[r])
