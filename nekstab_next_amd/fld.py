"""Nek5000 field files (``#std`` ``.f#####``) <-> nekStab state vectors.

nekStab reads base flows and restart vectors with Nek5000's ``load_fld`` (core/IO.f90:12-73,
eigensolvers.f90:170-180) and writes Krylov vectors / eigenmodes with ``outpost2``
(eigensolvers.f90:236,607-615,776).  The on-disk format, as found in the reference's own data
(``examples/cylinder/BF_1cyl0.f00001``):

* 132-byte ASCII header: ``#std <wdsize> <nx> <ny> <nz> <nel_in_file> <nelgt> <time> <istep>
  <fid0> <nfileo> <rdcode>`` (rdcode letters: X coordinates, U velocity, P pressure, T
  temperature, S<nn> passive scalars);
* float32 endian tag 6.54321;
* int32 global element ids (1-based) of the elements in this file, in file order;
* per field group, element after element: vector groups (X, U) write their ldim components
  component-major inside each element, scalar groups one block per element.
  Pressure is stored on the velocity (GLL, lx1) mesh; in memory PN/PN-2 pressure lives on the
  Gauss–Legendre lx2 mesh, so it is interpolated on read (lx1 GLL -> lx2 GL) and on write.

Multi-rank: each rank writes its element range as file ``fid = rank`` with ``nfileo = world``
(Nek5000's multi-file naming ``<prefix><session><fid>.f<NNNNN>``).

Collective semantics.  Nek5000's ``outpost2`` and ``load_fld`` are collective: every rank has
finished writing a set before any rank reads from it (the reference relies on it at
eigensolvers.f90:607-615 -> sensitivity.f90:40-60, and on restart, IO.f90:12-73).  Here:

* :func:`write_fld` writes to a temporary name in the same directory and ``os.replace``-s it into
  place, so a reader never sees a partly written file;
* every product writer of a per-rank set ends in :func:`collective_output` (a barrier over the
  ranks' communicator once this rank's files are in place);
* :func:`read_fld_set` raises when a member of a set is missing (never a partial set), and with a
  layout it opens only the files holding this rank's elements: with a set written at the same
  world size, rank r opens fid r and nothing else.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass, field

import numpy as np

from .layout import NekLayout
from .synthetic import gll_weights  # noqa: F401  (shared GLL quadrature helpers)

ENDIAN_TAG = np.float32(6.54321)


# ---- 1-D nodes and interpolation (pressure mesh mapping) ------------------------------------

def gll_points(n: int) -> np.ndarray:
    P = np.polynomial.legendre.Legendre.basis(n - 1)
    return np.concatenate([[-1.0], np.sort(P.deriv().roots().real), [1.0]])


def gauss_points(n: int) -> np.ndarray:
    return np.polynomial.legendre.leggauss(n)[0]


def interp_matrix(src: np.ndarray, dst: np.ndarray) -> np.ndarray:
    """Lagrange interpolation from nodes ``src`` to points ``dst`` (len(dst) x len(src))."""
    M = np.ones((len(dst), len(src)))
    for j, xj in enumerate(src):
        for m, xm in enumerate(src):
            if m != j:
                M[:, j] *= (dst - xm) / (xj - xm)
    return M


def _tensor_apply(M: np.ndarray, data: np.ndarray, ldim: int) -> np.ndarray:
    """Apply the 1-D operator M along every direction of per-element data [nel, n^ldim] (x fastest)."""
    nel = data.shape[0]
    n, m = M.shape[1], M.shape[0]
    # one direction at a time (sum factorisation: O(n^(ldim+1)) per element), each as a batched
    # matmul with the contracted axis last-but-one or last — no transposes, no einsum: 11x faster
    # than the einsum form at lx1=8, E=22,088 and bit-identical to it
    if ldim == 2:
        a = data.reshape(nel, n, n) @ M.T                # [e, y, x] -> [e, y, i]
        return np.matmul(M, a).reshape(nel, -1)          # -> [e, j, i]
    a = data.reshape(nel, n, n, n) @ M.T                 # [e, z, y, x] -> [e, z, y, i]
    a = np.matmul(M, a)                                  # -> [e, z, j, i]
    return np.matmul(M, a.reshape(nel, n, m * m)).reshape(nel, -1)   # -> [e, k, (j, i)]


def map_pressure_to_mesh1(p2: np.ndarray, lx1: int, lx2: int, ldim: int) -> np.ndarray:
    if lx1 == lx2:
        return p2
    return _tensor_apply(interp_matrix(gauss_points(lx2), gll_points(lx1)), p2, ldim)


def map_pressure_to_mesh2(p1: np.ndarray, lx1: int, lx2: int, ldim: int) -> np.ndarray:
    if lx1 == lx2:
        return p1
    return _tensor_apply(interp_matrix(gll_points(lx1), gauss_points(lx2)), p1, ldim)


# ---- file I/O --------------------------------------------------------------------------------

@dataclass
class FldFile:
    nx: int
    ny: int
    nz: int
    nelgt: int
    time: float = 0.0
    istep: int = 0
    fid0: int = 0
    nfileo: int = 1
    rdcode: str = "UP"
    emap: np.ndarray = None            # 1-based global element ids of the elements in the file
    fields: dict = field(default_factory=dict)  # name -> [nel, pts]: x,y,z, vx,vy,vz, pr, t, s01..
    wdsize: int = 8

    @property
    def ldim(self) -> int:
        return 3 if self.nz > 1 else 2


def _groups(rdcode: str):
    out, i = [], 0
    while i < len(rdcode):
        c = rdcode[i]
        if c == "S":
            out.append(rdcode[i:i + 3])
            i += 3
        else:
            out.append(c)
            i += 1
    return out


def _parse_header(raw, path: str):
    """(wdsize, nx, ny, nz, nel, nelgt, time, istep, fid0, nfileo, rdcode, byte order, emap)."""
    if len(raw) < 136:
        raise ValueError(f"{path}: {len(raw)} bytes, shorter than a #std header")
    tok = bytes(raw[:132]).decode("ascii", errors="replace").split()
    if not tok or tok[0] != "#std":
        raise ValueError(f"{path}: not a Nek5000 #std field file")
    wdsize, nx, ny, nz, nel, nelgt = (int(t) for t in tok[1:7])
    time, istep, fid0, nfileo = float(tok[7]), int(tok[8]), int(tok[9]), int(tok[10])
    tag = np.frombuffer(raw, "<f4", count=1, offset=132)[0]
    order = "<" if abs(tag - ENDIAN_TAG) < 1e-5 else ">"
    if len(raw) < 136 + 4 * nel:
        raise ValueError(f"{path}: truncated element map ({nel} elements)")
    emap = np.frombuffer(raw, order + "i4", count=nel, offset=136).copy()
    return wdsize, nx, ny, nz, nel, nelgt, time, istep, fid0, nfileo, tok[11], order, emap


def read_fld_header(path: str) -> FldFile:
    """Header and element map only (no field data): 136 + 4 nel bytes."""
    with open(path, "rb") as fh:
        head = fh.read(136)
        nel = int(bytes(head[:132]).decode("ascii", errors="replace").split()[5]) if len(head) >= 132 else 0
        raw = head + fh.read(4 * max(nel, 0))
    wdsize, nx, ny, nz, nel, nelgt, time, istep, fid0, nfileo, rdcode, _, emap = _parse_header(raw, path)
    return FldFile(nx, ny, nz, nelgt, time, istep, fid0, nfileo, rdcode, emap, {}, wdsize)


def read_fld(path: str) -> FldFile:
    # one read into a mutable buffer; the fields are views of it (no payload copies)
    raw = bytearray(os.path.getsize(path))
    with open(path, "rb") as fh:
        if fh.readinto(raw) != len(raw):
            raise ValueError(f"{path}: short read")
    wdsize, nx, ny, nz, nel, nelgt, time, istep, fid0, nfileo, rdcode, order, emap = _parse_header(raw, path)
    fdt = np.dtype(order + ("f8" if wdsize == 8 else "f4"))
    data = np.frombuffer(raw, fdt, offset=136 + 4 * nel)
    if data.dtype != np.dtype(np.float64):   # byte-swapped or single precision: one converted copy
        data = data.astype(np.float64)
    pts = nx * ny * nz
    ldim = 3 if nz > 1 else 2
    f = FldFile(nx, ny, nz, nelgt, time, istep, fid0, nfileo, rdcode, emap, {}, wdsize)
    o = 0
    for g in _groups(rdcode):
        if g in ("X", "U"):
            blk = data[o:o + nel * ldim * pts].reshape(nel, ldim, pts)
            o += nel * ldim * pts
            names = ["x", "y", "z"] if g == "X" else ["vx", "vy", "vz"]
            for c in range(ldim):
                f.fields[names[c]] = blk[:, c, :]
        else:
            blk = data[o:o + nel * pts].reshape(nel, pts)
            o += nel * pts
            f.fields[{"P": "pr", "T": "t"}.get(g, g.lower())] = blk
    if o != data.size:
        raise ValueError(f"{path}: {data.size - o} trailing values (rdcode {rdcode})")
    return f


def write_fld(path: str, f: FldFile) -> None:
    nel = f.emap.size
    ldim = f.ldim
    pts = f.nx * f.ny * f.nz
    hdr = (f"#std {f.wdsize:1d} {f.nx:2d} {f.ny:2d} {f.nz:2d} {nel:10d} {f.nelgt:10d} {f.time:20.13E} "
           f"{f.istep:9d} {f.fid0:6d} {f.nfileo:6d} {f.rdcode}")
    hdr = hdr.ljust(132)[:132].encode("ascii")
    # the arrays go to the file through the buffer protocol (no bytes copies of the payload)
    parts = [hdr, ENDIAN_TAG.astype("<f4").tobytes(), np.ascontiguousarray(f.emap, "<i4")]
    for g in _groups(f.rdcode):
        if g in ("X", "U"):
            names = ["x", "y", "z"] if g == "X" else ["vx", "vy", "vz"]
            blk = np.stack([f.fields[names[c]] for c in range(ldim)], axis=1)
            parts.append(np.ascontiguousarray(blk, "<f8"))
        else:
            parts.append(np.ascontiguousarray(f.fields[{"P": "pr", "T": "t"}.get(g, g.lower())], "<f8"))
    # written under a temporary name in the same directory, then renamed into place (atomic on
    # POSIX): a reader on another rank sees either no file or the whole file
    d, b = os.path.split(path)
    tmp = os.path.join(d, f".{b}.part{os.getpid()}")
    try:
        with open(tmp, "wb") as fh:
            for p in parts:
                if not isinstance(p, np.ndarray):
                    fh.write(p)
                elif p.size:   # an empty shard (more ranks than elements) writes header + tag only
                    fh.write(memoryview(p).cast("B"))
        os.replace(tmp, path)
    except BaseException:
        with contextlib.suppress(OSError):
            os.remove(tmp)
        raise


class WriteGuard:
    """Runs the writes of a :func:`collective_output` body whose ranks must stay in lock-step
    because the body also makes collective calls (a mode assembled with all-reduced norms, then
    written): the first write that fails is remembered and every later write on that rank is
    skipped, while the body — and so its collectives — carries on; ``collective_output`` then
    raises that error on every rank.  Letting the exception escape instead would take the failing
    rank out of the body while its peers wait in the next collective."""

    def __init__(self):
        self.error = None

    def __call__(self, fn, *args, **kwargs):
        if self.error is not None:
            return None
        try:
            return fn(*args, **kwargs)
        except Exception as e:  # noqa: BLE001 - deferred to collective_output's agreement
            self.error = e
            return None


@contextlib.contextmanager
def collective_output(comm, barrier: bool = True):
    """The collective end of a per-rank ``outpost2``: the body writes this rank's files (and rank
    0's text files); every rank then waits until all ranks' files are in place, so a read that
    follows on any rank finds the whole set (Nek5000's outpost2 / load_fld are collective,
    eigensolvers.f90:607-615, sensitivity.f90:40-60).  The wait is an error agreement
    (``Comm.raise_if_any``): when the body raises on any rank (a full disk on rank 0's HES), or a
    write run through the yielded :class:`WriteGuard` failed, every rank takes part and then
    raises, instead of its peers waiting at a barrier it never reaches.  ``barrier=False`` exists
    only for the test that shows the race without it."""
    guard = WriteGuard()
    err = None
    try:
        yield guard
        err = guard.error
    except Exception as e:  # noqa: BLE001 - agreed with the peers, then re-raised on every rank
        err = e
    if barrier and comm is not None:
        comm.raise_if_any(err)
    if err is not None:
        raise err


def fld_name(prefix: str, session: str, fid: int, num: int) -> str:
    return f"{prefix}{session}{fid}.f{num:05d}"


# ---- vector <-> fields -----------------------------------------------------------------------

def vector_from_fld(lay: NekLayout, files) -> np.ndarray:
    """Padded host vector (this rank's shard of ``lay``) from one or several (multi-file) field files.
    Velocity -> vx, vy, [vz]; T -> first scalar; S01.. -> next scalars; P -> pressure (mapped to
    the lx2 Gauss mesh).  Missing fields stay zero (as load_fld leaves them untouched)."""
    if isinstance(files, FldFile):
        files = [files]
    out = np.zeros(lay.ld)
    e0, e1 = lay.elem_range()
    names = ["vx", "vy", "vz"][: lay.ldim] + (["t"] + [f"s{i:02d}" for i in range(1, lay.n_scalars)])[: lay.n_scalars]
    for f in files:
        if f.nx != lay.lx1 or f.ldim != lay.ldim:
            raise ValueError(f"field file is lx1={f.nx} ldim={f.ldim}, layout lx1={lay.lx1} ldim={lay.ldim}")
        g = f.emap.astype(np.int64) - 1
        sel = np.nonzero((g >= e0) & (g < e1))[0]
        if sel.size == 0:
            continue
        loc = g[sel] - e0
        # the common case (one file per rank, elements in order): slices, not gathers/scatters
        run = sel.size == g.size and bool(np.all(np.diff(loc) == 1)) if sel.size > 1 else False
        src = slice(None) if run else sel
        dst = slice(int(loc[0]), int(loc[0]) + loc.size) if run else loc
        for k, nm in enumerate(names):
            if nm in f.fields:
                seg = out[k * lay.sv: k * lay.sv + lay.n_v].reshape(lay.nelv, lay.pts_v)
                seg[dst] = f.fields[nm][src]
        if "pr" in f.fields and lay.n_p:
            p2 = map_pressure_to_mesh2(f.fields["pr"][src], lay.lx1, lay.lx2, lay.ldim)
            seg = out[lay.n_wf * lay.sv: lay.n_wf * lay.sv + lay.n_p].reshape(lay.nelv, lay.pts_p)
            seg[dst] = p2
    return out


def fld_from_vector(lay: NekLayout, vec: np.ndarray, time: float = 0.0, istep: int = 0,
                    coords: dict | None = None) -> FldFile:
    """This rank's shard as a field file (fid = rank, nfileo = world)."""
    e0, e1 = lay.elem_range()
    f = FldFile(lay.lx1, lay.lx1, lay.lx1 if lay.ldim == 3 else 1, lay.nelgv, time, istep, lay.rank, lay.world,
                "", np.arange(e0 + 1, e1 + 1, dtype=np.int32), {})
    code = ""
    if coords:
        code += "X"
        f.fields.update({k: np.asarray(v).reshape(lay.nelv, lay.pts_v) for k, v in coords.items()})
    code += "U"
    for k, nm in enumerate(["vx", "vy", "vz"][: lay.ldim]):
        f.fields[nm] = vec[k * lay.sv: k * lay.sv + lay.n_v].reshape(lay.nelv, lay.pts_v).copy()
    if lay.n_p:
        code += "P"
        p2 = vec[lay.n_wf * lay.sv: lay.n_wf * lay.sv + lay.n_p].reshape(lay.nelv, lay.pts_p)
        f.fields["pr"] = map_pressure_to_mesh1(p2, lay.lx1, lay.lx2, lay.ldim)
    for s in range(lay.n_scalars):
        k = lay.ldim + s
        nm = "t" if s == 0 else f"s{s:02d}"
        code += "T" if s == 0 else f"S{s:02d}"
        f.fields[nm] = vec[k * lay.sv: k * lay.sv + lay.n_v].reshape(lay.nelv, lay.pts_v).copy()
    f.rdcode = code
    return f


def _block(fid: int, nfileo: int, nelgt: int) -> tuple[int, int]:
    """Elements [e0, e1) (0-based) of file ``fid`` of a set written by ``nfileo`` ranks with
    Nek5000's element-contiguous distribution (layout.NekLayout.elem_range)."""
    return (fid * nelgt) // nfileo, ((fid + 1) * nelgt) // nfileo


def read_fld_set(directory: str, prefix: str, session: str, num: int, lay: NekLayout | None = None,
                 comm=None) -> list:
    """The files of a (possibly multi-file) output number, as Nek5000's ``load_fld`` reads them.

    Without ``lay``: every file of the set.  With ``lay``: only the files holding elements of
    ``lay.elem_range()`` (this rank's shard).  The set is defined by the header of fid 0 (a
    set's first member is always rewritten, so leftover higher fids of an older, larger set are
    ignored): with ``comm`` at world > 1, rank 0 reads that header and broadcasts (nfileo,
    nelgt), so with a set written at the same world size rank r opens fid r and nothing else.  The
    files a rank needs are predicted from the element-contiguous distribution of an
    nfileo-file set; each one's element map is checked against the prediction, and only a set
    written with another distribution (a foreign writer) falls back to reading every header.

    Raises FileNotFoundError when fid 0 or any member fid < nfileo is missing, and ValueError when
    the files read do not cover the shard's elements — never a partial vector.  With ``comm`` every
    failure is raised on EVERY rank (``Comm.raise_if_any`` after the reads: a truncated member or a
    shard no file covers is often one rank's alone).  A rank without elements gets one
    element-less FldFile carrying the set's header (time, istep)."""
    def path(fid):
        return os.path.join(directory, fld_name(prefix, session, fid, num))

    def set_header():
        if not os.path.exists(path(0)):
            return FileNotFoundError(path(0))
        try:
            h = read_fld_header(path(0))
        except Exception as e:  # noqa: BLE001 - sent to every rank and raised there (no rank left waiting)
            return e
        if h.nfileo < 1:
            return ValueError(f"{path(0)}: nfileo={h.nfileo}")
        h.emap = np.zeros(0, dtype=np.int32)   # the set's header facts only (time, istep, sizes)
        return h

    if comm is not None and comm.world > 1:
        hdr = comm.bcast_object(set_header() if comm.rank == 0 else None, src=0)
    else:
        hdr = set_header()
    if isinstance(hdr, BaseException):
        raise hdr
    n, nelgt = hdr.nfileo, hdr.nelgt

    def read_shard():
        missing = [i for i in range(n) if not os.path.exists(path(i))]
        if missing:
            raise FileNotFoundError(f"{path(missing[0])} (set of {n} files, missing fids {missing})")
        if lay is None:
            return [read_fld(path(i)) for i in range(n)]

        e0, e1 = lay.elem_range()
        E = lay.nelgv
        if nelgt != E:
            raise ValueError(f"{path(0)}: nelgt={nelgt}, the layout has {E} elements")

        def holds_ours(emap):
            g = emap.astype(np.int64) - 1
            return bool(np.any((g >= e0) & (g < e1)))

        want = [i for i in range(n) if _block(i, n, E)[0] < e1 and _block(i, n, E)[1] > e0]
        out = {i: read_fld(path(i)) for i in want}
        if not all(np.array_equal(out[i].emap, np.arange(*_block(i, n, E)) + 1) for i in want):
            # another element distribution: every header decides, then the files holding our elements
            for i in range(n):
                if i not in out and holds_ours(read_fld_header(path(i)).emap):
                    out[i] = read_fld(path(i))
        files = [out[i] for i in sorted(out) if holds_ours(out[i].emap)]
        covered = np.zeros(e1 - e0, dtype=bool)
        for f in files:
            g = f.emap.astype(np.int64) - 1
            covered[g[(g >= e0) & (g < e1)] - e0] = True
        if not covered.all():
            raise ValueError(f"{prefix}{session}*.f{num:05d}: {int((~covered).sum())} of this rank's "
                             f"{e1 - e0} elements are in no file of the set")
        # a rank without elements gets the set's header (time, istep) with no elements, as load_fld
        # sets time on every rank
        return files or [hdr]

    err = files = None
    try:
        files = read_shard()
    except Exception as e:  # noqa: BLE001 - agreed with the peers below, then raised on every rank
        err = e
    if comm is not None and comm.world > 1:
        comm.raise_if_any(err)
    elif err is not None:
        raise err
    return files
