"""Checkpoint / field-file I/O of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/ may use this module, as the checker of the product's checkpoint/restart
(nekstab_next_amd/checkpoint.py, fld.py): it is an independent restatement (struct-level byte
layout, its own Lagrange interpolation), written without importing the product, so a symmetric
misreading of the format by the product's own writer and reader cannot pass unnoticed.

What it restates (reference file:line):

* ``arnoldi_checkpoint`` (core/eigensolvers.f90:758-857): after Arnoldi step k, the new Krylov
  vector Q(k+1) goes to the field file ``KRY<session>0.f<k+1>`` (``whereyouwant("KRY", k+1)``,
  core/IO.f90:2-10, then Nek5000 ``outpost2``) and the Hessenberg matrix to ``HES<session><k:04d>``
  with the list-directed ``write (67, *) ((H(i, j), j=1, k), i=1, k+1)`` (:837) — one record,
  row-major over (k+1) x k.  The list-directed layout emitted here is gfortran's (17 significant
  digits, E-format with a three-digit exponent outside [0.1, 1e16), records wrapped at 80 columns),
  a different text form from the product's writer (one ``%.17E`` value per line) on purpose.
* the restart read (eigensolvers.f90:240-285): ``read (67, *) ((H(i, j), j=1, mstart), i=1,
  mstart+1)`` — list-directed, so any whitespace/comma layout and ``r*c`` repeat counts parse;
  then ``mstart = mstart + 1`` and ``load_files(Q, mstart, k_dim+1, 'KRY')`` (core/IO.f90:12-73)
  reads KRY 1..mstart into Q(1..mstart): velocity, pressure (``if (ifpo)``) and the scalars — not
  the ``time`` component of the Krylov vector, which a field file does not carry.
* Nek5000 ``#std`` field files (the format of the reference's own ``BF_1cyl0.f00001``; Nek5000 is
  external): 132-byte ASCII header, float32 endian tag 6.54321, int32 global element ids, then per
  field group element after element (U: ldim components per element; P, T: one block).  Pressure
  is written on the velocity (GLL, lx1) mesh and mapped back to the lx2 Gauss mesh on read
  (Nek5000's ``mappr`` / ``map21``), exact on the polynomials the lx2 mesh carries.
"""
from __future__ import annotations

import os
import struct

import numpy as np

# ---- 1-D nodes and Lagrange interpolation (independent of nekstab_next_amd/fld.py) -------------


def _gll_nodes(n):
    """Gauss–Lobatto–Legendre nodes: -1, the roots of P'_{n-1}, 1 (Newton on the Chebyshev guess)."""
    N = n - 1
    x = -np.cos(np.pi * np.arange(n) / N)
    for _ in range(100):
        P = np.zeros((n, N + 1))
        P[:, 0], P[:, 1] = 1.0, x
        for k in range(2, N + 1):
            P[:, k] = ((2 * k - 1) * x * P[:, k - 1] - (k - 1) * P[:, k - 2]) / k
        dx = (x * P[:, N] - P[:, N - 1]) / (n * P[:, N])
        x = x - dx
        if np.max(np.abs(dx)) < 1e-16:
            break
    x[0], x[-1] = -1.0, 1.0
    return x


def _gauss_nodes(n):
    return np.polynomial.legendre.leggauss(n)[0]


def _lagrange(src, dst):
    """Barycentric Lagrange interpolation matrix, len(dst) x len(src)."""
    bw = np.array([1.0 / np.prod([src[j] - src[m] for m in range(len(src)) if m != j]) for j in range(len(src))])
    M = np.zeros((len(dst), len(src)))
    for i, x in enumerate(dst):
        d = x - src
        hit = np.nonzero(np.abs(d) < 1e-15)[0]
        if hit.size:
            M[i, hit[0]] = 1.0
            continue
        t = bw / d
        M[i] = t / t.sum()
    return M


def _tensor(M, blocks, ldim):
    """Apply the 1-D matrix M along every direction of per-element blocks [nel, n^ldim] (x fastest)."""
    nel, n = blocks.shape[0], M.shape[1]
    out = blocks.reshape((nel,) + (n,) * ldim)
    for ax in range(ldim):
        out = np.moveaxis(np.tensordot(out, M, axes=([ldim - ax], [1])), -1, ldim - ax)
    return out.reshape(nel, -1)


# ---- geometry of one shard ---------------------------------------------------------------------

class Geom:
    """Spectral-element facts of the vector (SIZE): ldim, lx1, lx2, global elements, the first
    global element of this shard and its element count, active scalars."""

    def __init__(self, ldim, lx1, lx2, nelgv, e0=0, nelv=None, n_scalars=0):
        self.ldim, self.lx1, self.lx2, self.nelgv = ldim, lx1, lx2, nelgv
        self.e0, self.nelv = e0, (nelgv if nelv is None else nelv)
        self.n_scalars = n_scalars
        self.p1 = lx1 ** ldim
        self.p2 = lx2 ** ldim
        self.nv = self.p1 * self.nelv
        self.np = self.p2 * self.nelv


def _slices(g: Geom):
    """Reference-order segments of a krylov_vector: vx, vy, [vz], t.., pr (then time)."""
    names = ["vx", "vy", "vz"][: g.ldim] + ["t"] + [f"s{i:02d}" for i in range(1, g.n_scalars)]
    names = names[: g.ldim + g.n_scalars]
    out, o = [], 0
    for nm in names:
        out.append((nm, o, g.nv))
        o += g.nv
    out.append(("pr", o, g.np))
    return out


# ---- Nek5000 #std files ------------------------------------------------------------------------

def write_std(path, g: Geom, vec_ref, time=0.0, istep=0, fid=0, nfileo=1):
    """outpost2 of a reference-order vector: groups U, P, T (, S01..) in 64-bit, little endian."""
    seg = {nm: vec_ref[o:o + n] for nm, o, n in _slices(g)}
    nel, nz = g.nelv, (g.lx1 if g.ldim == 3 else 1)
    rd = "UP" + ("T" if g.n_scalars else "") + "".join(f"S{i:02d}" for i in range(1, g.n_scalars))
    head = "#std 8 %2d %2d %2d %10d %10d %20.13E %9d %6d %6d %s" % (
        g.lx1, g.lx1, nz, nel, g.nelgv, time, istep, fid, nfileo, rd)
    blob = [head.ljust(132).encode("ascii"), struct.pack("<f", 6.54321),
            struct.pack("<%di" % nel, *range(g.e0 + 1, g.e0 + nel + 1))]
    vel = np.stack([seg[c].reshape(nel, g.p1) for c in ["vx", "vy", "vz"][: g.ldim]], axis=1)
    blob.append(vel.astype("<f8").tobytes())
    p2 = seg["pr"].reshape(nel, g.p2)
    p1 = _tensor(_lagrange(_gauss_nodes(g.lx2), _gll_nodes(g.lx1)), p2, g.ldim)
    blob.append(p1.astype("<f8").tobytes())
    for s in range(g.n_scalars):
        blob.append(seg["t" if s == 0 else f"s{s:02d}"].reshape(nel, g.p1).astype("<f8").tobytes())
    with open(path, "wb") as fh:
        fh.write(b"".join(blob))


def read_std(path):
    """(header tokens, element ids (1-based), {field: [nel, pts]}) of a #std file."""
    raw = open(path, "rb").read()
    tok = raw[:132].decode("ascii").split()
    wd, nx, ny, nz, nel = (int(t) for t in tok[1:6])
    bo = "<" if abs(struct.unpack("<f", raw[132:136])[0] - 6.54321) < 1e-5 else ">"
    ids = np.array(struct.unpack("%s%di" % (bo, nel), raw[136:136 + 4 * nel]))
    pts, ldim = nx * ny * nz, (3 if nz > 1 else 2)
    off, fields, rd, i = 136 + 4 * nel, {}, tok[11], 0
    while i < len(rd):
        grp = rd[i:i + 3] if rd[i] == "S" else rd[i]
        i += len(grp)
        nc = ldim if grp in ("X", "U") else 1
        cnt = nel * nc * pts
        v = np.array(struct.unpack("%s%d%s" % (bo, cnt, "d" if wd == 8 else "f"), raw[off:off + cnt * wd]))
        off += cnt * wd
        v = v.reshape(nel, nc, pts)
        names = {"X": ["x", "y", "z"], "U": ["vx", "vy", "vz"], "P": ["pr"], "T": ["t"]}.get(grp, [grp.lower()])
        for c in range(nc):
            fields[names[c]] = v[:, c, :]
    return tok, ids, fields


def read_std_vector(paths, g: Geom):
    """load_fld + the opcopy / copy of load_files (core/IO.f90:63-70) into a reference-order vector
    of this shard (time slot 0).  ``paths``: the files of one output number (multi-file sets)."""
    out = np.zeros(g.nv * (g.ldim + g.n_scalars) + g.np + 1)
    M21 = _lagrange(_gll_nodes(g.lx1), _gauss_nodes(g.lx2))
    for p in paths:
        _, ids, fields = read_std(p)
        loc = ids - 1 - g.e0
        keep = np.nonzero((loc >= 0) & (loc < g.nelv))[0]
        for nm, o, n in _slices(g):
            if nm not in fields:
                continue
            if nm == "pr":
                blk = _tensor(M21, fields["pr"][keep], g.ldim)
                seg = out[o:o + n].reshape(g.nelv, g.p2)
            else:
                blk = fields[nm][keep]
                seg = out[o:o + n].reshape(g.nelv, g.p1)
            seg[loc[keep]] = blk
    return out


def kry_name(session, num, fid=0, prefix="KRY"):
    return f"{prefix}{session}{fid}.f{num:05d}"


# ---- list-directed Hessenberg text ---------------------------------------------------------------

def _gfortran_real8(x: float) -> str:
    """One real(8) item as gfortran's list-directed output writes it (17 significant digits)."""
    if x == 0.0:
        return "   0.0000000000000000     "
    ax = abs(x)
    if 0.1 <= ax < 1e16:
        e = int(np.floor(np.log10(ax))) + 1          # digits before the point
        s = f"{x:.{max(17 - e, 0)}f}"
        return f"{s:>23}     "
    m, ex = f"{x:.16E}".split("E")
    return f"{m}E{int(ex):+04d}".rjust(26)


def write_hes_list_directed(path, H, k):
    """``write (67, *) ((H(i, j), j=1, k), i=1, k+1)`` — one list-directed record, wrapped."""
    items = [_gfortran_real8(float(H[i, j])) for i in range(k + 1) for j in range(k)]
    lines, cur = [], ""
    for it in items:
        if len(cur) + len(it) > 80:
            lines.append(cur)
            cur = ""
        cur += it
    lines.append(cur)
    with open(path, "w") as fh:
        fh.write("\n".join(" " + ln for ln in lines) + "\n")


def read_list_directed(path, count):
    """The first ``count`` items of a list-directed real read (separators: blanks, commas, line
    ends; ``r*c`` repeat counts)."""
    vals = []
    for tok in open(path).read().replace(",", " ").split():
        if "*" in tok:
            r, c = tok.split("*")
            vals += [float(c)] * int(r)
        else:
            vals.append(float(tok.replace("D", "E").replace("d", "e")))
        if len(vals) >= count:
            break
    if len(vals) < count:
        raise ValueError(f"{path}: {len(vals)} values, {count} expected")
    return np.array(vals[:count])


def read_hes(path, mstart, k_dim):
    """The restart read of H (eigensolvers.f90:261-263): rows 1..mstart+1, cols 1..mstart of a
    (k_dim+1) x k_dim zero matrix, row-major.  mstart > k_dim is the reference's (1E15.7)
    "subsampling" branch (:250-256), which reads one 15-column field per record and so cannot
    read the several-per-record file arnoldi_checkpoint writes: refused here as in the product."""
    if mstart > k_dim:
        raise ValueError(f"mstart={mstart} > k_dim={k_dim}: the reference's subsampling read is not restated")
    H = np.zeros((k_dim + 1, k_dim))
    H[: mstart + 1, :mstart] = read_list_directed(path, (mstart + 1) * mstart).reshape(mstart + 1, mstart)
    return H


def hes_name(session, k):
    return f"HES{session}{k:04d}"


def checkpoint_writer(directory, session, g: Geom, fid=0, nfileo=1):
    """``on_step(mstep, Q, H)`` hook for oracle.krylov_schur: arnoldi_checkpoint's KRY + HES files
    (Q(1) at the first step, as eigensolvers.f90:235-236 writes it when the run starts)."""
    os.makedirs(directory, exist_ok=True)

    def hook(k, Q, H):
        if k == 1:
            write_std(os.path.join(directory, kry_name(session, 1, fid)), g, Q[0], 0.0, 1, fid, nfileo)
        write_std(os.path.join(directory, kry_name(session, k + 1, fid)), g, Q[k], float(k), k + 1, fid, nfileo)
        if fid == 0:
            write_hes_list_directed(os.path.join(directory, hes_name(session, k)), H, k)
    return hook


def load_restart(directory, session, g: Geom, mstart, k_dim, nfiles=1):
    """(H, Q[0:mstart+1]) as the reference's restart branch builds them (eigensolvers.f90:240-285)."""
    H = read_hes(os.path.join(directory, hes_name(session, mstart)), mstart, k_dim)
    Q = [read_std_vector([os.path.join(directory, kry_name(session, i, f)) for f in range(nfiles)], g)
         for i in range(1, mstart + 2)]
    return H, np.array(Q)
