"""Spectral-element state-vector geometry (the SIZE / TOTAL facts nekStab's vectors are sized by).

Reference: ``krylov_vector`` / ``real_nek_vector`` hold ``vx, vy, vz(lv)``, ``pr(lp)``,
``t(lv, ldimt)`` and a scalar ``time`` (core/krylov_subspace.f90:7-17, core/nek_vectors.f90:16-31)
with ``lv = lx1*ly1*lz1*lelv`` and ``lp = lx2*ly2*lz2*lelv``.  Only vx, vy, [vz] and the active
scalars enter the weighted dot (k_dot, krylov_subspace.f90:40-50); pressure is stored and carried
by every BLAS-1 op but never dotted.

Sharding follows Nek5000's element distribution: rank r owns the element-contiguous block
``[r*E//P, (r+1)*E//P)`` and every field/pressure/weight of those elements.
"""
from __future__ import annotations

from dataclasses import dataclass

NKV_TILE = 4096  # include/nekkrylov.h


def _roundup(n: int, m: int) -> int:
    return ((n + m - 1) // m) * m


@dataclass(frozen=True)
class NekLayout:
    """Geometry of one nekStab state vector, optionally restricted to one rank's shard.

    ldim      : 2 or 3 (``if3d``)
    lx1, lx2  : GLL points per direction for velocity / pressure (``lx2 = lx1 - 2`` for PN-PN-2)
    nelgv     : global number of velocity elements
    n_scalars : active scalar fields in the dot (``ifto`` + ``ifpsco(:)``), 0 for pure flow
    ifpo      : pressure stored (``ifpo``); when False the pressure segment is empty
    rank/world: this shard of an element-contiguous partition
    nelgt     : global number of temperature/scalar elements (Nek5000's ``nelgt``), None = nelgv.
                Only ``nelgt == nelgv`` is supported when a scalar is dotted: conjugate heat
                transfer (``nelt > nelv``) is refused, see ``__post_init__``.
    """

    ldim: int
    lx1: int
    lx2: int
    nelgv: int
    n_scalars: int = 0
    ifpo: bool = True
    rank: int = 0
    world: int = 1
    nelgt: int | None = None

    def __post_init__(self):
        if self.ldim not in (2, 3):
            raise ValueError("ldim must be 2 or 3")
        if self.lx1 < 2 or self.lx2 < 1 or self.nelgv < 0 or self.n_scalars < 0:
            raise ValueError("bad layout parameters")
        if not (0 <= self.rank < self.world):
            raise ValueError("rank out of range")
        if self.nelgt is not None and self.nelgt != self.nelgv and self.n_scalars > 0:
            # the reference dots a scalar over nt = nx1*ny1*nz1*nelt points with the velocity-mesh
            # weights bm1s(lx1,ly1,lz1,lelv) (core/krylov_subspace.f90:36-44, nek_vectors.f90:88-99;
            # bm1s declared at core/NEKSTAB:86): with nelt > nelv it reads past bm1s, so there is no
            # reference result to reproduce.  Every weighted field here has n_v points and shares one
            # weight array; such a layout is refused rather than given a made-up meaning.
            raise ValueError(f"nelgt={self.nelgt} != nelgv={self.nelgv} with {self.n_scalars} dotted scalar(s): "
                             "conjugate heat transfer layouts (nelt > nelv) are not supported — the reference "
                             "weights the scalar over nelt elements with the nelv-element bm1s "
                             "(krylov_subspace.f90:36-44, NEKSTAB:86)")

    # ---- per element ------------------------------------------------------------------------
    @property
    def pts_v(self) -> int:
        return self.lx1 ** self.ldim

    @property
    def pts_p(self) -> int:
        return self.lx2 ** self.ldim if self.ifpo else 0

    @property
    def n_wf(self) -> int:
        """Weighted fields: vx, vy, [vz], scalars."""
        return self.ldim + self.n_scalars

    # ---- shard --------------------------------------------------------------------------------
    def elem_range(self, rank: int | None = None) -> tuple[int, int]:
        r = self.rank if rank is None else rank
        return (r * self.nelgv) // self.world, ((r + 1) * self.nelgv) // self.world

    def shard(self, rank: int, world: int) -> "NekLayout":
        return NekLayout(self.ldim, self.lx1, self.lx2, self.nelgv, self.n_scalars, self.ifpo, rank, world,
                         self.nelgt)

    @property
    def nelv(self) -> int:
        e0, e1 = self.elem_range()
        return e1 - e0

    @property
    def n_v(self) -> int:
        return self.pts_v * self.nelv

    @property
    def n_p(self) -> int:
        return self.pts_p * self.nelv

    @property
    def v_offset(self) -> int:
        return self.pts_v * self.elem_range()[0]

    @property
    def p_offset(self) -> int:
        return self.pts_p * self.elem_range()[0]

    # ---- padded device storage (include/nekkrylov.h) ------------------------------------------
    @property
    def sv(self) -> int:
        return _roundup(self.n_v, NKV_TILE)

    @property
    def sp(self) -> int:
        return _roundup(self.n_p, NKV_TILE)

    @property
    def rows(self) -> int:
        """Streamed rows (weighted fields + pressure, padded); the time slot is at this offset."""
        return self.n_wf * self.sv + self.sp

    @property
    def time_offset(self) -> int:
        return self.rows

    @property
    def ld(self) -> int:
        return _roundup(self.rows + 1, NKV_TILE)

    # ---- live sizes (the algorithmic byte model) ------------------------------
    @property
    def N(self) -> int:
        """Stored doubles per vector on this shard (weighted fields + pressure)."""
        return self.n_wf * self.n_v + self.n_p

    @property
    def N_w(self) -> int:
        """Dot-participating doubles per vector on this shard."""
        return self.n_wf * self.n_v

    @property
    def N_global(self) -> int:
        return self.n_wf * self.pts_v * self.nelgv + self.pts_p * self.nelgv

    def c_struct(self, rank0: bool | None = None):
        from ._lib import nkv_layout

        return nkv_layout(
            n_v=self.n_v,
            n_p=self.n_p,
            sv=self.sv,
            sp=self.sp,
            ld=self.ld,
            n_wf=self.n_wf,
            rank0=int(self.rank == 0 if rank0 is None else rank0),
        )

    # ---- host-side field views ----------------------------------------------------------------
    def field_slices(self):
        """(name, start, live_length) of every stored segment in the padded vector."""
        names = ["vx", "vy", "vz"][: self.ldim] + [f"t{i + 1}" for i in range(self.n_scalars)]
        out = [(nm, i * self.sv, self.n_v) for i, nm in enumerate(names)]
        out.append(("pr", self.n_wf * self.sv, self.n_p))
        return out


def cylinder_layout(nelgv: int = 1996) -> NekLayout:
    """2-D cylinder example geometry: ldim=2, lx1=6, lx2=lx1-2 (examples/cylinder/SIZE:12-20)."""
    return NekLayout(ldim=2, lx1=6, lx2=4, nelgv=nelgv)


def box3d_layout(nelgv: int, n_scalars: int = 1) -> NekLayout:
    """3-D lx1=8 layout with one scalar, as SURVEY.md §8(d) config 3 (E=44,176 -> N=1.0e8)."""
    return NekLayout(ldim=3, lx1=8, lx2=6, nelgv=nelgv, n_scalars=n_scalars)


@dataclass(frozen=True)
class PairLayout(NekLayout):
    """A complex state vector ``cmplx_nek_vector{re, im}`` (core/nek_vectors.f90:33-42) stored as
    ONE real vector: in every field segment (and the pressure segment) of this rank's shard the
    ``re`` part of the base shard's elements comes first, then the ``im`` part.  The weighted dot
    of two such vectors is re.re + im.im — the cmplx dot (:164-175) — so every kernel, the
    Gram–Schmidt and the solvers run on complex vectors unchanged.  Rank r owns the pair of the
    base layout's element block: elem_range = 2 x base elem_range, for any world size."""

    base_nelgv: int = 0

    def elem_range(self, rank: int | None = None) -> tuple[int, int]:
        r = self.rank if rank is None else rank
        return 2 * ((r * self.base_nelgv) // self.world), 2 * (((r + 1) * self.base_nelgv) // self.world)

    def shard(self, rank: int, world: int) -> "PairLayout":
        return pair_layout(NekLayout(self.ldim, self.lx1, self.lx2, self.base_nelgv, self.n_scalars, self.ifpo,
                                     rank, world))

    @property
    def base(self) -> NekLayout:
        return NekLayout(self.ldim, self.lx1, self.lx2, self.base_nelgv, self.n_scalars, self.ifpo, self.rank,
                         self.world)

    def pack(self, re, im):
        """Host: padded pair vector from two padded base vectors (time: re's)."""
        import numpy as np

        b = self.base
        out = np.zeros(self.ld)
        for (_, s0, n0), (_, s1, _) in zip(b.field_slices(), self.field_slices()):
            out[s1: s1 + n0] = re[s0: s0 + n0]
            out[s1 + n0: s1 + 2 * n0] = im[s0: s0 + n0]
        out[self.time_offset] = re[b.time_offset]
        return out

    def unpack(self, v):
        """Host: (re, im) padded base vectors from a pair vector."""
        import numpy as np

        b = self.base
        re, im = np.zeros(b.ld), np.zeros(b.ld)
        for (_, s0, n0), (_, s1, _) in zip(b.field_slices(), self.field_slices()):
            re[s0: s0 + n0] = v[s1: s1 + n0]
            im[s0: s0 + n0] = v[s1 + n0: s1 + 2 * n0]
        re[b.time_offset] = v[self.time_offset]
        return re, im


def pair_layout(lay: NekLayout) -> PairLayout:
    """The complex (re/im pair) counterpart of ``lay`` (same shard)."""
    return PairLayout(lay.ldim, lay.lx1, lay.lx2, 2 * lay.nelgv, lay.n_scalars, lay.ifpo, lay.rank, lay.world,
                      base_nelgv=lay.nelgv)
