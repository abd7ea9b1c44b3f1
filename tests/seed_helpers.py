"""Test helpers for the seed noise (tests only): a structured 3-D box mesh of GLL points."""
import numpy as np

from nekstab_next_amd.fld import gll_points


def box_mesh_coords(lay, ne=(2, 2, 2), L=(2.0, 1.0, 3.0)):
    """GLL coordinates (Nek point order, il fastest; elements x fastest) of a conforming ne[0] x ne[1]
    x ne[2] box mesh for a 3-D layout with nelgv = prod(ne); this rank's elements only."""
    n = lay.lx1
    g = 0.5 * (gll_points(n) + 1.0)
    e0, e1 = lay.elem_range()
    xs, ys, zs = [], [], []
    for e in range(e0, e1):
        ex, ey, ez = e % ne[0], (e // ne[0]) % ne[1], e // (ne[0] * ne[1])
        kk, jj, ii = np.meshgrid(g, g, g, indexing="ij")   # il fastest in C order of (kl, jl, il)
        xs.append(((ex + ii) * L[0] / ne[0]).ravel())
        ys.append(((ey + jj) * L[1] / ne[1]).ravel())
        zs.append(((ez + kk) * L[2] / ne[2]).ravel())
    cat = lambda a: np.concatenate(a) if a else np.zeros(0)  # noqa: E731
    return {"x": cat(xs), "y": cat(ys), "z": cat(zs)}
