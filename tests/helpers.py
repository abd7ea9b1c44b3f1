"""Shared test helpers: build matched product/oracle problems from the same synthetic inputs."""
import ctypes

import numpy as np

import oracle as orc
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout


def olayout(lay: NekLayout, time_in_dot=False):
    return orc.OLayout(lay.n_v, lay.n_p, lay.n_wf, time_in_dot, lay.ldim)


def oracle_diag_matvec(L, dref):
    return lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.0)


def oracle_rot2_matvec(lay: NekLayout, c, s, d_rest, transpose=False):
    """Reference-order rot2 operator (numpy), same math as nkv_op_rot2."""
    nv = lay.n_v
    cc, ss = c[:nv], (-1.0 if transpose else 1.0) * s[:nv]
    dr = syn.to_reference_order(lay, d_rest)

    def mv(x, y):
        u, v = x[:nv], x[nv:2 * nv]
        y[:nv] = cc * u - ss * v
        y[nv:2 * nv] = ss * u + cc * v
        y[2 * nv:-1] = dr[2 * nv:-1] * x[2 * nv:-1]
        y[-1] = 0.0
    return mv


def ritz_compare_set(ref_vals, ref_res, eigen_tol, top=8):
    """converged Ritz values + the top-8 by modulus."""
    idx = set(np.nonzero(ref_res < eigen_tol)[0].tolist()) | set(range(min(top, len(ref_vals))))
    return np.array(sorted(idx))


def match_ritz(a, b):
    """Greedy nearest matching of eigenvalue lists (order may differ inside conjugate pairs)."""
    b = list(b)
    out = []
    for x in a:
        j = int(np.argmin([abs(x - y) for y in b]))
        out.append(b.pop(j))
    return np.asarray(out)


def oracle_rank2_matvec(lay, d, u, v, u2, v2, sigma, w, transpose=False):
    """Reference-order twin of operators.RankTwoPerturbed: D x + sigma (u <v,x>_W + u2 <v2,x>_W)."""
    L = olayout(lay)
    dr = syn.to_reference_order(lay, d)
    U, V, U2, V2 = (syn.to_reference_order(lay, a) for a in (u, v, u2, v2))
    if transpose:
        U, V, U2, V2 = V, U, V2, U2

    def mv(x, y):
        a = orc.k_dot(L, w, V, x)
        b = orc.k_dot(L, w, U2, x)
        y[:] = dr * x
        y[-1] = 0.0
        y[:-1] += sigma * (U[:-1] * a + V2[:-1] * b)
    return mv
