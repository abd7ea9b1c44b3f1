"""Synthetic, exactly known workloads for the BASELINE configs.

Everything here is generated from (global element, local point, field) keys with a counter-based
hash, so a 1-, 2-, 4- or 8-way element-contiguous shard sees bit-identical inputs.  Functions
return host numpy arrays already placed in the padded device layout of a (possibly sharded)
:class:`NekLayout`; :func:`to_reference_order` gives the reference's unpadded order
``[vx | vy | (vz) | t.. | pr | time]`` for CPU cross-checks.

* weights: GLL tensor weights x per-element Jacobian J_e ~ U(0.5, 1.5) (a Nek ``bm1`` look-alike).
* config 1/2/4: a diagonal spectrum (0.99 … 0.89 on six seeded dofs + bulk 0.5 (1 - g/n)) and a
  per-point rotation-scaling with three dominant conjugate pairs.
* config 3: the "diagonalised shift-invert Laplacian" mu_g = 1/(lambda_{pi(g)} - sigma),
  lambda_k = -4 sin^2(k pi / (2(n+1))), pi an affine permutation.
"""
from __future__ import annotations

from math import gcd

import numpy as np

from .layout import NekLayout

_M64 = (1 << 64) - 1


def _mix(z: np.ndarray) -> np.ndarray:
    z = z + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, stream: int, keys: np.ndarray) -> np.ndarray:
    """u in [0, 1) with 53 exact bits for integer keys (same mixer as the device generator)."""
    with np.errstate(over="ignore"):
        key0 = np.uint64((int(seed) * 0xD1342543DE82EF95) & _M64)
        z = _mix(key0 + np.uint64((int(stream) * 0x9E3779B97F4A7C15) & _M64) + keys.astype(np.uint64))
    return (z >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def hash_vector(lay: NekLayout, seed: int) -> np.ndarray:
    """Host twin of ``nkv_fill_hash``: 2u-1 on live rows, 0 on padding and time."""
    out = np.zeros(lay.ld)
    gv = np.arange(lay.v_offset, lay.v_offset + lay.n_v, dtype=np.uint64)
    for f in range(lay.n_wf):
        out[f * lay.sv: f * lay.sv + lay.n_v] = 2.0 * hash_uniform(seed, f, gv) - 1.0
    gp = np.arange(lay.p_offset, lay.p_offset + lay.n_p, dtype=np.uint64)
    s = lay.n_wf * lay.sv
    out[s: s + lay.n_p] = 2.0 * hash_uniform(seed, 31, gp) - 1.0
    return out


def to_reference_order(lay: NekLayout, padded: np.ndarray) -> np.ndarray:
    """Padded device layout -> reference order [vx|vy|(vz)|t..|pr|time] (unpadded)."""
    parts = [padded[s: s + n] for _, s, n in lay.field_slices()]
    return np.concatenate(parts + [padded[lay.time_offset: lay.time_offset + 1]])


def from_reference_order(lay: NekLayout, ref: np.ndarray) -> np.ndarray:
    out = np.zeros(lay.ld)
    o = 0
    for _, s, n in lay.field_slices():
        out[s: s + n] = ref[o: o + n]
        o += n
    out[lay.time_offset] = ref[o]
    return out


# ---- weights ----------------------------------------------------------------------------------

def gll_weights(n_pts: int) -> np.ndarray:
    """Gauss–Lobatto–Legendre quadrature weights on [-1, 1] for ``n_pts`` points."""
    N = n_pts - 1
    PN = np.polynomial.legendre.Legendre.basis(N)
    interior = np.sort(PN.deriv().roots().real)
    x = np.concatenate([[-1.0], interior, [1.0]])
    return 2.0 / (N * (N + 1) * PN(x) ** 2)


def mass_weights(lay: NekLayout, seed: int = 7) -> np.ndarray:
    """Local bm1-like weights (length n_v): GLL tensor weights x J_e, J_e ~ U(0.5, 1.5) keyed by
    the global element id."""
    w1 = gll_weights(lay.lx1)
    wt = w1
    for _ in range(lay.ldim - 1):
        wt = np.multiply.outer(wt, w1)
    wt = wt.reshape(-1)
    e0, e1 = lay.elem_range()
    J = 0.5 + hash_uniform(seed, 101, np.arange(e0, e1, dtype=np.uint64))
    return (J[:, None] * wt[None, :]).reshape(-1)


def sponge(weights: np.ndarray, frac: float = 0.1) -> np.ndarray:
    """Zero the last ``frac`` of the weights, as activate_sponge does inside the sponge
    (core/forcing.f90:101-104)."""
    w = weights.copy()
    w[int(len(w) * (1 - frac)):] = 0.0
    return w


# ---- config 1: diagonal spectrum ---------------------------------------------------------------

DOMINANT = (0.99, 0.97, 0.95, 0.93, 0.91, 0.89)


def _dominant_positions(lay: NekLayout, count: int, seed: int) -> np.ndarray:
    """Global weighted indices carrying the dominant eigenvalues (spread, distinct, seeded)."""
    n = lay.n_wf * lay.pts_v * lay.nelgv
    pos = []
    for i in range(count):
        u = hash_uniform(seed, 211, np.array([i], dtype=np.uint64))[0]
        p = int(u * n)
        while p in pos:
            p = (p + 1) % n
        pos.append(p)
    return np.asarray(pos, dtype=np.int64)


def weighted_global_index(lay: NekLayout, f: int) -> np.ndarray:
    return f * lay.pts_v * lay.nelgv + lay.v_offset + np.arange(lay.n_v, dtype=np.int64)


def diag_spectrum(lay: NekLayout, seed: int = 1, dominant=DOMINANT, pr_value: float = 0.5) -> tuple:
    """(padded diag, exact dominant eigenvalues).  Bulk lambda_g = 0.5 (1 - g/n) over global
    weighted dofs g; ``dominant`` values on seeded dofs; pressure ``pr_value``."""
    n = lay.n_wf * lay.pts_v * lay.nelgv
    pos = _dominant_positions(lay, len(dominant), seed)
    d = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        g = weighted_global_index(lay, f)
        v = 0.5 * (1.0 - g / n)
        for p, lam in zip(pos, dominant):
            hit = g == p
            v[hit] = lam
        d[f * lay.sv: f * lay.sv + lay.n_v] = v
    s = lay.n_wf * lay.sv
    d[s: s + lay.n_p] = pr_value
    return d, np.asarray(dominant, dtype=np.float64)


# ---- config 2: rotation-scaling with conjugate pairs -------------------------------------------

DOMINANT_PAIRS = ((0.99, 0.35), (0.96, 0.8), (0.93, 1.3))  # (r, theta)


def rot2_operator(lay: NekLayout, seed: int = 2, pairs=DOMINANT_PAIRS, rest_value: float = 0.1):
    """(c[sv], s[sv], d_rest[ld], exact eigenvalues).  Per global point p: r_p ~ U[0, 0.5],
    theta_p ~ U[0, pi]; three seeded points carry the dominant pairs r e^{±i theta}."""
    npts = lay.pts_v * lay.nelgv
    gp = lay.v_offset + np.arange(lay.n_v, dtype=np.int64)
    r = 0.5 * hash_uniform(seed, 301, gp.astype(np.uint64))
    th = np.pi * hash_uniform(seed, 302, gp.astype(np.uint64))
    for i, (rr, tt) in enumerate(pairs):
        p = int(hash_uniform(seed, 303, np.array([i], dtype=np.uint64))[0] * npts)
        hit = gp == p
        r[hit] = rr
        th[hit] = tt
    c = np.zeros(lay.sv)
    s = np.zeros(lay.sv)
    c[: lay.n_v] = r * np.cos(th)
    s[: lay.n_v] = r * np.sin(th)
    d_rest = np.zeros(lay.ld)  # scalars (if any) and pressure scaled by rest_value
    for f in range(2, lay.n_wf):
        d_rest[f * lay.sv: f * lay.sv + lay.n_v] = rest_value
    d_rest[lay.n_wf * lay.sv: lay.n_wf * lay.sv + lay.n_p] = rest_value
    exact = []
    for rr, tt in pairs:
        exact += [rr * np.exp(1j * tt), rr * np.exp(-1j * tt)]
    return c, s, d_rest, np.asarray(exact)


# ---- a clustered spectrum that needs Krylov–Schur restarts at m = 128 ------------------------------

def clustered_spectrum(lay: NekLayout, spacing: float = 0.002, n_cluster: int = 400, bulk: float = 0.2,
                       seed: int = 5, pr_value: float = 0.1) -> tuple:
    """(padded diag, exact cluster eigenvalues, decreasing).  A time-stepper-like spectrum: a dense
    cluster below 1, lambda_k = 1 - spacing (k - 1/2) for k = 1..n_cluster on seeded distinct
    global weighted dofs (an affine permutation), over a bulk U[0, bulk] (hashed per global dof);
    pressure ``pr_value``.  The cluster's spacing makes the leading eigenvalues converge slowly, so a
    128-vector Krylov–Schur with schur_tgt=4 restarts (the half-step keeps every eigenvalue away
    from select_eigvals' |lambda| > 0.9 boundary); shard-independent like every generator here."""
    n = lay.n_wf * lay.pts_v * lay.nelgv
    a, b = _affine_perm_params(n, seed)
    k = np.arange(n_cluster, dtype=np.int64)
    pos = (a * k + b) % n
    order = np.argsort(pos)
    pos_sorted, val_sorted = pos[order], (1.0 - spacing * (k + 0.5))[order]
    d = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        g = weighted_global_index(lay, f)
        v = bulk * hash_uniform(seed, 501, g.astype(np.uint64))
        i = np.searchsorted(pos_sorted, g)
        hit = (i < pos_sorted.size) & (pos_sorted[np.minimum(i, pos_sorted.size - 1)] == g)
        v[hit] = val_sorted[i[hit]]
        d[f * lay.sv: f * lay.sv + lay.n_v] = v
    s = lay.n_wf * lay.sv
    d[s: s + lay.n_p] = pr_value
    return d, 1.0 - spacing * (k + 0.5)


# ---- config 3: diagonalised shift-invert Laplacian ----------------------------------------------

def _affine_perm_params(n: int, seed: int) -> tuple[int, int]:
    a = int(hash_uniform(seed, 401, np.array([0], dtype=np.uint64))[0] * n) | 1
    while gcd(a, n) != 1:
        a += 2
    b = int(hash_uniform(seed, 402, np.array([0], dtype=np.uint64))[0] * n)
    return a % n if n > 1 else 1, b


def laplacian_shift_invert(lay: NekLayout, seed: int = 3, k0: int = 3, frac: float = 0.3,
                           pr_value: float = 0.1, n_exact: int = 4096):
    """(padded diag, exact top-|mu| eigenvalues).  mu_g = 1/(lambda_{pi(g)} - sigma) with the
    1-D Dirichlet Laplacian spectrum lambda_k = -4 sin^2(k pi / (2(n+1))), k = 1..n (n = global
    weighted dofs), pi(g) = (a g + b) mod n + 1, sigma = lambda_k0 + frac (lambda_{k0+1} - lambda_k0)."""
    n = lay.n_wf * lay.pts_v * lay.nelgv
    a, b = _affine_perm_params(n, seed)

    def lam(k):
        return -4.0 * np.sin(k * np.pi / (2.0 * (n + 1))) ** 2

    sigma = lam(k0) + frac * (lam(k0 + 1) - lam(k0))
    d = np.zeros(lay.ld)
    for f in range(lay.n_wf):
        g = weighted_global_index(lay, f)
        k = ((a * g + b) % n) + 1
        d[f * lay.sv: f * lay.sv + lay.n_v] = 1.0 / (lam(k.astype(np.float64)) - sigma)
    s = lay.n_wf * lay.sv
    d[s: s + lay.n_p] = pr_value
    # |mu_k| decays like 1/k^2 away from k0, so the n_exact largest are among k <= k0 + 2 n_exact
    ks = np.arange(1, min(n, k0 + 2 * n_exact + 8) + 1, dtype=np.float64)
    mu = 1.0 / (lam(ks) - sigma)
    exact = mu[np.argsort(-np.abs(mu), kind="stable")][:n_exact]
    return d, exact


# ---- resolvent (complex) test operator ----------------------------------------------------------

RESOLVENT_GAMMAS = (0.02, 0.05, 0.11, 0.2, 0.31)   # decay rates of the least-stable modes


def resolvent_diag(lay, omega: float = 0.3, gammas=RESOLVENT_GAMMAS, seed: int = 3):
    """Resolvent R = (i omega I - L)^-1 of a W-normal stable diagonal L, on the re/im pair layout
    ``lay`` (a :class:`~nekstab_next_amd.layout.PairLayout` shard): eigenvalues of L are
    -gamma_p (seeded weighted dofs, ``gammas``) and a bulk -g in [0.5, 5] over the global weighted
    dofs; pressure -1.  Returns (cr, ci) padded pair vectors (R's diagonal at the re rows) and the
    exact leading singular values 1/sqrt(omega^2 + gamma^2), decreasing."""
    base = lay.base
    n = base.n_wf * base.pts_v * base.nelgv
    pos = _dominant_positions(base, len(gammas), seed)
    cr = np.zeros(lay.ld)
    ci = np.zeros(lay.ld)
    for (_, s0, n0), (_, s1, _), f in zip(base.field_slices(), lay.field_slices(), range(base.n_wf + 1)):
        if f < base.n_wf:
            g = weighted_global_index(base, f)
            gam = 0.5 + 4.5 * g / n
            for p, gm in zip(pos, gammas):
                gam[g == p] = gm
        else:
            gam = np.ones(n0)
        # 1/(i omega + gamma) = (gamma - i omega)/(gamma^2 + omega^2)
        den = gam * gam + omega * omega
        cr[s1: s1 + n0] = gam / den
        ci[s1: s1 + n0] = -omega / den
    sv = np.sort(1.0 / np.sqrt(omega * omega + np.asarray(gammas) ** 2))[::-1]
    return cr, ci, sv
