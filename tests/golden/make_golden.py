#!/usr/bin/env python
"""Generate the golden fixtures under tests/golden/ (run in the build container; committed output).

Provenance, per fixture:

* ``fld_headers.json`` — the four Nek5000 base-flow files the reference ships
  (``examples/cylinder/BF_1cyl0.f00001``, ``BFRe40_1cyl0.f00001``,
  ``examples/back_fstep/{baseflow,transient_growth}/BF_bfs0.f00001``), parsed HERE by an
  independent byte-offset reader (``_parse_std`` below, not ``nekstab_next_amd.fld``): header
  tokens, endian tag, element-map checksum and per-field sum / sum of squares / min / max.
  Data held by the reference itself: these pin the product's ``.fld`` reader.
* ``bf_1cyl0_seed.npz`` — the cylinder base flow (U, V and P mapped to the lx2 mesh) of
  ``BF_1cyl0.f00001`` as one state vector on the real cylinder mesh (E=1996, N=175,648, reference
  order), the seed of the config-2 golden run; lets the GPU box run on the reference's own data
  without ``/root/reference``.
* ``ks_*.npz`` / ``gmres_*.npz`` — outputs of the CPU oracle (``oracle/``: the C restatement of
  ``update_hessenberg_matrix`` and the numpy restatement of the drivers) on the synthetic BASELINE
  operators, with the dense steps on Intel MKL (``oracle/mkl_lapack.py``, the LAPACK the
  reference's build links, bin/mks:32-44) as the primary keys and the same run on SciPy's OpenBLAS
  (the product's LAPACK) as ``*_openblas`` keys; the Krylov–Schur ones also hold every restart's
  input Hessenberg matrix (``H_restart``) and selected mask.  The reference's Fortran is not buildable in this image (DESIGN.md
  §3), so these are oracle outputs, not reference outputs: they freeze the oracle (a change to it
  shows up as a fixture mismatch) and let the GPU tests check the HIP path without running the
  oracle.  Parity against the reference itself stays "unpinned" (DESIGN.md §3).
* ``wavemaker_cyl.npz`` — the oracle's ``wave_maker`` (core/sensitivity.f90:3-77: bi-orthogonalise,
  then sqrt(sum dRe^2 + dIm^2) sqrt(sum aRe^2 + aIm^2)) on the real cylinder mesh (E=1996, 2-D):
  the direct mode's real part is the reference's own base flow (U, V of ``BF_1cyl0.f00001``, from
  ``bf_1cyl0_seed.npz``), the other three parts hashed (``synthetic.hash_vector`` seeds 41-43).
  Oracle output: freezes the restatement and lets the GPU test run the product's file chain
  against it without the oracle.
* ``lapack_split.npz`` — the restart's dense chain (dgees sorted -> select_eigenvalues -> dtrsen)
  under MKL on Hessenberg matrices built with ``ordering.npz``'s spectra, OpenBLAS's Schur order
  beside it (``gen_lapack_split``).
* ``ordering.npz`` — inputs/outputs of the C transliteration of ``quicksort2``
  (core/utils.f90:29-138), ``select_eigenvalues`` (core/eigensolvers.f90:688-754) and
  ``sort_eigendecomp`` (core/lapack_wrapper.f90:181-228), including the pivot defect.

usage: python tests/golden/make_golden.py        (writes next to this file)
       python tests/golden/make_golden.py --only-solvers   (the LAPACK-dependent fixtures only)
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

REF = "/root/reference"
FLD_FILES = [
    "examples/cylinder/BF_1cyl0.f00001",
    "examples/cylinder/BFRe40_1cyl0.f00001",
    "examples/back_fstep/baseflow/BF_bfs0.f00001",
    "examples/back_fstep/transient_growth/BF_bfs0.f00001",
]


def _parse_std(path):
    """Byte-offset parse of a Nek5000 '#std' file: 132-byte ASCII header, 4-byte endian tag
    (6.54321 as float32), nel int32 element ids, then per element group the data, X/U as ldim
    blocks per element, P/T one block per element."""
    raw = open(path, "rb").read()
    tok = raw[:132].decode("ascii").split()
    wd, nx, ny, nz, nel = (int(t) for t in tok[1:6])
    rd = tok[11]
    tag_le = struct.unpack("<f", raw[132:136])[0]
    bo = "<" if abs(tag_le - 6.54321) < 1e-5 else ">"
    emap = np.array(struct.unpack(f"{bo}{nel}i", raw[136:136 + 4 * nel]), dtype=np.int64)
    pts = nx * ny * nz
    ldim = 3 if nz > 1 else 2
    off = 136 + 4 * nel
    fmt = "d" if wd == 8 else "f"
    fields = {}
    for g in rd:
        ncomp = ldim if g in "XU" else 1
        cnt = nel * ncomp * pts
        vals = np.array(struct.unpack(f"{bo}{cnt}{fmt}", raw[off:off + cnt * wd]), dtype=np.float64)
        off += cnt * wd
        blk = vals.reshape(nel, ncomp, pts)
        names = {"X": ["x", "y", "z"], "U": ["vx", "vy", "vz"], "P": ["pr"], "T": ["t"]}[g]
        for c in range(ncomp):
            fields[names[c]] = blk[:, c, :]
    assert off == len(raw), (path, off, len(raw))
    return tok, tag_le, emap, fields


def gen_fld():
    out = {}
    for rel in FLD_FILES:
        tok, tag, emap, fields = _parse_std(os.path.join(REF, rel))
        out[rel] = {
            "header_tokens": tok[:12],
            "size_bytes": os.path.getsize(os.path.join(REF, rel)),
            "endian_tag": tag,
            "emap_sum": int(emap.sum()), "emap_first": emap[:8].tolist(),
            "emap_sha1": hashlib.sha1(emap.astype("<i8").tobytes()).hexdigest(),
            "fields": {k: {"sum": float(v.sum()), "sumsq": float((v * v).sum()), "min": float(v.min()),
                           "max": float(v.max()), "elem0": v[0].tolist()} for k, v in fields.items()},
        }
    json.dump(out, open(os.path.join(HERE, "fld_headers.json"), "w"), indent=1)


def _checksum(a):
    return np.array([np.sum(a), np.sum(a * a), a[0], a[-1]])


def _stack_masks(masks, k):
    return np.array(masks, dtype=bool).reshape(len(masks), k)


def _both(fn):
    """Run an oracle computation under MKL (the fixture's primary keys) and under SciPy's OpenBLAS
    (the ``*_openblas`` keys): SURVEY §8(c), "record both in fixtures to detect ordering ties"."""
    import oracle as orc

    out = {}
    prev = orc.lapack_name()
    try:
        for lp in ("mkl", "openblas"):
            orc.use_lapack(lp)
            out[lp] = fn()
    finally:
        orc.use_lapack(prev)
    return out["mkl"], out["openblas"]


def _ks_keys(rm, ro, k):
    """Krylov–Schur fixture keys: MKL trajectory + the restart inputs (H before each
    schur_condensation) + the OpenBLAS trajectory side by side."""
    import oracle as orc

    z = dict(vals=rm["vals"], residual=rm["residual"], mstart=np.array(rm["mstart"], dtype=np.int64),
             cnt=np.array(rm["cnt"], dtype=np.int64), schur_cnt=rm["schur_cnt"], H_first=rm["H_first"],
             selected=_stack_masks(rm["selected"], k),
             H_restart=np.array(rm["H_restart"]).reshape(len(rm["H_restart"]), k + 1, k),
             vals_openblas=ro["vals"], residual_openblas=ro["residual"],
             mstart_openblas=np.array(ro["mstart"], dtype=np.int64), cnt_openblas=np.array(ro["cnt"], dtype=np.int64),
             schur_cnt_openblas=ro["schur_cnt"], selected_openblas=_stack_masks(ro["selected"], k),
             lapack=np.array(orc._mkl.version()))
    return z


def gen_solvers():
    import oracle as orc
    from helpers import olayout, oracle_diag_matvec, oracle_rot2_matvec
    from nekstab_next_amd import fld
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import NekLayout, box3d_layout, cylinder_layout

    orc.set_threads(8)

    def seed_of(lay, L, w, s):
        return orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, s)))

    # config 1: 2-D lx1=6, E=1136 (N=99,968), diag spectrum, Krylov–Schur k_dim=16, schur_tgt=5
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1136)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    d, exact = syn.diag_spectrum(lay)
    dref = syn.to_reference_order(lay, d)
    q1 = seed_of(lay, L, w, 11)
    rm, ro = _both(lambda: orc.krylov_schur(L, w, oracle_diag_matvec(L, dref), q1, 16, 5))
    np.savez(os.path.join(HERE, "ks_config1.npz"), **_ks_keys(rm, ro, 16), H_final=rm["H"],
             seed_checksum=_checksum(q1), d_checksum=_checksum(dref), w_checksum=_checksum(w), exact=exact)

    # config 2 on the real cylinder mesh (E=1996, N=175,648) seeded with the reference's own base
    # flow BF_1cyl0.f00001 (U, V, P); rotation-scaling operator, Krylov–Schur schur_tgt=2 (1cyl.usr:15)
    # at k_dim=16 (two restarts through conjugate pairs) and k_dim=64 (BASELINE's m, no restart)
    lay = cylinder_layout(1996)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    if not os.path.exists(os.path.join(HERE, "bf_1cyl0_seed.npz")):   # frozen once written
        f = fld.read_fld(os.path.join(REF, FLD_FILES[0]))
        bf = syn.to_reference_order(lay, fld.vector_from_fld(lay, f))
        np.savez_compressed(os.path.join(HERE, "bf_1cyl0_seed.npz"), seed_ref=bf)
    bf = np.load(os.path.join(HERE, "bf_1cyl0_seed.npz"))["seed_ref"]
    q1 = orc.prepare_seed(L, w, bf)
    c, s, dr, exact = syn.rot2_operator(lay)
    for k in (16, 64):
        rm, ro = _both(lambda: orc.krylov_schur(L, w, oracle_rot2_matvec(lay, c, s, dr), q1, k, 2))
        np.savez(os.path.join(HERE, f"ks_config2_bf_k{k}.npz"), **_ks_keys(rm, ro, k),
                 seed_checksum=_checksum(q1), exact=exact)

    # config 3 family, reduced (box3d E=40, N=90,592): plain 40-step Arnoldi on the shift-invert
    # Laplacian (|mu| from 0.1 to 3e8: the strongly graded spectrum of the headline config)
    lay = box3d_layout(40)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    d, exact = syn.laplacian_shift_invert(lay)
    q1 = seed_of(lay, L, w, 11)
    rm, ro = _both(lambda: orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 40, 0))
    np.savez(os.path.join(HERE, "ks_config3_arnoldi.npz"), vals=rm["vals"], residual=rm["residual"],
             H=rm["H"], seed_checksum=_checksum(q1), exact=exact[:64], vals_openblas=ro["vals"],
             residual_openblas=ro["residual"], lapack=np.array(orc.lapack_version()))

    # config 3 layout (E=128, N=289,792) at BASELINE's m: a real k_dim=128 restart on a
    # time-stepper-like clustered spectrum (one condensation keeping 25 columns), and the
    # shift-invert family's Krylov–Schur at k_dim=32, schur_tgt=4 (converges without a restart)
    lay = box3d_layout(128)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    q1 = seed_of(lay, L, w, 11)
    d, exact = syn.clustered_spectrum(lay)
    rm, ro = _both(lambda: orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 128, 4))
    np.savez_compressed(os.path.join(HERE, "ks_restart_m128.npz"), **_ks_keys(rm, ro, 128),
                        seed_checksum=_checksum(q1), exact=exact)
    d, exact = syn.laplacian_shift_invert(lay)
    rm, ro = _both(lambda: orc.krylov_schur(L, w, oracle_diag_matvec(L, syn.to_reference_order(lay, d)), q1, 32, 4))
    np.savez(os.path.join(HERE, "ks_config3_k32.npz"), **_ks_keys(rm, ro, 32), exact=exact[:64])

    # config 4: ts_gmres on J = D - I (cylinder layout E=1996, the real mesh size), k_dim=200,
    # maxiter=10, tol=1e-9 (1cyl.usr:14, newton_krylov.f90:44, 1cyl.par:18,23)
    lay = cylinder_layout(1996)
    L = olayout(lay)
    w = syn.mass_weights(lay)
    d, _ = syn.diag_spectrum(lay)
    J = syn.to_reference_order(lay, d) - 1.0
    rhs = syn.to_reference_order(lay, syn.hash_vector(lay, 3))

    def mv(x, y):
        y[:] = J * x
        y[-1] = 0.0

    (sol, hist), (sol_o, hist_o) = _both(lambda: orc.ts_gmres(L, w, mv, rhs, maxiter=10, ksize=200, tol=1e-9))
    np.savez(os.path.join(HERE, "gmres_config4.npz"), outer=np.array(hist["outer"]),
             inner=np.array(hist["inner"]), y_last=hist["y"][-1], sol_checksum=_checksum(sol), sol_head=sol[:256],
             sol_wnorm2=orc.k_dot(L, w, sol, sol), rhs_checksum=_checksum(rhs),
             outer_openblas=np.array(hist_o["outer"]), inner_openblas=np.array(hist_o["inner"]),
             y_last_openblas=hist_o["y"][-1], sol_head_openblas=sol_o[:256], lapack=np.array(orc.lapack_version()))
    orc.set_threads(1)


def _spectrum_matrix(vals, rng):
    """A real upper Hessenberg matrix with the given (conjugate-closed) spectrum: real 1x1 and
    [[a, b], [-b, a]] 2x2 blocks, a random similarity (well conditioned), then a Householder
    Hessenberg reduction — the shape of the k x k matrix a Krylov–Schur restart hands dgees."""
    from scipy.linalg import hessenberg

    n = vals.size
    D = np.zeros((n, n))
    used = np.zeros(n, dtype=bool)
    i = 0
    for j in range(n):
        if used[j]:
            continue
        v = vals[j]
        used[j] = True
        if v.imag == 0:
            D[i, i] = v.real
            i += 1
        else:
            p = [q for q in range(n) if not used[q] and vals[q] == np.conj(v)][0]
            used[p] = True
            D[i:i + 2, i:i + 2] = [[v.real, abs(v.imag)], [-abs(v.imag), v.real]]
            i += 2
    S = np.eye(n) + 0.3 * rng.standard_normal((n, n)) / np.sqrt(n)
    return hessenberg(S @ D @ np.linalg.inv(S))


def gen_lapack_split():
    """The restart's dense chain (dgees with the |lambda| > 0.9 sort -> select_eigenvalues ->
    dtrsen) under MKL on matrices with the ordering fixture's spectra (real values, conjugate
    pairs, zeros, values on both sides of 1 - schur_del and 0.9): per case the input matrix, MKL's
    Schur-order eigenvalues, selected mask and count, and the reordered leading block's eigenvalues;
    OpenBLAS's Schur-order eigenvalues beside them (to name where the two order differently)."""
    import oracle as orc

    z = np.load(os.path.join(HERE, "ordering.npz"))
    rng = np.random.default_rng(505)
    out = dict(n=[], A=[], vals_mkl=[], sel_mkl=[], cnt_mkl=[], lead_mkl=[], vals_openblas=[], args=[])
    for n, v, (delta, nev) in zip(z["sel_len"], z["sel_vals"], z["sel_args"]):
        A = _spectrum_matrix(v[:n], rng)
        res = {}
        for lp in ("mkl", "openblas"):
            orc.use_lapack(lp)
            T, Z, vals = orc.schur_sorted(A)
            sel, cnt = orc.select_eigenvalues(vals, delta, int(nev))
            T2, _ = orc.ordschur(T, Z, sel)
            lead = np.linalg.eigvals(T2[:cnt, :cnt]) if cnt else np.zeros(0)
            res[lp] = (vals, sel, cnt, lead)
        orc.use_lapack("mkl")
        out["n"].append(n)
        out["A"].append(A)
        out["vals_mkl"].append(res["mkl"][0])
        out["sel_mkl"].append(res["mkl"][1])
        out["cnt_mkl"].append(res["mkl"][2])
        out["lead_mkl"].append(np.sort_complex(res["mkl"][3]))
        out["vals_openblas"].append(res["openblas"][0])
        out["args"].append((delta, nev))
    nmax = max(out["n"])
    padv = lambda xs, dt: np.array([np.pad(x, (0, nmax - len(x))) for x in xs], dtype=dt)  # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "lapack_split.npz"), n=np.array(out["n"]),
        A=np.array([np.pad(a, ((0, nmax - a.shape[0]), (0, nmax - a.shape[0]))) for a in out["A"]]),
        vals_mkl=padv(out["vals_mkl"], np.complex128), sel_mkl=padv(out["sel_mkl"], bool),
        cnt_mkl=np.array(out["cnt_mkl"]), lead_mkl=padv(out["lead_mkl"], np.complex128),
        vals_openblas=padv(out["vals_openblas"], np.complex128), args=np.array(out["args"]),
        lapack=np.array(orc.lapack_version()))


def wavemaker_inputs():
    """(velocity layout, weights, [dRe, dIm, aRe, aIm] in reference order incl. the time slot)."""
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import cylinder_layout
    from nekstab_next_amd.sensitivity import velocity_layout

    vlay = velocity_layout(cylinder_layout(1996))
    nvel = vlay.ldim * vlay.n_v
    bf = np.load(os.path.join(HERE, "bf_1cyl0_seed.npz"))["seed_ref"]
    vecs = [np.concatenate([bf[:nvel], [0.0]])]
    for s_ in (41, 42, 43):
        vecs.append(syn.to_reference_order(vlay, syn.hash_vector(vlay, s_)))
    vecs[1] = 0.3 * vecs[1]
    return vlay, syn.mass_weights(vlay), vecs


def gen_wavemaker():
    import oracle as orc

    vlay, w, vecs = wavemaker_inputs()
    L = orc.OLayout(vlay.n_v, 0, vlay.ldim, False, vlay.ldim)
    wm, out = orc.wave_maker(L, w, *vecs)
    ip = lambda p, q: orc.k_dot(L, w, p, q)  # noqa: E731
    d, di, a, ai = out
    np.savez_compressed(os.path.join(HERE, "wavemaker_cyl.npz"), wavemaker=wm,
                        ad_after=np.array([ip(a, d) + ip(ai, di), ip(a, di) - ip(ai, d)]),
                        inputs_checksum=np.array([_checksum(v) for v in vecs]))


def gen_noise():
    """The reference's default seed noise on the real cylinder mesh: the GLL coordinates of
    BF_1cyl0.f00001 (X block, byte-offset parse) in global element order, and the oracle's
    op_add_noise (vx, vy: mth_rand, utils.f90:297-359, then dssum/vmult and dsavg by coincident
    points) as checksums and every 97th value."""
    import oracle as orc

    _, _, emap, fields = _parse_std(os.path.join(REF, FLD_FILES[0]))
    order = np.argsort(emap)
    x, y = fields["x"][order].ravel(), fields["y"][order].ravel()
    np.savez_compressed(os.path.join(HERE, "cyl_mesh_xy.npz"), x=x, y=y)
    coords = {"x": x, "y": y}
    out = {}
    for c, fc in enumerate(((3.0e4, -1.5e3, 0.5e5), (2.3e4, 2.3e3, -2.0e5))):
        q = orc.noise_field(6, 6, 1, 0, x, y, None, fc)
        q = orc.coincident_average(orc.coincident_average(q, coords), coords)
        out[f"c{c}_checksum"] = _checksum(q)
        out[f"c{c}_sample"] = q[::97]
    np.savez(os.path.join(HERE, "noise_cyl.npz"), **out)


def gen_ordering():
    import oracle as orc

    rng = np.random.default_rng(2024)
    qs_in, qs_idx, qs_out = [], [], []
    for n in list(range(1, 41)) + [64, 100, 128]:
        for rep in range(3):
            a = rng.standard_normal(n) * (10.0 ** rng.integers(-3, 3))
            if rep == 2 and n > 3:
                a[rng.integers(0, n, size=n // 3)] = a[0]   # ties
            idx, srt = orc.quicksort2(a)
            qs_in.append(a)
            qs_idx.append(idx)
            qs_out.append(srt)
    # the documented defect: [3,1,2,0.5,7,6,5,4] loses an index
    sel_vals, sel_mask, sel_cnt, sel_args = [], [], [], []
    for n in (8, 9, 16, 24, 40, 64, 128):   # n >= nev + 4 (the reference indexes idx(n-(nev+4)))
        for rep in range(4):
            if n < 2 + rep + 4:
                continue
            nr = n // 2
            re = rng.uniform(-1.1, 1.1, nr)
            pairs = (n - nr) // 2
            z = rng.uniform(0.2, 1.05, pairs) * np.exp(1j * rng.uniform(0.05, 3.0, pairs))
            v = np.concatenate([re + 0j, z, np.conj(z)])
            v = np.concatenate([v, np.zeros(n - v.size)])
            rng.shuffle(v)
            delta, nev = (0.1, 2 + rep)
            mask, cnt = orc.select_eigenvalues(v, delta, nev)
            sel_vals.append(v)
            sel_mask.append(mask)
            sel_cnt.append(cnt)
            sel_args.append((delta, nev))
    pad = lambda xs, dt: np.array([np.pad(x, (0, 128 - len(x))) for x in xs], dtype=dt)  # noqa: E731
    np.savez(os.path.join(HERE, "ordering.npz"),
             qs_len=np.array([len(a) for a in qs_in]), qs_in=pad(qs_in, np.float64),
             qs_idx=pad(qs_idx, np.int64), qs_out=pad(qs_out, np.float64),
             sel_len=np.array([len(v) for v in sel_vals]), sel_vals=pad(sel_vals, np.complex128),
             sel_mask=pad(sel_mask, bool), sel_cnt=np.array(sel_cnt), sel_args=np.array(sel_args))


if __name__ == "__main__":
    if "--only-wavemaker" in sys.argv:   # needs only the committed bf_1cyl0_seed.npz, not /root/reference
        gen_wavemaker()
        sys.exit(0)
    if "--only-noise" in sys.argv:
        gen_noise()
        sys.exit(0)
    if "--only-solvers" in sys.argv:   # the LAPACK-dependent fixtures (needs no /root/reference)
        gen_solvers()
        gen_lapack_split()
        sys.exit(0)
    gen_fld()
    gen_ordering()
    gen_solvers()
    gen_lapack_split()
    gen_wavemaker()
    gen_noise()
    for n in sorted(os.listdir(HERE)):
        print(f"{os.path.getsize(os.path.join(HERE, n)):10d}  {n}")
