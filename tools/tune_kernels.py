#!/usr/bin/env python
"""Build compile-time variants of libnekkrylov (tile rows, columns in flight, non-temporal loads,
grid size) and time the Gram–Schmidt entry points at BASELINE size in ONE process, interleaved
over rounds (cdna_hip_programming.md §5.4 rule 24).

Every variant is derived from the product sources at build time: ``-D`` values of its speed knobs,
and optionally a code experiment as a unified diff against them (``"patch": NAME`` applies
``tools/experiments/NAME.patch`` with ``patch -p1`` inside a copy of ``nekstab_next_amd/csrc/``).  No
copy of the kernels is kept: a patch that no longer applies fails the build (and the CPU test
tests/test_product_source.py), and the unpatched variant is the product's own sources, compiled by
the product's own build function (``__graft_entry__.build_hip``).  The round-1..3 experiment patches
were written against the single-file source that round 5 split into per-family translation units;
they were retired with it (git history and their logs under profiles/ keep them).

  python tools/tune_kernels.py build            # here (hipcc cross-compiles)
  python tools/tune_kernels.py run [--E 44176]  # on the MI355X box
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "tools", "variants")
PRODUCT_CSRC = os.path.join(ROOT, "nekstab_next_amd", "csrc")
EXP_DIR = os.path.join(ROOT, "tools", "experiments")

# Speed-only knobs of the product kernel.  The round-1 experiment switches (store skipping, soft
# grid barriers, tile-interleaved / field-major sweeps, XCD maps, buffer-store policies, register-
# budget schedules) were removed from nekkrylov.hip in round 2; their logs stay under profiles/.
VARIANTS = {
    "base": {},
    "nt": {"NKV_NT": 1},
    "pairs2": {"NKV_PAIRS": 2},
    "pairs8": {"NKV_PAIRS": 8},
    "colu2": {"NKV_COLU": 2},
    "colu8": {"NKV_COLU": 8},
    "maxb1024": {"NKV_MAXB": 1024},
    "maxb4096": {"NKV_MAXB": 4096},
    "nt_pairs8": {"NKV_NT": 1, "NKV_PAIRS": 8},
    "nt_p8_b1024": {"NKV_NT": 1, "NKV_PAIRS": 8, "NKV_MAXB": 1024},
    "nt_p8_c2": {"NKV_NT": 1, "NKV_PAIRS": 8, "NKV_COLU": 2},
    "nt_p4_c8_b1024": {"NKV_NT": 1, "NKV_COLU": 8, "NKV_MAXB": 1024},
    "nt_f16": {"NKV_NT": 1, "NKV_FUSE_NW": 16},
    "nt_fg512": {"NKV_NT": 1, "NKV_FUSE_G": 512},
    "nt_fg2048": {"NKV_NT": 1, "NKV_FUSE_G": 2048},
    "nt_f16_g512": {"NKV_NT": 1, "NKV_FUSE_NW": 16, "NKV_FUSE_G": 512},
    "rot_staged": {"NKV_ROT_STREAM": 0},
    "rot_w8": {"NKV_ROT_WAVES": 8},
    "rot_w8_nb2": {"NKV_ROT_WAVES": 8, "NKV_ROT_NB": 2},
    "rot_u2": {"NKV_ROT_U": 2},
    "rot_u8": {"NKV_ROT_U": 8},
    "rot_nopipe_u8": {"NKV_ROT_PIPE": 0, "NKV_ROT_U": 8},   # the round-2 streaming rotation before r02az
    "rot_pipe": {"NKV_ROT_PIPE": 1},
    "rot_pipe_u4": {"NKV_ROT_PIPE": 1, "NKV_ROT_U": 4},
    "rot_u4": {"NKV_ROT_U": 4},
    "rot_pipe_u2": {"NKV_ROT_PIPE": 1, "NKV_ROT_U": 2},
    "rot_chunk5": {"NKV_ROT_CHUNK_FROM": 5},
    "rot_nb2": {"NKV_ROT_NB": 2},
    "upd_r1": {"NKV_UPD_ROUNDS": 1},
    "upd_r2": {"NKV_UPD_ROUNDS": 2},
    "upd_r4": {"NKV_UPD_ROUNDS": 4},
    "upd_r0": {"NKV_UPD_ROUNDS": 0},   # the single-launch update before r02bh
    "pairs4": {"NKV_PAIRS": 4},
    "fg512": {"NKV_FUSE_G": 512},
    "fg2048": {"NKV_FUSE_G": 2048},
    "fnw4": {"NKV_FUSE_NW": 4},
    "fsmall0": {"NKV_FUSE_SMALL_J": 0},
    "usmall4": {"NKV_UPD_SMALL_J": 4},
    "usmall8": {"NKV_UPD_SMALL_J": 8},   # the fused pass before r02bn (8 waves at every small j)
    "maxb2048": {"NKV_MAXB": 2048},
    "axd_r1": {"NKV_AXD_ROUNDS": 1},
    "axd_r2": {"NKV_AXD_ROUNDS": 2},
    "axd_r4": {"NKV_AXD_ROUNDS": 4},
    "fuse_r1": {"NKV_FUSE_ROUNDS": 1},
    "fuse_r2": {"NKV_FUSE_ROUNDS": 2},
    "fuse_r4": {"NKV_FUSE_ROUNDS": 4},
    "rot_chunk_nosb": {"NKV_ROT_CHUNK_SB": 0},
    "rot_chunk_w8": {"NKV_ROT_CHUNK_W8_MAX": 8},
    "rot_nb2_w8": {"NKV_ROT_NB": 2, "NKV_ROT_WAVES": 8},
    "rot_w8u8": {"NKV_ROT_WAVES": 8, "NKV_ROT_U": 8},
    "dc_u4": {"NKV_DC_U": 4},
    "dc_p4": {"NKV_DC_PAIRS": 4},
    "dc_p4_u4": {"NKV_DC_PAIRS": 4, "NKV_DC_U": 4, "NKV_D2_U": 4},
    "d2_u1": {"NKV_D2_U": 1},
    "dc_nt0": {"NKV_NT": 0},
    "d2_nofl": {"NKV_D2_FIELDLOOP": 0},
    "ntst0": {"NKV_NT_ST": 0},
    "unr1_ntst0": {"NKV_NT_ST": 0, "NKV_STREAM_UNR": 1},
    "unr8": {"NKV_STREAM_UNR": 8},
    "d2_b768": {"NKV_D2_MAXB": 768},
    "d2_b512": {"NKV_D2_MAXB": 512},
    "d2_b256": {"NKV_D2_MAXB": 256},
    "d2_b384": {"NKV_D2_MAXB": 384},
    "d2_b1024": {"NKV_D2_MAXB": 1024},
    "dc_u16": {"NKV_DC_U": 16},
    "rotf_off": {"NKV_ROTF_MAX": 0},
    "rotf_p2u8": {"NKV_ROTF_P": 2, "NKV_ROTF_U": 8},
    "rotf_p8u2": {"NKV_ROTF_P": 8, "NKV_ROTF_U": 2},
    "rotf_p1u16": {"NKV_ROTF_P": 1, "NKV_ROTF_U": 16},
    "dc_g2048": {"NKV_DC_G": 2048},
    "dc_g256": {"NKV_DC_G": 256},
    "dc_g512": {"NKV_DC_G": 512},
    "dc_g768": {"NKV_DC_G": 768},
    "dc_g640": {"NKV_DC_G": 640},
    "dc_g1024": {"NKV_DC_G": 1024},
    "st_g2048": {"NKV_STREAM_G": 2048},
    "st_g1024": {"NKV_STREAM_G": 1024},
    "st_g768": {"NKV_STREAM_G": 768},
    "dc_g896": {"NKV_DC_G": 896},
    "dc_g1536": {"NKV_DC_G": 1536},
    "dc_g384": {"NKV_DC_G": 384},
    "dc_r0": {"NKV_DC_ROUNDS": 0},
    "dc_r1": {"NKV_DC_ROUNDS": 1},
    "dc_r4": {"NKV_DC_ROUNDS": 4},
    # code experiments: unified diffs against the product sources (tools/experiments/*.patch, none
    # at present: the round-1..3 patches targeted the pre-split single file; logs under profiles/)
    "small_tiles0": {"NKV_SMALL_TILES": 0},
    "maxb256": {"NKV_MAXB": 256},
    "maxb512": {"NKV_MAXB": 512},
    "ps2": {"NKV_PAIRS_SMALL": 2},
    "d2s_b256": {"NKV_D2_SMALL_B": 256},
    "d2s_b384": {"NKV_D2_SMALL_B": 384},
    "d2s_b768": {"NKV_D2_SMALL_B": 768},
    "d2s_b1024": {"NKV_D2_SMALL_B": 1024},   # the grid before r03aa
    "dots_b1024": {"NKV_DOT_SMALL_B": 1024},   # the grid before r03ac
    "dots_b256": {"NKV_DOT_SMALL_B": 256},
    "dots_b768": {"NKV_DOT_SMALL_B": 768},
    "fmid512": {"NKV_FUSE_G_MID": 512},
    "fmid384": {"NKV_FUSE_G_MID": 384},
    "fmid768": {"NKV_FUSE_G_MID": 768},
    "ps4": {"NKV_PAIRS_SMALL": 4},
    "ps1": {"NKV_PAIRS_SMALL": 1},
    "d2u4": {"NKV_D2_U": 4},
    "ps4_d2u4": {"NKV_PAIRS_SMALL": 4, "NKV_D2_U": 4},
    "d2red": {"NKV_D2_RED": 1},
    # round 5: the multi-dot's next column pair loaded while the current pair is reduced (software
    # pipeline: twice the bytes in flight per wave at one wave per SIMD); the multi-dot is the
    # box-sensitive kernel (6.55-6.79 TB/s across boxes, the dual update 6.97-7.02)
    "d2_pf": {"patch": "d2_prefetch"},
    # round 5: the streaming MFMA rotation's pipeline sat behind guarded (exec-masked) loads, after
    # which the compiler waits with vmcnt(0) for every load in flight: unguarded steady-state loads
    # with two batches ahead, adopted from 5 column blocks (one wave per SIMD; +9-13 % at 65-128
    # kept columns, r05aj), no change at 17-64 (r05ai, whose experiment patches were retired)
    "rot_p3_off": {"NKV_ROT_PIPE3_FROM": 99},   # the rotation before r05aj
    "rot_p3_from4": {"NKV_ROT_PIPE3_FROM": 4},
    # the k-chunked rotation (V not in LDS whole: k = 200 beyond 80 kept columns, or > 128 kept)
    # has the same guarded loads: the steady chunks with unguarded ones are bit-identical but
    # 12-55 % slower at k = 160-200 (r05al): not adopted
    "rot_chunk_unc": {"patch": "rot_chunk_unc"},
    # round 6: the wide-load rotation (k_rotate_wide: 16 B/lane, two MFMAs per V operand, clamped
    # unguarded loads, three batches in flight, next tile's loads before the stores) for 17-64 kept
    "rotw_off": {"NKV_ROTW": 0},   # the rotation before r06
    "rotw_w4": {"NKV_ROTW_W": 4},
    "rotw_w16": {"NKV_ROTW_W": 16},
    "rotw_u2": {"NKV_ROTW_U": 2},
    "rotw_mb8": {"NKV_ROTW_MAX_MB": 8},
    # timing-only diagnostics (wrong results), tools/experiments/rotw_diag.patch: 1 = L2-resident rows
    # (issue / MFMA ceiling), 2 = VALU adds instead of MFMAs (access-pattern ceiling); APRE: V operands
    # of a batch read from LDS before its first MFMA
    "rotw_diag1": {"patch": "rotw_diag", "NKV_ROTW_DIAG": 1},
    "rotw_diag2": {"patch": "rotw_diag", "NKV_ROTW_DIAG": 2},
    "rotw_apre": {"patch": "rotw_diag", "NKV_ROTW_APRE": 1},
    # the diagnostics above: the L2-resident MFMA stream runs at 9 TB/s-equivalent, the access pattern
    # alone (no MFMA) at 5.3 -> the persistent grid's drift, not the MFMAs, limits 17-32 kept; row bands
    "rotw_r0": {"NKV_ROTW_ROUNDS": 0},
    "rotw_r1": {"NKV_ROTW_ROUNDS": 1},
    "rotw_r4": {"NKV_ROTW_ROUNDS": 4},
    "rotw_r8": {"NKV_ROTW_ROUNDS": 8},
    "rotw_r2_diag2": {"patch": "rotw_diag", "NKV_ROTW_ROUNDS": 2, "NKV_ROTW_DIAG": 2},
    # the LDS-staged rotation (k_rotate_glds, tools/experiments/rot_glds.patch: 1 KiB one-column
    # LDS-DMA loads, MFMA fragments from LDS, outputs transposed through LDS into 1 KiB one-column
    # stores): 5-15 % slower than the wide-load kernel at 20-64 kept columns, k = 64-200 (r06k), not
    # adopted; in r06f-k the product's "base" was this kernel and "rotg_off" the wide-load one
    "rot_glds": {"patch": "rot_glds"},
    "rotg_d6": {"patch": "rot_glds", "NKV_ROTG_D": 6},
    "rotg_d5": {"patch": "rot_glds", "NKV_ROTG_D": 5},
    "rot_old": {"NKV_ROTW": 0},   # the rotation before round 6
    "rw_ntst0": {"NKV_NT_ST": 0},   # cached stores (every streaming kernel)
    "rw_nt0": {"NKV_NT": 0},        # cached loads
    "rw_nt00": {"NKV_NT": 0, "NKV_NT_ST": 0},
    # the VALU few-column rotation past 16 kept columns (NO accumulators per row pair,
    # tools/experiments/rotf_wide.patch): 11-60 % slower than the wide-load MFMA kernel at 20-32 kept,
    # k = 64-200 (r06u), not adopted
    # round 6: the multi-dot's L1 request queue is full (TA stalled by the TC 34 % of cycles, r06e):
    # the same bytes in flight per CU spread over more waves with fewer loads each
    "d2p4_b512": {"NKV_D2_PAIRS": 4, "NKV_D2_MAXB": 512},
    "d2p4_b256": {"NKV_D2_PAIRS": 4},
    "d2p2_b1024": {"NKV_D2_PAIRS": 2, "NKV_D2_MAXB": 1024},
    "d2p8_u1_b512": {"NKV_D2_U": 1, "NKV_D2_MAXB": 512},
    "d2p4_u4_b256": {"NKV_D2_PAIRS": 4, "NKV_D2_U": 4},
    "rotf32": {"patch": "rotf_wide", "NKV_ROTF_MAX": 32},
    "rotf32_p2": {"patch": "rotf_wide", "NKV_ROTF_MAX": 32, "NKV_ROTF_P_WIDE": 2},
    # workgroup visits of NKV_ROTW_SPAN consecutive tiles (SPAN 16 = 4096 rows per column) in row-band
    # launches (tools/experiments/rotw_span.patch): tools/write_streams.hip's plain shape gains 6 % from
    # 16-64 bands of 4096-row tiles, the wide-load rotation within +-1 % (r06o): not adopted
    "rotw_s16": {"patch": "rotw_span", "NKV_ROTW_SPAN": 16},
    "rotw_s16_r1": {"patch": "rotw_span", "NKV_ROTW_SPAN": 16, "NKV_ROTW_ROUNDS": 1},
    "rotw_s16_r2": {"patch": "rotw_span", "NKV_ROTW_SPAN": 16, "NKV_ROTW_ROUNDS": 2},
    "rotw_s4_r4": {"patch": "rotw_span", "NKV_ROTW_SPAN": 4, "NKV_ROTW_ROUNDS": 4},
    "rotw_s8_r2": {"patch": "rotw_span", "NKV_ROTW_SPAN": 8, "NKV_ROTW_ROUNDS": 2},
    "rotw_s32_r1": {"patch": "rotw_span", "NKV_ROTW_SPAN": 32, "NKV_ROTW_ROUNDS": 1},
}


def variant_sources(name: str, out_dir: str = VDIR) -> list:
    """The variant's translation units: a copy of the product's csrc/ (sources + nkv_internal.h), with
    the variant's patch applied if it has one (``patch`` fails loudly when the diff no longer applies)."""
    import shutil

    import __graft_entry__ as ge

    d = os.path.join(out_dir, f"src_{name}")
    if os.path.isdir(d):
        shutil.rmtree(d)
    shutil.copytree(PRODUCT_CSRC, d)
    pname = VARIANTS[name].get("patch")
    if pname:
        subprocess.run(["patch", "-s", "-p1", "-d", d, "-i", os.path.join(EXP_DIR, pname + ".patch")], check=True)
    return [os.path.join(d, os.path.basename(src)) for src in ge.HIP_SRCS]


def variant_defines(name: str) -> list:
    return [f"-D{k}={v}" for k, v in VARIANTS[name].items() if k != "patch"]


def build(names):
    import __graft_entry__ as ge

    os.makedirs(VDIR, exist_ok=True)
    for n in names:   # each build compiles its translation units in parallel
        ge.build_hip(variant_sources(n), lib=os.path.join(VDIR, f"lib_{n}.so"),
                     obj_dir=os.path.join(VDIR, f"obj_{n}"), extra_flags=variant_defines(n))


def run(names, E, rounds, js, only=None):
    import numpy as np
    import torch

    from nekstab_next_amd import _lib
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    libs = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(VDIR, f"lib_{n}.so"))
        for name, (res, args) in _lib._SIGNATURES.items():
            if not hasattr(L, name):   # an older build compared against this one
                continue
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        libs[n] = L
    lay = box3d_layout(E)
    jmax = max(js)
    dev = torch.device("cuda", 0)
    Lc = lay.c_struct()
    ldpad = int(os.environ.get("NKV_TUNE_LDPAD", "0"))   # extra doubles of column stride (multiple of 4096,
    # or any even number with the "ldany" build)
    svpad = int(os.environ.get("NKV_TUNE_SVPAD", "0"))   # extra 4096-row tiles per field segment (field stride)
    if svpad:
        Lc.sv += 4096 * svpad
        Lc.ld = -(-(Lc.n_wf * Lc.sv + Lc.sp + 1) // 4096) * 4096
    Lc.ld += ldpad
    Lp = ctypes.byref(Lc)
    Q = torch.empty((jmax + 1, Lc.ld), dtype=torch.float64, device=dev)
    lib0 = libs[names[0]]
    st = torch.cuda.current_stream().cuda_stream
    for i in range(jmax + 1):
        _lib.check(lib0.nkv_fill_hash(Lp, Q[i].data_ptr(), 100 + i, 0, 0, st), "fill")
    f = torch.empty(Lc.ld, dtype=torch.float64, device=dev)
    _lib.check(lib0.nkv_fill_hash(Lp, f.data_ptr(), 5, 0, 0, st), "fill")
    w = torch.zeros(Lc.sv, dtype=torch.float64, device=dev)
    w[: lay.n_v] = torch.as_tensor(syn.mass_weights(lay)).to(dev)
    ws = torch.zeros((lib0.nkv_workspace_bytes(Lp, jmax + 1) + 7) // 8 + 4096 * (jmax + 2), dtype=torch.float64, device=dev)
    h = torch.full((jmax + 1,), 1e-3, dtype=torch.float64, device=dev)
    h2 = torch.zeros(jmax + 1, dtype=torch.float64, device=dev)
    nrm = torch.zeros(8, dtype=torch.float64, device=dev)
    N, Nw, nv = lay.N, lay.N_w, lay.n_v
    V = torch.eye(jmax, dtype=torch.float64, device=dev).flatten()  # rotation by I keeps Q bounded
    if os.environ.get("NKV_TUNE_VRAND", "0") == "1":   # a dense orthogonal V (the MFMAs on real data,
        # as a restart's Schur vectors; orthonormal columns keep the repeatedly rotated Q bounded)
        V = torch.as_tensor(np.linalg.qr(np.random.default_rng(5).standard_normal((jmax, jmax)))[0].ravel(order="F").copy()).to(dev)
    hd = torch.zeros(2 * (jmax + 1), dtype=torch.float64, device=dev)
    f2 = torch.zeros(Lc.ld, dtype=torch.float64, device=dev)
    dgl = torch.full((Lc.ld,), 0.5, dtype=torch.float64, device=dev)
    nrm1 = torch.ones(8, dtype=torch.float64, device=dev)
    coefs = {}
    for jj in js:   # DCGS2 coefficients for m = jj-1: small x, y, a; rinv = s = 1 (vectors stay bounded)
        mm = jj - 1
        cj = torch.full((4 * jmax + 8,), 1e-4, dtype=torch.float64, device=dev)
        cj[2 * mm + 1] = 1.0
        cj[2 * mm + 4] = 1.0
        coefs[jj] = cj

    def ops(L, j):
        return {
            "dot": (lambda: L.nkv_block_dot(Lp, w.data_ptr(), Q.data_ptr(), j, f.data_ptr(), h2.data_ptr(), ws.data_ptr(), 0, st),
                    8.0 * (j * Nw + Nw + nv)),
            "update_norm": (lambda: L.nkv_block_update(Lp, w.data_ptr(), Q.data_ptr(), j, h.data_ptr(), f.data_ptr(), nrm.data_ptr(), ws.data_ptr(), 0x1 | 0x8, st),
                            8.0 * (j * N + 2 * N + nv)),
            "update_dot": (lambda: L.nkv_block_update_dot(Lp, w.data_ptr(), Q.data_ptr(), j, h.data_ptr(), f.data_ptr(), h2.data_ptr(), ws.data_ptr(), 0x1, st),
                           8.0 * (j * N + 2 * N + nv)),
            "dot2": (lambda: L.nkv_block_dot2(Lp, w.data_ptr(), Q.data_ptr(), j, Q[j - 1].data_ptr(), f.data_ptr(),
                                              hd.data_ptr(), ws.data_ptr(), 0x20 if hasattr(L, "nkv_dcgs2_coef") else 0,
                                              st),
                     8.0 * ((j - 1) * Nw + 2 * Nw + nv)),
            "dcgs2_update": (lambda: L.nkv_dcgs2_update(Lp, w.data_ptr(), Q.data_ptr(), j - 1, coefs[j].data_ptr(),
                                                        Q[j - 1].data_ptr(), f.data_ptr(), f2.data_ptr(), nrm.data_ptr(),
                                                        ws.data_ptr(), 0x1, st),
                             8.0 * ((j - 1) * N + 4 * N + nv)),
            "dcgs2_upd0": (lambda: L.nkv_dcgs2_update(Lp, w.data_ptr(), Q.data_ptr(), j - 1, coefs[j].data_ptr(),
                                                      Q[j - 1].data_ptr(), f.data_ptr(), f2.data_ptr(), None,
                                                      ws.data_ptr(), 0x1, st),
                           8.0 * ((j - 1) * N + 4 * N)),
            "dcgs2_inpl": (lambda: L.nkv_dcgs2_update(Lp, w.data_ptr(), Q.data_ptr(), j - 1, coefs[j].data_ptr(),
                                                      Q[j - 1].data_ptr(), f2.data_ptr(), f2.data_ptr(), None,
                                                      ws.data_ptr(), 0x1, st),
                           8.0 * ((j - 1) * N + 4 * N)),
            "axpy_dot": (lambda: L.nkv_axpy_dot(Lp, w.data_ptr(), f2.data_ptr(), nrm1.data_ptr(), Q[0].data_ptr(),
                                                Q[1].data_ptr(), nrm.data_ptr(), ws.data_ptr(), 0x1, st)
                         if hasattr(L, "nkv_axpy_dot") else 0, 8.0 * (3 * N + Nw + nv)),
            "finish": (lambda: L.nkv_arnoldi_finish(Lp, f.data_ptr(), nrm1.data_ptr(), f2.data_ptr(), 0, None, None,
                                                    None, 0, st), 16.0 * N),
            "op_diag": (lambda: L.nkv_op_diag(Lp, dgl.data_ptr(), f.data_ptr(), f2.data_ptr(), 0.0, st), 24.0 * N),
            "rotate": (lambda: L.nkv_rotate(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, st), 16.0 * j * N),
            "rotate_6": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, 6, st), 8.0 * (j + 6) * N),
            "rotate_12": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, min(12, j), st),
                          8.0 * (j + min(12, j)) * N),
            "rotate_16": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, min(16, j), st),
                          8.0 * (j + min(16, j)) * N),
            "rotate_32": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, min(32, j), st),
                          8.0 * (j + min(32, j)) * N),
            "rotate_64": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, min(64, j), st),
                          8.0 * (j + min(64, j)) * N),
            **{f"rotate_{n}": ((lambda n=n: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, min(n, j), st)),
                               8.0 * (j + min(n, j)) * N) for n in (20, 25, 40, 48)},
            "rotate_half": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, max(1, j // 2), st),
                            8.0 * (j + max(1, j // 2)) * N),
            "rotate_part": (lambda: L.nkv_rotate_cols(Lp, Q.data_ptr(), j, V.data_ptr(), jmax, max(1, j // 6), st),
                            8.0 * (j + max(1, j // 6)) * N),
        }

    res = {}
    for r in range(rounds):
        for n in names:
            for j in js:
                for opname, (fn, nbytes) in ops(libs[n], j).items():
                    if only and opname not in only:
                        continue
                    if opname == "rotate_part" and not hasattr(libs[n], "nkv_rotate_cols"):
                        continue
                    fn()  # warm
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    reps = 3
                    for _ in range(reps):
                        rc = fn()
                        assert rc == 0, (n, opname, rc)
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / reps
                    res.setdefault((n, j, opname), []).append(nbytes / (ms * 1e-3) / 1e9)
    out = {}
    for (n, j, op), v in sorted(res.items()):
        out[f"{n} j={j} {op}"] = dict(median_gbs=float(np.median(v)), min_gbs=float(np.min(v)), max_gbs=float(np.max(v)))
        extra = ""
        if op == "rotate":  # 2 N k^2 flop over 16 N k bytes
            tf = np.median(v) * 1e9 / (16.0 * j * N) * 2.0 * N * j * j / 1e12
            extra = f"  = {tf:.1f} TFLOP/s fp64"
        print(f"{n:10s} j={j:4d} {op:12s} median {np.median(v):8.1f} GB/s  (min {np.min(v):.1f}){extra}", flush=True)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["build", "run"])
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--E", type=int, default=44176)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--js", default="32,128")
    ap.add_argument("--ops", default="", help="comma list (default: all)")
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "tune.json"))
    a = ap.parse_args()
    names = a.variants.split(",")
    if a.cmd == "build":
        build(names)
    else:
        out = run(names, a.E, a.rounds, [int(x) for x in a.js.split(",")],
                  [x for x in a.ops.split(",") if x])
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        json.dump(out, open(a.out, "w"), indent=1)
