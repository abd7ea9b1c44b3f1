#!/usr/bin/env python
"""The two-vector multi-dot in isolation and in the Arnoldi step's context, at BASELINE's N=1e8.

Isolated: the same ``nkv_block_dot2`` call three times back to back (as tools/tune_kernels.py times it).
In context: the DCGS2 step's order — dual update (writes two vectors), the synthetic matvec (writes
one), then the multi-dot — with HIP events around the multi-dot only.  Variants are libraries built by
``tools/tune_kernels.py build`` (``base`` = the product source).  Prints one line per (variant, j, mode).

  python tools/dot2_context.py --variants base,ntst0 --js 64,128
"""
import argparse
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="base")
    ap.add_argument("--js", default="64,128")
    ap.add_argument("--E", type=int, default=44176)
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    import torch

    from nekstab_next_amd import _lib
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    names = a.variants.split(",")
    js = [int(x) for x in a.js.split(",")]
    libs = {}
    for n in names:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"lib_{n}.so"))
        for name, (res, args) in _lib._SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, args
        libs[n] = L
    lay = box3d_layout(a.E)
    Lc = lay.c_struct()
    Lp = ctypes.byref(Lc)
    dev = torch.device("cuda", 0)
    jmax = max(js)
    st = torch.cuda.current_stream().cuda_stream
    Q = torch.empty((jmax + 1, Lc.ld), dtype=torch.float64, device=dev)
    lib0 = libs[names[0]]
    for i in range(jmax + 1):
        _lib.check(lib0.nkv_fill_hash(Lp, Q[i].data_ptr(), 100 + i, 0, 0, st), "fill")
    f = torch.empty(Lc.ld, dtype=torch.float64, device=dev)
    _lib.check(lib0.nkv_fill_hash(Lp, f.data_ptr(), 5, 0, 0, st), "fill")
    f2 = torch.zeros(Lc.ld, dtype=torch.float64, device=dev)
    w = torch.zeros(Lc.sv, dtype=torch.float64, device=dev)
    w[: lay.n_v] = torch.as_tensor(syn.mass_weights(lay)).to(dev)
    ws = torch.zeros((lib0.nkv_workspace_bytes(Lp, jmax + 1) + 7) // 8 + 4096 * (jmax + 2), dtype=torch.float64,
                     device=dev)
    hd = torch.zeros(2 * (jmax + 1), dtype=torch.float64, device=dev)
    dgl = torch.full((Lc.ld,), 0.5, dtype=torch.float64, device=dev)
    Nw, nv = lay.N_w, lay.n_v
    res = {}
    for _ in range(a.rounds):
        for n in names:
            L = libs[n]
            for j in js:
                m = j - 1
                cj = torch.full((4 * jmax + 8,), 1e-4, dtype=torch.float64, device=dev)
                cj[2 * m + 1] = 1.0
                cj[2 * m + 4] = 1.0
                x = Q[j - 1]
                nbytes = 8.0 * ((j - 1) * Nw + 2 * Nw + nv)

                def dot2():
                    assert L.nkv_block_dot2(Lp, w.data_ptr(), Q.data_ptr(), j, x.data_ptr(), f.data_ptr(),
                                            hd.data_ptr(), ws.data_ptr(), 0x20, st) == 0

                def update():   # writes x (the finished column) and f2; x stays bounded (rinv = s = 1)
                    assert L.nkv_dcgs2_update(Lp, w.data_ptr(), Q.data_ptr(), m, cj.data_ptr(), x.data_ptr(),
                                              f.data_ptr(), f2.data_ptr(), None, ws.data_ptr(), 0x1, st) == 0

                def matvec():   # y = A u into f (the multi-dot's second right-hand side)
                    assert L.nkv_op_diag(Lp, dgl.data_ptr(), f2.data_ptr(), f.data_ptr(), 0.0, st) == 0

                for mode in ("isolated", "context"):
                    ts = []
                    for _r in range(3):
                        if mode == "context":
                            update()
                            matvec()
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        dot2()
                        e1.record()
                        torch.cuda.synchronize()
                        ts.append(e0.elapsed_time(e1))
                    res.setdefault((n, j, mode), []).append(nbytes / (np.median(ts) * 1e-3) / 1e9)
    for (n, j, mode), v in sorted(res.items()):
        print(f"{n:10s} j={j:4d} {mode:9s} median {np.median(v):8.1f} GB/s  (min {np.min(v):.1f})", flush=True)


if __name__ == "__main__":
    main()
