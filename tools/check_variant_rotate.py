#!/usr/bin/env python
"""Bit-compare the restart rotation of two tune-tool builds (tools/variants/lib_<name>.so) on the
same inputs: nkv_rotate_cols over a hashed basis for several (k, n_out).  Used before a layout or
schedule change of a rotation kernel moves from the experiment copy into the product (the MFMA
accumulation order must not change, so the results must be identical bit for bit).

usage (on the MI355X box): python tools/check_variant_rotate.py BASE_VARIANT NEW_VARIANT [--report-only]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from nekstab_next_amd import _lib
    from nekstab_next_amd.layout import box3d_layout

    libs = []
    for n in sys.argv[1:3]:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"lib_{n}.so"))
        for name, (res, args) in _lib._SIGNATURES.items():
            if not hasattr(L, name):   # a build older than the current ABI
                continue
            fn = getattr(L, name)
            fn.restype, fn.argtypes = res, args
        libs.append(L)
    lay = box3d_layout(200)
    Lc = lay.c_struct()
    Lp = ctypes.byref(Lc)
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", 0)
    bad = 0
    for k, n_out in ((128, 128), (128, 20), (128, 25), (128, 64), (37, 33), (200, 17), (96, 96), (150, 40),
                     (200, 100), (200, 200), (257, 129), (1000, 40), (100, 17), (130, 48), (64, 64), (17, 17),
                     (129, 33), (83, 70), (128, 65), (150, 100)):
        outs = []
        V = torch.as_tensor(np.random.default_rng(k * 1000 + n_out).standard_normal((n_out, k))).to(dev)
        for L in libs:
            Q = torch.empty((k + 1, Lc.ld), dtype=torch.float64, device=dev)
            for i in range(k + 1):
                _lib.check(L.nkv_fill_hash(Lp, Q[i].data_ptr(), 700 + i, 0, 0, st), "fill")
            _lib.check(L.nkv_rotate_cols(Lp, Q.data_ptr(), k, V.data_ptr(), k, n_out, st), "rotate")
            torch.cuda.synchronize()
            outs.append(Q.cpu().numpy())
        same = np.array_equal(outs[0], outs[1])
        diff = float(np.max(np.abs(outs[0] - outs[1])))
        print(f"k={k:4d} n_out={n_out:4d} bit-identical={same} max|diff|={diff:.3e}", flush=True)
        bad += 0 if same else 1
    sys.exit(1 if bad and "--report-only" not in sys.argv else 0)


if __name__ == "__main__":
    main()
