#!/usr/bin/env python
"""Compare the two-vector multi-dot (nkv_block_dot2: Q^T W x and Q^T W y in one read of Q) of two
tune-tool builds (tools/variants/lib_<name>.so) on the same inputs, with and without
NKV_X_IS_LAST, at large-tile sizes (the column-split experiment changes only those) and one small
size.  A variant that keeps each block's tile set (same grid per column group) must be
bit-identical; one that changes the grid must agree to rounding (printed).

usage (on the MI355X box): python tools/check_variant_dot2.py BASE_VARIANT NEW_VARIANT
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
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    libs = []
    for n in sys.argv[1:3]:
        L = ctypes.CDLL(os.path.join(ROOT, "tools", "variants", f"lib_{n}.so"))
        for name, (res, args) in _lib._SIGNATURES.items():
            if hasattr(L, name):
                fn = getattr(L, name)
                fn.restype, fn.argtypes = res, args
        libs.append(L)
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", 0)
    worst = 0.0
    identical = True
    for E in (200, 5522):
        lay = box3d_layout(E)
        Lc = lay.c_struct()
        Lp = ctypes.byref(Lc)
        w = torch.zeros(Lc.sv, dtype=torch.float64, device=dev)
        w[: lay.n_v] = torch.as_tensor(syn.mass_weights(lay)).to(dev)
        jmax = 129
        Q = torch.zeros((jmax, Lc.ld), dtype=torch.float64, device=dev)
        for i in range(jmax):
            _lib.check(libs[0].nkv_fill_hash(Lp, Q[i].data_ptr(), 900 + i, 0, 0, st), "fill")
        y = torch.zeros(Lc.ld, dtype=torch.float64, device=dev)
        _lib.check(libs[0].nkv_fill_hash(Lp, y.data_ptr(), 17, 0, 0, st), "fill")
        for j in (1, 2, 33, 63, 64, 65, 66, 96, 127, 128, 129):
            for xlast in (False, True):
                x = Q[j - 1] if xlast else Q[jmax - 1 - (j % 3)]
                outs = []
                for L in libs:
                    ws = torch.zeros((L.nkv_workspace_bytes(Lp, jmax + 1) + 7) // 8, dtype=torch.float64, device=dev)
                    hd = torch.full((2 * j,), float("nan"), dtype=torch.float64, device=dev)
                    _lib.check(L.nkv_block_dot2(Lp, w.data_ptr(), Q.data_ptr(), j, x.data_ptr(), y.data_ptr(),
                                                hd.data_ptr(), ws.data_ptr(), 0x20 if xlast else 0, st), "dot2")
                    torch.cuda.synchronize()
                    outs.append(hd.cpu().numpy())
                same = np.array_equal(outs[0], outs[1])
                rel = float(np.max(np.abs(outs[0] - outs[1])) / max(np.max(np.abs(outs[0])), 1e-300))
                if not np.all(np.isfinite(outs[1])):
                    rel = float("inf")
                worst = max(worst, rel)
                identical &= same
                print(f"E={E:5d} j={j:4d} x_last={int(xlast)} bit-identical={same} max|dh|/|h|={rel:.3e}", flush=True)
    print(f"ALL bit-identical={identical} worst rel={worst:.3e}")
    return 0 if worst < 1e-13 else 1


if __name__ == "__main__":
    sys.exit(main())
