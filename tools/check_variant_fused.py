#!/usr/bin/env python
"""Bit-compare the fused CGS2 middle pass (nkv_block_update_dot: f -= Q h and h2 = Q^T W f) of two
tune-tool builds (tools/variants/lib_<name>.so) on the same inputs, for several j and sizes (small
tiles, large tiles, ragged shards).  A schedule change of the pass must leave f and h2 identical.

usage (on the MI355X box): python tools/check_variant_fused.py BASE_VARIANT NEW_VARIANT
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
    bad = 0
    for E in (7, 200, 2000):
        lay = box3d_layout(E)
        Lc = lay.c_struct()
        Lp = ctypes.byref(Lc)
        w = torch.zeros(Lc.sv, dtype=torch.float64, device=dev)
        w[: lay.n_v] = torch.as_tensor(syn.mass_weights(lay)).to(dev)
        for j in (1, 3, 8, 12, 13, 31, 64, 128):
            outs = []
            h = torch.as_tensor(np.random.default_rng(j).standard_normal(j) * 1e-2).to(dev)
            for L in libs:
                Q = torch.zeros((j, Lc.ld), dtype=torch.float64, device=dev)
                for i in range(j):
                    _lib.check(L.nkv_fill_hash(Lp, Q[i].data_ptr(), 900 + i, 0, 0, st), "fill")
                f = torch.zeros(Lc.ld, dtype=torch.float64, device=dev)
                _lib.check(L.nkv_fill_hash(Lp, f.data_ptr(), 17, 0, 0, st), "fill")
                ws = torch.zeros((L.nkv_workspace_bytes(Lp, j + 1) + 7) // 8, dtype=torch.float64, device=dev)
                h2 = torch.zeros(j, dtype=torch.float64, device=dev)
                _lib.check(L.nkv_block_update_dot(Lp, w.data_ptr(), Q.data_ptr(), j, h.data_ptr(), f.data_ptr(),
                                                  h2.data_ptr(), ws.data_ptr(), 0x1, st), "update_dot")
                torch.cuda.synchronize()
                outs.append((f.cpu().numpy(), h2.cpu().numpy()))
            same = np.array_equal(outs[0][0], outs[1][0]) and np.array_equal(outs[0][1], outs[1][1])
            df = float(np.max(np.abs(outs[0][0] - outs[1][0])))
            dh = float(np.max(np.abs(outs[0][1] - outs[1][1])) / max(np.max(np.abs(outs[0][1])), 1e-300))
            print(f"E={E:5d} j={j:4d} bit-identical={same} max|df|={df:.3e} max|dh|/|h|={dh:.3e}", flush=True)
            bad += 0 if same else 1
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
