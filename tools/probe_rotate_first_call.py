#!/usr/bin/env python
"""Kept-column restart rotation at config 3 (N=1e8, k=128), each shape called three times in a fresh
process, event-bracketed on the launch stream: is the bench line's single-call figure (18.4 ms for
6 kept columns vs 16.2 ms of summed kernel time) the kernel's rate or a first-launch cost?

  python tools/probe_rotate_first_call.py [n_out ...]      (default: 6 26)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout
    from nekstab_next_amd.vector import NekContext

    outs = [int(a) for a in sys.argv[1:]] or [6, 26]
    k = 128
    lay = box3d_layout(44176)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=k + 1)
    Q = ctx.basis(k + 1)
    for i in range(k + 1):
        Q[i].fill_hash(100 + i)
    rng = np.random.default_rng(5)
    stream = torch.cuda.current_stream()
    for n_out in outs:
        V = torch.as_tensor(np.linalg.qr(rng.standard_normal((k, k)))[0][:, :n_out].ravel(order="F").copy()).cuda()
        gb = 8.0 * lay.N * (k + n_out) / 1e9
        for call in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(stream)
            ctx.call("nkv_rotate_cols", Q.ptr, k, V.data_ptr(), k, n_out, ctx.stream)
            e1.record(stream)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            print(f"n_out={n_out:3d} call {call}: {ms:8.3f} ms  {gb / ms * 1e3:7.1f} GB/s", flush=True)
    ctx.check_nan()


if __name__ == "__main__":
    main()
