#!/usr/bin/env python
"""Vendor-library yardsticks for the two Gram–Schmidt kernel shapes at BASELINE size (N=1e8):
rocBLAS dgemv through torch (y = Q_j x: the multi-dot; f -= Q_j^T a: the update) and plain
streaming ops (copy, add, sum), next to this build's kernels on the same buffers.  Achieved GB/s
of the algorithmic bytes, median of 5 interleaved rounds, HIP events on the current stream.

  python tools/vendor_baseline.py   # on the MI355X box
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from nekstab_next_amd import _lib
    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import box3d_layout

    lib = _lib.load()
    lay = box3d_layout(44176)
    dev = torch.device("cuda", 0)
    jmax = 128
    Lc = lay.c_struct()
    Lp = _lib.ctypes.byref(Lc)
    st = torch.cuda.current_stream().cuda_stream
    Q = torch.empty((jmax + 1, lay.ld), dtype=torch.float64, device=dev)
    for i in range(jmax + 1):
        _lib.check(lib.nkv_fill_hash(Lp, Q[i].data_ptr(), 100 + i, 0, 0, st), "fill")
    Q.mul_(1e-2)
    x = torch.empty(lay.ld, dtype=torch.float64, device=dev)
    _lib.check(lib.nkv_fill_hash(Lp, x.data_ptr(), 5, 0, 0, st), "fill")
    y = torch.empty_like(x)
    z = torch.empty_like(x)
    w = torch.zeros(lay.sv, dtype=torch.float64, device=dev)
    w[: lay.n_v] = torch.as_tensor(syn.mass_weights(lay)).to(dev)
    ws = torch.zeros((lib.nkv_workspace_bytes(Lp, jmax + 1) + 7) // 8 + 4096 * (jmax + 2), dtype=torch.float64, device=dev)
    hd = torch.zeros(2 * (jmax + 1), dtype=torch.float64, device=dev)
    N, Nw, ld = lay.N, lay.N_w, lay.ld
    coefs = {}
    for j in (32, 64, 128):
        cj = torch.full((4 * jmax + 16,), 1e-4, dtype=torch.float64, device=dev)
        cj[2 * (j - 1) + 1] = 1.0
        cj[2 * (j - 1) + 4] = 1.0
        coefs[j] = cj

    def cases(j):
        a = torch.full((j,), 1e-3, dtype=torch.float64, device=dev)
        return {
            "rocblas_dgemv_dot  y=Q_j x": (lambda: torch.mv(Q[:j], x, out=hd[:j]), 8.0 * (j + 1) * ld),
            "rocblas_dgemv_upd  f-=Q_j^T a": (lambda: torch.addmv(x, Q[:j].t(), a, beta=1.0, alpha=-1.0, out=y),
                                             8.0 * (j + 2) * ld),
            "nkv_block_dot2 (2 RHS, weighted)": (
                lambda: lib.nkv_block_dot2(Lp, w.data_ptr(), Q.data_ptr(), j, Q[j - 1].data_ptr(), x.data_ptr(),
                                           hd.data_ptr(), ws.data_ptr(), 0x20, st),
                8.0 * ((j - 1) * Nw + 2 * Nw + lay.n_v)),
            "nkv_dcgs2_update (2 outputs)": (
                lambda: lib.nkv_dcgs2_update(Lp, w.data_ptr(), Q.data_ptr(), j - 1, coefs[j].data_ptr(),
                                             Q[j - 1].data_ptr(), x.data_ptr(), z.data_ptr(), None, ws.data_ptr(),
                                             0x1, st),
                8.0 * ((j - 1) * N + 4 * N)),
        }

    stream_cases = {
        "torch copy (1R 1W)": (lambda: y.copy_(x), 16.0 * ld),
        "torch add (2R 1W)": (lambda: torch.add(x, z, out=y), 24.0 * ld),
        "torch sum Q_64 (read only)": (lambda: torch.sum(Q[:64], dim=1, out=hd[:64]), 8.0 * 64 * ld),
    }
    res = {}
    for r in range(5):
        items = [(f"j={j} {k}", v) for j in (32, 64, 128) for k, v in cases(j).items()] + list(stream_cases.items())
        for name, (fn, nbytes) in items:
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                rc = fn()
                assert rc is None or isinstance(rc, torch.Tensor) or rc == 0, (name, rc)
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / 3
            res.setdefault(name, []).append(nbytes / (ms * 1e-3) / 1e9)
    out = {}
    for name, v in res.items():
        out[name] = float(np.median(v))
        print(f"{name:45s} {np.median(v):8.1f} GB/s  ({np.median(v) / 8000:.3f} of 8 TB/s)", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "vendor_baseline.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
