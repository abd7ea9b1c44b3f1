"""Time nkv_gradm1 (bf_sensitivity's gradient, sensitivity.f90:170-199) on BASELINE-sized meshes.

  python tools/bench_gradm1.py [--lib path/to/libnekkrylov.so] [--reps 10]

3-D lx1=8 E=22,088 (config 5's mesh, 11.3M points per field) and 2-D lx1=6 E=22,728 (config 2's
cylinder-scaled mesh), one field and one mode (ldim fields) per launch.  Algorithmic traffic per
launch: the ldim coordinate arrays and the nfld fields read once, ldim * nfld gradients written."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from nekstab_next_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=_lib.LIB_PATH)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    _lib.load(a.lib)
    from seed_helpers import box_mesh_coords

    from nekstab_next_amd import synthetic as syn
    from nekstab_next_amd.layout import NekLayout
    from nekstab_next_amd.sensitivity import Gradm1, velocity_layout
    from nekstab_next_amd.vector import NekContext

    rows = []
    for ldim, lx1, ne in ((3, 8, (22, 22, 46)), (2, 6, (152, 150, 1))):
        nel = 22088 if ldim == 3 else 22728
        full = NekLayout(ldim=3, lx1=lx1, lx2=lx1 - 2, nelgv=int(np.prod(ne)))
        box = box_mesh_coords(full, ne if ldim == 3 else (ne[0], ne[1], 1), L=(1.0, 1.0, 2.0))
        pts = lx1 ** ldim
        if ldim == 2:   # the kl = 0 plane of each element of a one-layer box
            co = {k: box[k].reshape(-1, lx1, lx1 * lx1)[:, 0, :].ravel()[: nel * pts] for k in ("x", "y")}
        else:
            co = {k: box[k][: nel * pts] for k in ("x", "y", "z")}
        del box
        lay = velocity_layout(NekLayout(ldim=ldim, lx1=lx1, lx2=lx1 - 2, nelgv=nel))
        ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=2)
        op = Gradm1(ctx, co)
        v = ctx.vector()
        v.fill_hash(3)
        out = torch.empty(ldim * ldim * lay.sv, dtype=torch.float64, device=ctx.device)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for nfld in (1, ldim):
            op(v.ptr, out.data_ptr(), nfld=nfld, u_stride=lay.sv, g_stride=lay.sv)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.reps):
                op(v.ptr, out.data_ptr(), nfld=nfld, u_stride=lay.sv, g_stride=lay.sv)
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.reps
            byts = 8 * lay.n_v * (ldim + nfld + ldim * nfld)
            rows.append(dict(ldim=ldim, lx1=lx1, E=nel, nfld=nfld, ms=round(ms, 4),
                             gbs=round(byts / (ms * 1e-3) / 1e9, 1), frac=round(byts / (ms * 1e-3) / 8e12, 3)))
            print(json.dumps(rows[-1]), flush=True)
        del ctx, op, out, v
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
