#!/usr/bin/env python
"""How many dispatches one entry-point call issues, per kernel instantiation and layout — the
host-side launch arithmetic of the banded entry points restated, so that
profile tools can split a run of back-to-back dispatches of one kernel into calls:

* ``k_dcgs2_update<P, false>`` (nkv_dcgs2_update without the fused norm,
  csrc/gram_schmidt.hip band_tiles): NKV_DC_ROUNDS grid-stride rounds of a min(tiles, NKV_DC_G,
  NKV_MAXB)-block grid per launch, all tiles in one launch when fewer than two bands;
  ``<P, true>`` (fused norm) is one launch;
* ``k_op_diag`` (nkv_op_diag, csrc/operators.hip): NKV_STREAM_ROUNDS rounds of a grid_for(rows/2)
  grid per launch, one launch when fewer than two bands;
* ``k_rotate_few<NO, P, U>`` (nkv_rotate_cols, csrc/rotate.hip launch_rotate_few):
  NKV_ROTF_ROUNDS rounds of a min(tiles, NKV_ROTF_G) grid per launch;
* ``k_rotate_wide<MB, W, U>`` (17-64 kept columns): one launch while NKV_ROTW_ROUNDS = 0 (the
  default; a banded build's grid comes from the runtime occupancy query, so it is not modelled and
  ``dispatches_per_call`` refuses it);
* everything else: one dispatch per call.

The knob values are read from the product sources (``#define NKV_...`` defaults), so a retuned
default is picked up; tests/test_profile_tools.py checks the model against the dispatch counts of
committed rocprofv3 kernel traces.
"""
import math
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nekstab_next_amd", "csrc")
K_THREADS = 256


def knobs() -> dict:
    """``#define NKV_NAME <int>`` defaults of the product sources (first definition wins)."""
    out = {}
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith((".h", ".hip")):
            continue
        for m in re.finditer(r"^#define (NKV_[A-Z0-9_]+) (-?\d+)\b", open(os.path.join(CSRC, f)).read(), re.M):
            out.setdefault(m.group(1), int(m.group(2)))
    return out


def _targs(name: str, kernel: str):
    m = re.search(re.escape(kernel) + r"<([^>]*)>", name)
    return [a.strip() for a in m.group(1).split(",")] if m else None


def dispatches_per_call(kernel_name: str, rows: int, kn: dict | None = None) -> int:
    """Dispatches of one call of the entry point that launches ``kernel_name`` over a vector of
    ``rows`` streamed rows (nkv_layout rows_of: n_wf*sv + sp)."""
    kn = kn or knobs()
    a = _targs(kernel_name, "k_dcgs2_update")
    if a is not None:
        P, nrm = int(a[0]), a[1] == "true"
        if nrm:
            return 1
        tiles = rows // (K_THREADS * P * 2)
        g = max(1, min(tiles, min(kn["NKV_DC_G"], kn["NKV_MAXB"])))
        if kn["NKV_DC_ROUNDS"] <= 0:
            return 1
        b = kn["NKV_DC_ROUNDS"] * g
        band = tiles if (b >= tiles or tiles < 2 * b) else b
        return max(1, math.ceil(tiles / max(band, 1)))
    if "k_op_diag(" in kernel_name or kernel_name.endswith("k_op_diag"):
        g = max(1, min(-(-(rows // 2) // K_THREADS), kn["NKV_STREAM_G"]))
        chunks = rows // (2 * K_THREADS * kn["NKV_STREAM_UNR"])
        r = kn["NKV_STREAM_ROUNDS"]
        band = r * g if (r > 0 and chunks >= 2 * r * g) else max(chunks, 1)
        return max(1, math.ceil(chunks / band))
    if _targs(kernel_name, "k_rotate_wide") is not None and kn.get("NKV_ROTW_ROUNDS", 0) > 0:
        raise NotImplementedError("banded k_rotate_wide: the grid is the runtime occupancy query's")
    a = _targs(kernel_name, "k_rotate_few")
    if a is not None:
        P = int(a[1])
        tiles = rows // (K_THREADS * P * 2)
        g = min(tiles, kn["NKV_ROTF_G"])
        band = kn["NKV_ROTF_ROUNDS"] * g if kn["NKV_ROTF_ROUNDS"] > 0 else tiles
        return max(1, math.ceil(tiles / max(band, 1)))
    return 1


def rows_of_E(E: int, n_scalars: int = 1) -> int:
    """Streamed rows of bench.py's config-3 layout (3-D lx1=8, lx2=6) at E elements."""
    import sys

    sys.path.insert(0, ROOT)
    from nekstab_next_amd.layout import box3d_layout

    return box3d_layout(E, n_scalars).rows
