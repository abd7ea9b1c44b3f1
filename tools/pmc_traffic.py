#!/usr/bin/env python
"""Turn two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, MI355X_MICROARCH.md
§HBM) of ``bench.py`` into per-launch HBM traffic per kernel family
(a "launch" = one entry-point call, which may be several back-to-back row-band dispatches).

gfx950 corrections (MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7): counters are in KiB;
FETCH_SIZE reports exactly half of a wide (16 B/lane) coalesced streaming read, so it is doubled
(all our streaming loads are 16 B/lane double2 loads; the copy kernel k_blas1<COPY> calibrates it:
N*8 bytes read -> FETCH_SIZE*2*1024); WRITE_SIZE is exact for 16 B/lane stores.

usage: tools/pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_JSON OUT_JSON [--tag T --head H --box B]
"""
import collections
import csv
import json
import os
import sys

FAMILIES = {
    "block_dot": ("k_block_dot<",),
    "block_dot2": ("k_block_dot2<",),
    "dcgs2_update": ("k_dcgs2_update<",),
    "block_update": ("k_block_update",),
    "update_dot": ("k_update_dot",),
    "finish": ("k_finish",),
    "op_diag": ("k_op_diag",),
    "copy": ("k_blas1<1>",),
    # restart rotations of bench.py's restart leg (k_rotate_few: 16 B/lane loads; k_rotate_stream:
    # 8 B/lane loads, so its rows show how far the x2 FETCH correction holds for narrower loads)
    "rotate_kept": ("k_rotate_few<", "k_rotate_stream<1, 1,"),
    "rotate_full": ("k_rotate_stream<1, 8,",),
}


BANDED = ("dcgs2_update", "op_diag", "rotate_kept")  # families whose entry points issue row-band dispatches


def load(d):
    """Per-CALL counter values per family.  One entry-point call may issue several dispatches back
    to back (the row bands of the DCGS2 update, NKV_DC_ROUNDS; of the diagonal matvec,
    NKV_STREAM_ROUNDS; of the few-column restart rotation, NKV_ROTF_ROUNDS): a call = a run of
    consecutive dispatches of one family in dispatch order (k_reduce_cols, the second reduction
    stage, does not end a run); its value is their sum."""
    rows = sorted(csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))),
                  key=lambda r: int(r["Dispatch_Id"]))
    out = collections.defaultdict(list)
    cur_fam, cur = None, None
    for r in rows:
        fam = fam_of(r["Kernel_Name"])
        if fam is not None and fam == cur_fam and fam in BANDED:
            cur[0] += float(r["Counter_Value"])
            cur[1] += 1
            continue
        if fam is None and "k_reduce_cols" in r["Kernel_Name"]:
            continue
        if cur_fam is not None:
            out[cur_fam].append(tuple(cur))
        cur_fam, cur = fam, ([float(r["Counter_Value"]), 1] if fam is not None else None)
    if cur_fam is not None:
        out[cur_fam].append(tuple(cur))
    return out


def fam_of(name):
    for fam, keys in FAMILIES.items():
        if any(k in name for k in keys):
            return fam
    return None


def main():
    fdir, wdir, bench_json, out_json = sys.argv[1:5]
    opt = dict(zip(sys.argv[5::2], sys.argv[6::2]))
    F, W = load(fdir), load(wdir)
    bench = json.load(open(bench_json))
    agg = {}
    for fam in FAMILIES:
        fv = [v for v, _ in F.get(fam, [])]
        wv = [v for v, _ in W.get(fam, [])]
        if not fv:
            continue
        rd = 2.0 * 1024.0 * sum(fv) / len(fv)
        wr = 1024.0 * sum(wv) / len(wv) if wv else 0.0
        disp = sum(n for _, n in F[fam]) / len(fv)
        agg[fam] = dict(launches=len(fv), dispatches_per_launch=disp, read_bytes_per_launch=rd,
                        write_bytes_per_launch=wr, hbm_bytes_per_launch=rd + wr)
    dom = bench["roofline"]["kernel"]
    rec = dict(kernel_family=dom, E=bench["config"]["E"], m=bench["config"]["m"],
               hbm_bytes_per_launch=agg.get(dom, {}).get("hbm_bytes_per_launch"),
               algorithmic_bytes_per_launch=bench["roofline"]["avg_bytes_per_launch"],
               families=agg, correction="FETCH_SIZE x2 (16 B/lane streaming reads on gfx950), KiB -> bytes",
               source=[os.path.relpath(fdir), os.path.relpath(wdir)], tag=opt.get("--tag"),
               head=opt.get("--head"), box=opt.get("--box"))
    json.dump(rec, open(out_json, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
