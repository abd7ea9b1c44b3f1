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

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import launch_model  # noqa: E402

FAMILIES = {
    "block_dot": ("k_block_dot<",),
    "block_dot2": ("k_block_dot2<",),
    "dcgs2_update": ("k_dcgs2_update<",),
    "block_update": ("k_block_update",),
    "update_dot": ("k_update_dot",),
    "finish": ("k_finish",),
    "op_diag": ("k_op_diag",),
    "copy": ("k_blas1<1>",),
    # restart rotations of bench.py's restart leg: <= 16 kept columns (k_rotate_few, 16 B/lane loads),
    # 17-64 kept (k_rotate_wide, 16 B/lane; k_rotate_stream<1, 2..4 before round 6, 8 B/lane) and the
    # full k-column rotation (k_rotate_stream<1, 8,: 8 B/lane loads, where the x2 FETCH correction is
    # uncalibrated)
    "rotate_kept": ("k_rotate_few<",),
    "rotate_wide": ("k_rotate_wide<", "k_rotate_stream<1, 2,", "k_rotate_stream<1, 3,", "k_rotate_stream<1, 4,"),
    "rotate_full": ("k_rotate_stream<1, 8,",),
}


def load(d, rows, counter=None):
    """Per-CALL counter values per family.  One entry-point call may issue several dispatches back
    to back (the row bands of the DCGS2 update, NKV_DC_ROUNDS; of the diagonal matvec,
    NKV_STREAM_ROUNDS; of the few-column restart rotation, NKV_ROTF_ROUNDS), and the bench calls
    some entry points back to back (the restart leg's three kept-column rotations).  A call is
    therefore the number of dispatches the entry point issues at this layout
    (tools/launch_model.dispatches_per_call, from the kernel instantiation and ``rows``), counted
    off consecutive dispatches of the family; k_reduce_cols (the second reduction stage) is
    skipped; its value is their sum."""
    kn = launch_model.knobs()
    disp = {}   # dispatch id -> [kernel name, counter value summed over the dispatch's rows]
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if counter is not None and r["Counter_Name"] != counter:
            continue
        e = disp.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], 0.0])
        e[1] += float(r["Counter_Value"])
    out = collections.defaultdict(list)
    cur_fam, cur, left = None, None, 0
    for did in sorted(disp):
        name, value = disp[did]
        fam = fam_of(name)
        if fam is None and "k_reduce_cols" in name:
            continue
        if fam is not None and fam == cur_fam and left > 0:
            cur[0] += value
            cur[1] += 1
            left -= 1
            continue
        if cur_fam is not None:
            out[cur_fam].append(tuple(cur))
        cur_fam = fam
        if fam is not None:
            cur = [value, 1]
            left = launch_model.dispatches_per_call(name, rows, kn) - 1
        else:
            cur, left = None, 0
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
    bench = json.load(open(bench_json))
    rows = launch_model.rows_of_E(bench["config"]["E"])
    F, W = load(fdir, rows, "FETCH_SIZE"), load(wdir, rows, "WRITE_SIZE")
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
