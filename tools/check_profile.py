#!/usr/bin/env python
"""Compare rocprofv3 --stats per-kernel-family average durations with bench.py's live HIP-event
phase timings (the bench's `roofline.avg_launch_ms` must agree with the profiler).

usage: tools/check_profile.py KERNEL_STATS_CSV BENCH_JSON   (run_kernel_trace.csv beside the stats
       file, when present, gives the per-launch comparison for families with unbracketed launches)
"""
import csv
import json
import os
import sys

FAM = {"block_dot": "k_block_dot<", "block_dot2": "k_block_dot2<", "dcgs2_update": "k_dcgs2_update<",
       "update_dot": "k_update_dot", "block_update": "k_block_update<false, true",
       "finish": "k_finish", "op_diag": "k_op_diag"}


def main():
    stats = list(csv.DictReader(open(sys.argv[1])))
    bench = json.load(open(sys.argv[2]))
    tpath = os.path.join(os.path.dirname(sys.argv[1]), "run_kernel_trace.csv")
    trace = list(csv.DictReader(open(tpath))) if os.path.exists(tpath) else None
    print(f"{'family':14s} {'rocprof calls':>13s} {'rocprof avg ms':>15s} {'events launches':>16s} {'events avg ms':>14s} {'ratio':>7s}")
    for fam, key in FAM.items():
        rows = [r for r in stats if key in r["Name"]]
        if not rows:
            continue
        calls = sum(int(r["Calls"]) for r in rows)
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        ph = bench.get("phases", {}).get(fam)
        ev = f"{ph['launches']:16d} {ph['avg_ms']:14.4f} {ph['avg_ms'] / (tot / calls / 1e6):7.3f}" if ph else ""
        print(f"{fam:14s} {calls:13d} {tot / calls / 1e6:15.4f} {ev}")
        if ph and trace and abs(ph["avg_ms"] / (tot / calls / 1e6) - 1.0) > 0.01:
            # the family also runs outside the bracketed launches (warm-up factorisations, the j=1
            # seed dots, the Krylov–Schur leg after the timed region).  DCGS2 step kernels run
            # exactly m times per factorisation, in order: compare the launches of the timed
            # factorisations; other families: the `launches` longest launches of the trace
            # one entry-point call may issue several dispatches back to back (the row bands of the
            # DCGS2 update, NKV_DC_ROUNDS): a call = a run of consecutive dispatches of the family in
            # the time-ordered trace; its duration spans first start .. last end (as the events do)
            allr = sorted(trace, key=lambda r: int(r["Start_Timestamp"]))
            calls_l, cur = [], None
            for r in allr:
                if key in r["Kernel_Name"]:
                    s0, e0 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    cur = [s0, e0, 1] if cur is None else [cur[0], e0, cur[2] + 1]
                elif cur is not None and "k_reduce_cols" not in r["Kernel_Name"]:
                    calls_l.append(cur)
                    cur = None
            if cur is not None:
                calls_l.append(cur)
            d = [(e - s0) / 1e6 for s0, e, _ in calls_l]
            m, w, st = bench["config"]["m"], bench["warmup"], bench["steps"]
            if fam in ("block_dot2", "dcgs2_update") and len(d) >= (w + st) * m and ph["launches"] == st * m:
                sel = calls_l[w * m:(w + st) * m]
                durs = d[w * m:(w + st) * m]
                label = "  (timed)" if all(c[2] == 1 for c in sel) else f"  (timed, {sel[0][2]} disp/call)"
            else:
                durs, label = sorted(d, reverse=True)[: ph["launches"]], "  (longest)"
            if durs:
                avg = sum(durs) / len(durs)
                print(f"{label:14s} {len(durs):13d} {avg:15.4f} {ph['launches']:16d} {ph['avg_ms']:14.4f} "
                      f"{ph['avg_ms'] / avg:7.3f}")
    print("(rocprof counts every launch incl. warm-up and the j=1 seed dots; events cover the timed steps; "
          "event brackets include the ~5 us second-stage reduction kernel)")
    rs = bench.get("restart")
    if rs:
        # restart rotations: n_out <= 16 kept columns (NKV_ROTF_MAX) run k_rotate_few<n_out, P, U>
        # (one dispatch per row band), wider ones k_rotate_stream<NB, MB, W, U> with
        # MB = ceil(n_out / 16) column blocks.  The kept shape runs 1 + 2 times (the solver's call,
        # then rotate_kept_steady twice, back to back), the full one twice: per call, the profiler's
        # summed kernel time over those calls, beside the steady event figure (the first call's
        # extra is a one-time launch cost outside the kernels)
        n_kept = rs["mstart"] - 1
        kept_key = f"k_rotate_few<{n_kept}," if n_kept <= 16 else f"k_rotate_stream<1, {(n_kept + 15) // 16},"
        steady = "rotate_kept_steady_ms" in rs
        for label, key, ms, ncall in (
                ("rotate kept", kept_key, rs.get("rotate_kept_steady_ms", rs["rotate_kept_ms"]), 3 if steady else 1),
                ("rotate full", "k_rotate_stream<1, 8,", rs["rotate_full_ms"], 2)):
            rows = [r for r in stats if key in r["Name"]]
            if rows:
                disp = sum(int(r["Calls"]) for r in rows)
                avg = sum(float(r["TotalDurationNs"]) for r in rows) / ncall / 1e6
                print(f"{label:14s} {ncall:13d} {avg:15.4f} {'':>16s} {ms:14.4f} {ms / avg:7.3f}"
                      f"  ({disp // ncall} disp/call)")

if __name__ == "__main__":
    main()
