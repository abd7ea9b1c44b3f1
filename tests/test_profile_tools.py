"""The measurement tools' grouping logic on small synthetic rocprofv3 CSVs (CPU only).

One entry-point call may issue several back-to-back dispatches (the row bands of the DCGS2 update,
the synthetic matvec and the few-column restart rotation).  tools/pmc_traffic.py must sum a call's
PMC values over its dispatches (k_reduce_cols does not end a call), and tools/check_profile.py must
time a call from its first dispatch's start to its last dispatch's end; two separate calls of the
full rotation must stay two calls."""
import csv
import importlib.util
import io
import json
import os
import sys
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

UPD = "void (anonymous namespace)::k_dcgs2_update<8, false>(double const*)"
DOT2 = "void (anonymous namespace)::k_block_dot2<8>(double const*)"
RED = "void (anonymous namespace)::k_reduce_cols(double const*)"
COEF = "void (anonymous namespace)::k_dcgs2_coef(int)"
ROTF = "void (anonymous namespace)::k_rotate_few<6, 4, 4>(double*)"
ROTS = "void (anonymous namespace)::k_rotate_stream<1, 8, 8, 8>(double*)"


def _tool(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "tools", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write_pmc(path, seq):
    """seq: (kernel name, counter value) in dispatch order."""
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        for i, (k, v) in enumerate(seq, 1):
            w.writerow([i, k, "FETCH_SIZE", v])


def test_pmc_traffic_sums_band_dispatches_per_call(tmp_path):
    pt = _tool("pmc_traffic")
    lm = _tool("launch_model")
    rows = 4608 * 4096   # 3 row bands of the DCGS2 update, 12 of the few-column rotation
    assert lm.dispatches_per_call(UPD, rows) == 3 and lm.dispatches_per_call(ROTF, rows) == 12
    # two DCGS2 steps: dot2 + its reduction, coef, then the update as 3 band dispatches
    seq = []
    for _ in range(2):
        seq += [(DOT2, 10.0), (RED, 0.5), (COEF, 0.1), (UPD, 1.0), (UPD, 2.0), (UPD, 3.0)]
    seq += [(ROTF, 4.0)] * 12   # one banded restart rotation (12 dispatches)
    d = tmp_path / "p"
    d.mkdir()
    _write_pmc(d / "run_counter_collection.csv", seq)
    out = pt.load(str(d), rows)
    assert out["dcgs2_update"] == [(6.0, 3), (6.0, 3)]       # k_reduce_cols/coef do not merge steps
    assert out["block_dot2"] == [(10.0, 1), (10.0, 1)]       # not banded: one dispatch per call
    assert out["rotate_kept"] == [(48.0, 12)]


def test_pmc_traffic_splits_back_to_back_calls(tmp_path):
    """bench.py's restart leg calls the kept-column rotation three times back to
    back; grouping by adjacency merged them (a phantom x1.5 over-fetch).  Calls are now counted off
    by the entry point's band count at the layout."""
    pt = _tool("pmc_traffic")
    rows = 4608 * 4096
    seq = [(ROTF, 1.0)] * 36 + [(UPD, 2.0)] * 6   # three rotations, then two dual updates, all adjacent
    d = tmp_path / "p"
    d.mkdir()
    _write_pmc(d / "run_counter_collection.csv", seq)
    out = pt.load(str(d), rows)
    assert out["rotate_kept"] == [(12.0, 12)] * 3
    assert out["dcgs2_update"] == [(6.0, 3)] * 2


def test_launch_model_matches_committed_traces():
    """The band counts the model derives for bench.py's layout (E=44,176) divide the dispatch counts
    of a committed full-size rocprofv3 trace into whole calls: the dual update and the diagonal
    matvec once per Arnoldi step (as many calls as multi-dots), the 6-kept rotation 3 times, the
    25-kept one (one dispatch per call) 3 times in the restart section + once in the restart leg."""
    lm = _tool("launch_model")
    rows = lm.rows_of_E(44176)
    calls = {}
    with open(os.path.join(ROOT, "profiles", "r06q_bench_n1_kernel_stats.csv")) as fh:
        for r in csv.DictReader(fh):
            calls[r["Name"]] = int(r["Calls"])
    n = {k: v for k, v in calls.items()}
    upd = next(k for k in n if "k_dcgs2_update<8, false>" in k)
    opd = next(k for k in n if "k_op_diag(" in k)
    rotf = next(k for k in n if "k_rotate_few<6, 4, 4>" in k)
    dot2 = next(k for k in n if "k_block_dot2<8>" in k)
    assert n[upd] == lm.dispatches_per_call(upd, rows) * n[dot2] == 16 * n[dot2]
    assert n[opd] == lm.dispatches_per_call(opd, rows) * n[dot2] == 6 * n[dot2]
    assert n[rotf] == 3 * lm.dispatches_per_call(rotf, rows) == 3 * 64
    rotw = next(k for k in n if "k_rotate_wide<2, 8, 4>" in k)
    assert n[rotw] == 4 * lm.dispatches_per_call(rotw, rows) == 4


def _write_trace(path, seq):
    """seq: (kernel name, start ns, end ns)."""
    with open(path, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for k, s, e in seq:
            w.writerow([k, s, e])


def test_check_profile_groups_calls(tmp_path):
    cp = _tool("check_profile")
    m, ms = 2, 1_000_000
    trace, t = [], 0
    for _step in range(m):   # one factorisation of m steps (warm-up 0, steps 1)
        trace.append((DOT2, t, t + 7 * ms)); t += 7 * ms
        trace.append((RED, t, t + 10_000)); t += 20_000
        trace.append((COEF, t, t + 10_000)); t += 20_000
        for _band in range(4):   # 4 band dispatches of 2 ms with 1 us gaps: one 8.003 ms call
            trace.append((UPD, t, t + 2 * ms)); t += 2 * ms + 1_000
    trace.append((ROTF, t, t + 5 * ms)); t += 5 * ms + 1_000
    trace.append((ROTF, t, t + 5 * ms)); t += 5 * ms + 1_000   # kept rotation: one call of 2 dispatches
    trace.append((DOT2, t, t + 1_000)); t += 2_000               # something in between
    trace.append((ROTS, t, t + 60 * ms)); t += 60 * ms + 1_000
    trace.append((ROTS, t, t + 60 * ms))                          # full rotation: two calls
    _write_trace(tmp_path / "run_kernel_trace.csv", trace)
    stats = [{"Name": DOT2, "Calls": str(m + 1), "TotalDurationNs": str(14 * ms + 1_000)},
             {"Name": UPD, "Calls": str(4 * m), "TotalDurationNs": str(16 * ms)},
             {"Name": ROTF, "Calls": "2", "TotalDurationNs": str(10 * ms)},
             {"Name": ROTS, "Calls": "2", "TotalDurationNs": str(120 * ms)}]
    with open(tmp_path / "run_kernel_stats.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Name", "Calls", "TotalDurationNs"])
        w.writeheader()
        w.writerows(stats)
    bench = {"config": {"m": m}, "warmup": 0, "steps": 1,
             "phases": {"block_dot2": {"launches": m, "avg_ms": 7.0},
                        "dcgs2_update": {"launches": m, "avg_ms": 8.003}},
             "restart": {"mstart": 7, "rotate_kept_ms": 10.001, "rotate_full_ms": 60.0}}
    bj = tmp_path / "bench.json"
    bj.write_text(json.dumps(bench))
    old = sys.argv
    sys.argv = ["check_profile.py", str(tmp_path / "run_kernel_stats.csv"), str(bj)]
    buf = io.StringIO()
    try:
        with redirect_stdout(buf):
            cp.main()
    finally:
        sys.argv = old
    txt = buf.getvalue()
    upd = [line for line in txt.splitlines() if "disp/call" in line and "timed" in line]
    assert upd and "4 disp/call" in upd[0] and upd[0].split()[-1] == "1.000", txt
    kept = [line for line in txt.splitlines() if line.startswith("rotate kept")][0]
    assert kept.split()[2] == "1" and "(2 disp/call)" in kept and abs(float(kept.split()[-3]) - 1.0) < 1e-3, kept
    full = [line for line in txt.splitlines() if line.startswith("rotate full")][0]
    assert full.split()[2] == "2" and abs(float(full.split()[-3]) - 1.0) < 1e-3, full
    # with the steady figure: the kept shape ran three times (the solver's call + two steady ones)
    stats[2] = {"Name": ROTF, "Calls": "6", "TotalDurationNs": str(30 * ms)}
    with open(tmp_path / "run_kernel_stats.csv", "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Name", "Calls", "TotalDurationNs"])
        w.writeheader()
        w.writerows(stats)
    bench["restart"].update(rotate_kept_ms=11.4, rotate_kept_steady_ms=10.001)
    bj.write_text(json.dumps(bench))
    sys.argv = ["check_profile.py", str(tmp_path / "run_kernel_stats.csv"), str(bj)]
    buf = io.StringIO()
    try:
        with redirect_stdout(buf):
            cp.main()
    finally:
        sys.argv = old
    kept = [line for line in buf.getvalue().splitlines() if line.startswith("rotate kept")][0]
    assert kept.split()[2] == "3" and "(2 disp/call)" in kept and abs(float(kept.split()[-3]) - 1.0) < 1e-3, kept
