#!/usr/bin/env python
"""Per-kernel counter table from the --pmc passes of tools/gpu_pmc_kernels.sh (one tuning-tool run
per pass, a few calls of each entry point).  Counters are averaged per DISPATCH of each kernel
instantiation (the ratios below do not depend on how a call is split into row-band dispatches),
and the usual derived figures are added:

* ``wait_inst_any/wave_cycle``, ``active_vmem/wave_cycle`` ...: SQ_* over SQ_WAVE_CYCLES;
* ``vmem_in_flight_per_wave``: SQ_INST_LEVEL_VMEM / SQ_WAVE_CYCLES (vector-memory instructions
  outstanding per resident wave, averaged over its life);
* ``L2_read_latency_cycles``: TCP_TCC_READ_REQ_LATENCY_sum / TCP_TCC_READ_REQ_sum;
* ``gui_cycles_per_xcd``: GRBM_GUI_ACTIVE / 8 (the counter is summed over the 8 XCDs), and every
  counter per such cycle (``/cycle``);
* ``mfma_f64_per_cycle_per_cu``: SQ_INSTS_VALU_MFMA_F64 / (gui_cycles_per_xcd x 256);
* ``hbm_read_bytes`` / ``hbm_write_bytes``: FETCH_SIZE x 2 x 1024 (the gfx950 correction for
  16 B/lane streaming reads, MI355X_MICROARCH.md §HBM; uncalibrated for 8 B/lane loads) and
  WRITE_SIZE x 1024, per dispatch.

usage: tools/pmc_kernel_table.py PASS_ROOT OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import sys

N_XCD, N_CU = 8, 256


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return name.split("(")[0]


def table(pass_root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [per dispatch]
    for f in sorted(glob.glob(os.path.join(pass_root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        val = collections.defaultdict(float)
        kname, dur = {}, {}
        for r in csv.DictReader(open(f)):
            d = int(r["Dispatch_Id"])
            kname[d] = short(r["Kernel_Name"])
            val[(d, r["Counter_Name"])] += float(r["Counter_Value"])
            if "End_Timestamp" in r and r["End_Timestamp"]:
                dur[d] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
        for (d, c), v in val.items():
            per[kname[d]][c].append(v)
        for d, t in dur.items():
            per[kname[d]]["duration_ns"].append(t)
    out = {}
    for k, cs in per.items():
        if not k.startswith("k_"):
            continue
        b = {c: sum(v) / len(v) for c, v in cs.items()}
        b["dispatches"] = max(len(v) for v in cs.values())
        cyc = b.get("GRBM_GUI_ACTIVE")
        if cyc:
            b["gui_cycles_per_xcd"] = cyc / N_XCD
            if b.get("duration_ns"):   # the clock the chip held (MI355X_MICROARCH.md 'DVFS give-back')
                b["effective_clock_ghz"] = cyc / N_XCD / b["duration_ns"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in b:   # per SIMD (1024 of them)
                b["mfma_busy_frac"] = b["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc / N_XCD * 4 * N_CU)
        wc = b.get("SQ_WAVE_CYCLES")
        if wc:
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                if n in b:
                    b[n + "/wave_cycle"] = b[n] / wc
            if "SQ_INST_LEVEL_VMEM" in b:
                b["vmem_in_flight_per_wave"] = b["SQ_INST_LEVEL_VMEM"] / wc
        if wc is None and "SQ_INST_LEVEL_VMEM" in b and "SQ_INSTS_VMEM_RD" in b:
            b["vmem_level_per_read_inst"] = b["SQ_INST_LEVEL_VMEM"] / b["SQ_INSTS_VMEM_RD"]
        nrq = b.get("TCP_TCC_READ_REQ_sum")
        if nrq and "TCP_TCC_READ_REQ_LATENCY_sum" in b:
            b["L2_read_latency_cycles"] = b["TCP_TCC_READ_REQ_LATENCY_sum"] / nrq
        if "FETCH_SIZE" in b:
            b["hbm_read_bytes"] = 2.0 * 1024.0 * b["FETCH_SIZE"]
        if "WRITE_SIZE" in b:
            b["hbm_write_bytes"] = 1024.0 * b["WRITE_SIZE"]
        out[k] = b
    # per-cycle figures need a GUI count from the same pass: every pass carries GRBM_GUI_ACTIVE, and
    # its per-dispatch average is the same kernel's, so one cycle count serves all passes
    for k, b in out.items():
        g = b.get("gui_cycles_per_xcd")
        if not g:
            continue
        for n in list(b):
            if n.startswith(("SQ_INSTS_", "SQ_VALU_MFMA_BUSY", "TCP_", "TA_", "SQ_VMEM_")) and "/" not in n:
                b[n + "/cycle"] = b[n] / g
        if "SQ_INSTS_VALU_MFMA_F64" in b:
            b["mfma_f64_per_cycle_per_cu"] = b["SQ_INSTS_VALU_MFMA_F64"] / (g * N_CU)
    return out


def main():
    out = table(sys.argv[1])
    json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)
    keys = ("dispatches", "duration_ns", "effective_clock_ghz", "mfma_busy_frac", "gui_cycles_per_xcd",
            "SQ_WAIT_INST_ANY/wave_cycle", "SQ_ACTIVE_INST_VMEM/wave_cycle",
            "vmem_in_flight_per_wave", "L2_read_latency_cycles", "mfma_f64_per_cycle_per_cu", "hbm_read_bytes",
            "hbm_write_bytes")
    for k, b in sorted(out.items()):
        print(k)
        for n in keys:
            if n in b:
                print(f"   {n:34s} {b[n]:.6g}")


if __name__ == "__main__":
    main()
