#!/usr/bin/env python
"""Per-Arnoldi-step view of rocprofv3 --pmc passes over ONE bench.py factorisation
(``--steps 1 --warmup 0``): the multi-dot and the dual update run once per step j, in order, so the
n-th call of a family is step j = n + 1 (a call of the dual update = its consecutive row-band
dispatches).  Counters are summed over a call's dispatches and averaged over j bins; where
GRBM_GUI_ACTIVE is in the pass they are also given per GPU cycle.  Used to ask whether the
multi-dot's slide from ~7.0 TB/s at j <= 64 to ~6.8 at j = 128 comes with address-translation
misses (UTCL1) growing with the number of basis columns touched.

usage: tools/pmc_by_j.py OUT_JSON PASS_DIR [PASS_DIR ...]
"""
import collections
import csv
import glob
import json
import os
import sys

FAMILIES = {"block_dot2": "k_block_dot2<", "dcgs2_update": "k_dcgs2_update<", "update_dot": "k_update_dot<",
            "block_update": "k_block_update<"}
BINS = ((1, 8), (9, 32), (33, 64), (65, 96), (97, 128), (8, 8), (32, 32), (64, 64), (128, 128))
MULTI_DISPATCH = ("dcgs2_update", "block_update")   # one call = consecutive row-band dispatches


def main():
    out = {}
    for d in sys.argv[2:]:
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
        rows = list(csv.DictReader(open(f)))
        kname = {int(r["Dispatch_Id"]): r["Kernel_Name"] for r in rows}
        order = sorted(kname)
        val = collections.defaultdict(float)
        for r in rows:
            val[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        names = sorted({r["Counter_Name"] for r in rows})
        for fam, key in FAMILIES.items():
            calls, cur, prev_in = [], [], False
            for did in order:
                inside = key in kname[did]
                if inside and not (fam in MULTI_DISPATCH and prev_in):
                    if cur:
                        calls.append(cur)
                    cur = [did]
                elif inside:
                    cur.append(did)
                prev_in = inside
            if cur:
                calls.append(cur)
            if len(calls) < 64:   # this run is another mode (e.g. DCGS2's one closing block_update)
                continue
            # one factorisation = the LAST m calls of the family (the seed's dots come first)
            calls = calls[-128:]
            rec = out.setdefault(fam, {"calls": len(calls), "dispatches_per_call": [len(calls[0]), len(calls[-1])]})
            for lo, hi in BINS:
                sel = calls[lo - 1:hi]
                if not sel:
                    continue
                b = rec.setdefault(f"j{lo}-{hi}" if lo != hi else f"j{lo}", {})
                for n in names:
                    b[n] = sum(sum(val[(did, n)] for did in c) for c in sel) / len(sel)
                cyc = b.get("GRBM_GUI_ACTIVE")
                if cyc:
                    for n in names:
                        if n != "GRBM_GUI_ACTIVE":
                            b[n + "/cycle"] = b[n] / cyc
                wc = b.get("SQ_WAVE_CYCLES")
                if wc:
                    for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                              "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM"):
                        if n in b:
                            b[n + "/wave_cycle"] = b[n] / wc
                nrq = b.get("TCP_TCC_READ_REQ_sum")
                if nrq and "TCP_TCC_READ_REQ_LATENCY_sum" in b:
                    b["L2_read_latency_cycles"] = b["TCP_TCC_READ_REQ_LATENCY_sum"] / nrq
                nv = b.get("SQ_INSTS_VMEM_RD")
                if nv and "SQ_INST_LEVEL_VMEM" in b and "SQ_WAVE_CYCLES" in b:
                    b["vmem_in_flight_per_wave"] = b["SQ_INST_LEVEL_VMEM"] / b["SQ_WAVE_CYCLES"]
                la = b.get("SQ_LDS_IDX_ACTIVE")
                if la and "SQ_LDS_BANK_CONFLICT" in b:
                    b["SQ_LDS_BANK_CONFLICT/lds_active"] = b["SQ_LDS_BANK_CONFLICT"] / la
                req = b.get("TCP_UTCL1_REQUEST_sum")
                if req:
                    for n in ("TCP_UTCL1_TRANSLATION_MISS_sum", "TCP_UTCL1_TRANSLATION_HIT_sum"):
                        if n in b:
                            b[n + "/request"] = b[n] / req
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
