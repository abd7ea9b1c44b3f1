#!/usr/bin/env python
"""Per-kernel-family summary of rocprofv3 --pmc passes over bench.py (is there
headroom in k_dcgs2_update's write path?).  For each pass directory, every counter is averaged per
launch of a family and, where GRBM_GUI_ACTIVE is in the same pass, normalised per GPU cycle.

usage: tools/pmc_write_path.py OUT_JSON PASS_DIR [PASS_DIR ...]
"""
import collections
import csv
import glob
import json
import os
import sys

FAMILIES = {"block_dot2": "k_block_dot2<", "dcgs2_update": "k_dcgs2_update<", "op_diag": "k_op_diag"}


def main():
    out = collections.defaultdict(dict)
    for d in sys.argv[2:]:
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            fam = next((k for k, key in FAMILIES.items() if key in r["Kernel_Name"]), None)
            if fam:
                acc[fam][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for fam, byd in acc.items():
            per = collections.defaultdict(list)
            for (_disp, name), vals in byd.items():
                per[name].append(sum(vals))            # sum over dimensions of one dispatch
            rec = {name: sum(v) / len(v) for name, v in per.items()}
            rec_launches = max(len(v) for v in per.values())
            cyc = rec.get("GRBM_GUI_ACTIVE")
            if cyc:
                for name in list(rec):
                    if name != "GRBM_GUI_ACTIVE":
                        rec[name + "/cycle"] = rec[name] / cyc
            out[fam].update(rec)
            out[fam]["launches"] = rec_launches
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
