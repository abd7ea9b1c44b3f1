#!/usr/bin/env python
"""One complete m=128 CPU factorisation of the reference algorithm at several sample sizes (VERDICT
r3 item 6): bench.cpu_baseline at E = 2,000 (the bench's default sample), 4,000 and 11,044 (N=2.5e7,
SURVEY.md §8(d)'s CPU sample) on all allowed threads, each after one warm-up step.  Shows that the
measured seconds scale linearly in N (so the bench's E=2,000 sample, scaled to N=1e8, stands for
the large sample) and the error of the round-3 single-step fit against each measured total.

At E=44,176 (BASELINE's own N=100,014,464: a 103 GB host basis) the factorisation is measured at
full size, nothing scaled.

``--variant cgs2`` times the optimised CPU line (oracle/cpu_cgs2.c, blocked OpenMP CGS2) instead;
``--threads T`` overrides the host's thread share.

usage (GPU box host): python tools/cpu_factorisation.py OUT.json [E ...] [--variant cgs2] [--threads T]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("E", nargs="*", type=int)
    ap.add_argument("--variant", default="mgs2", choices=("mgs2", "cgs2"))
    ap.add_argument("--threads", type=int, default=0)
    a = ap.parse_args()
    out = a.out
    Es = a.E or [2000, 4000, 11044]
    host = bench.host_threads()
    if a.threads > 0:
        host["threads"] = a.threads
    rows = []
    for E in Es:
        r = bench.cpu_baseline(E, 128, host["threads"], variant=a.variant, progress=True)
        r["E"] = E
        rows.append(r)
        print(json.dumps({k: r[k] for k in ("E", "seconds_per_factorisation_sample", "seconds_scaled_from_sample_N1e8",
                                            "value", "fit_check")}), flush=True)
    ref = rows[-1]
    for r in rows:
        r["N1e8_seconds_vs_largest_sample"] = round(r["seconds_scaled_from_sample_N1e8"] /
                                                    ref["seconds_scaled_from_sample_N1e8"] - 1.0, 4)
    with open(out, "w") as fh:
        json.dump({"host": host, "m": 128, "variant": a.variant, "runs": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
