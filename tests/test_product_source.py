"""The product kernel carries no timing-experiment code paths: the
round-1 switches that produced wrong results or could deadlock are gone from
nekstab_next_amd/csrc/nekkrylov.hip, and build() passes no -D that could change the product."""
import os
import re

import __graft_entry__ as ge

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "nekstab_next_amd", "csrc", "nekkrylov.hip")

REMOVED = ["NKV_DC_EXPERIMENT", "NKV_DC_SYNC", "NKV_QTILE_EXP", "NKV_D2_FIELDMAJOR", "NKV_DC_SCHED",
           "NKV_D2_SCHED", "NKV_ST_AUX", "NKV_XCD_MAP", "NKV_DC_FIELDLOOP", "NKV_FUSE_PF", "NKV_LD_ALIGN"]


def test_no_experiment_switches_in_product_kernel():
    src = open(SRC).read()
    # the only mention allowed is the #error guard that rejects a stray -D
    guard = src[src.index("#if defined(NKV_DC_EXPERIMENT)"):src.index("#error")]
    body = src.replace(guard, "")
    for m in REMOVED:
        assert re.search(r"\b%s\b" % m, body) is None, m
        assert m in guard, m
    # no spin barriers / sleeps / grid-wide atomics in the product kernel
    for pat in ("s_sleep", "s_memrealtime", "__hip_atomic"):
        assert pat not in src, pat


def test_build_passes_no_defines():
    assert not any(f.startswith("-D") for f in ge.HIP_FLAGS)
