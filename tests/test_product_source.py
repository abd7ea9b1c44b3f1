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


# ---- tuning variants derive from the product source --------------------

def _tune():
    import importlib.util

    spec = importlib.util.spec_from_file_location("tune_kernels", os.path.join(ROOT, "tools", "tune_kernels.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_no_kernel_copy_in_tools():
    """tools/ holds no copy of the product kernel: experiments are diffs against it."""
    exp = os.path.join(ROOT, "tools", "experiments")
    for f in os.listdir(exp):
        assert f.endswith(".patch"), f
    tk = _tune()
    for name, v in tk.VARIANTS.items():
        assert "src" not in v, name


def test_every_experiment_patch_applies(tmp_path):
    tk = _tune()
    for name, v in tk.VARIANTS.items():
        if "patch" in v:
            out = tk.variant_source(name, out_dir=str(tmp_path))
            assert open(out).read() != open(SRC).read(), name


def test_unmodified_variant_is_the_product_kernel(tmp_path):
    """The tuning tool's unpatched variant compiles to the same device code object as the product
    build (same source bytes, same flags): an A/B "base" leg is the product's kernel.  clang names
    each HIP module by a CUID hashed from its file path; both compiles get the same explicit CUID, so
    every other byte of the code objects is compared."""
    import subprocess

    tk = _tune()
    src = tk.variant_source("base", out_dir=str(tmp_path))
    assert open(src, "rb").read() == open(SRC, "rb").read()
    objs = []
    for s, tag in ((SRC, "product"), (src, "variant")):
        o = str(tmp_path / f"{tag}.co")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        "-I" + os.path.join(ROOT, "include"), "-cuid=nekkrylov", "--offload-device-only", "-c", s, "-o", o],
                       check=True)
        objs.append(open(o, "rb").read())
    assert objs[0] == objs[1]
