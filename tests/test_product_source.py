"""The product kernels carry no timing-experiment code paths:
the round-1 switches that produced wrong results or could deadlock are gone from
nekstab_next_amd/csrc/, the kernel generations kept only for A/B (the VALU and staged-MFMA restart
rotations, the lazy-basis DCGS2 update) were removed in round 5, and build() passes no -D that could
change the product."""
import glob
import os
import re
import subprocess

import __graft_entry__ as ge

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nekstab_next_amd", "csrc")
INTERNAL = os.path.join(CSRC, "nkv_internal.h")

REMOVED = ["NKV_DC_EXPERIMENT", "NKV_DC_SYNC", "NKV_QTILE_EXP", "NKV_D2_FIELDMAJOR", "NKV_DC_SCHED",
           "NKV_D2_SCHED", "NKV_ST_AUX", "NKV_XCD_MAP", "NKV_DC_FIELDLOOP", "NKV_FUSE_PF", "NKV_LD_ALIGN"]
RETIRED = ["k_rotate_mfma", "k_dcgs2_lazy_update", "NKV_ROT_VALU", "NKV_ROT_SMALLR", "NKV_ROT_CHUNKED", "NKV_DL_U",
           "dcgs2_coef_lazy", "dcgs2_update_lazy", "NKV_ROT_MAX_K",
           # round 6: the LDS-staged rotation and the wide kernel's timing diagnostics (experiment patches)
           "k_rotate_glds", "NKV_ROTG", "NKV_ROTW_DIAG", "NKV_ROTW_APRE"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + [INTERNAL])


def test_build_compiles_every_translation_unit():
    assert sorted(ge.HIP_SRCS) == sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    for src in ge.HIP_SRCS:
        assert '#include "nkv_internal.h"' in open(src).read(), src


def test_no_experiment_switches_in_product_kernels():
    internal = open(INTERNAL).read()
    # the only mention allowed is the #error guard that rejects a stray -D
    guard = internal[internal.index("#if defined(NKV_DC_EXPERIMENT)"):internal.index("#error")]
    for m in REMOVED:
        assert m in guard, m
    for path in _sources():
        body = open(path).read().replace(guard, "")
        for m in REMOVED + RETIRED:
            assert re.search(r"\b%s\b" % m, body) is None, (path, m)
        # no spin barriers / sleeps / grid-wide atomics in the product kernels
        for pat in ("s_sleep", "s_memrealtime", "__hip_atomic"):
            assert pat not in body, (path, pat)
    hdr = open(os.path.join(ROOT, "include", "nekkrylov.h")).read()
    assert "lazy" not in hdr.lower() and "NKV_ROT_MAX_K" not in hdr


def test_build_passes_no_defines():
    assert not any(f.startswith("-D") for f in ge.HIP_FLAGS)


# ---- tuning variants derive from the product sources -------------------

def _tune():
    import importlib.util

    spec = importlib.util.spec_from_file_location("tune_kernels", os.path.join(ROOT, "tools", "tune_kernels.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_no_kernel_copy_in_tools():
    """tools/ holds no copy of the product kernels: experiments are diffs against them, and every
    speed knob a variant sets still exists in the product sources."""
    exp = os.path.join(ROOT, "tools", "experiments")
    if os.path.isdir(exp):
        for f in os.listdir(exp):
            assert f.endswith(".patch"), f
    tk = _tune()
    text = "".join(open(p).read() for p in _sources())
    for name, v in tk.VARIANTS.items():
        assert "src" not in v, name
        # a knob lives in the product sources, or in the experiment patch that adds it
        t = text + (open(os.path.join(exp, v["patch"] + ".patch")).read() if "patch" in v else "")
        for knob in v:
            if knob != "patch":
                assert re.search(r"#ifndef %s\b" % knob, t), (name, knob)


def test_experiment_patches_apply(tmp_path):
    """Every patch variant of the tuning tool still applies to the current product sources (an A/B
    logged under profiles/ stays reproducible from this tree)."""
    tk = _tune()
    for name, v in tk.VARIANTS.items():
        if "patch" in v:
            srcs = tk.variant_sources(name, out_dir=str(tmp_path))
            assert all(os.path.exists(p) for p in srcs), name


def test_unmodified_variant_is_the_product_kernel(tmp_path):
    """The tuning tool's unpatched variant compiles to the same device code object as the product
    build (same source bytes, same flags): an A/B "base" leg is the product's kernel.  clang names
    each HIP module by a CUID hashed from its file path; both compiles get the same explicit CUID, so
    every other byte of the code objects is compared (the Gram–Schmidt translation unit)."""
    tk = _tune()
    srcs = tk.variant_sources("base", out_dir=str(tmp_path))
    for a, b in zip(ge.HIP_SRCS, srcs):
        assert open(a, "rb").read() == open(b, "rb").read()
    objs = []
    for s, tag in ((os.path.join(CSRC, "gram_schmidt.hip"), "product"),
                   (os.path.join(os.path.dirname(srcs[0]), "gram_schmidt.hip"), "variant")):
        o = str(tmp_path / f"{tag}.co")
        subprocess.run(["/opt/rocm/bin/hipcc", *[f for f in ge.HIP_FLAGS if f != "-fPIC"], "-cuid=nkv_gs",
                        "--offload-device-only", "-c", s, "-o", o], check=True)
        objs.append(open(o, "rb").read())
    assert objs[0] == objs[1]
