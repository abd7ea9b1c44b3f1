"""nekstab_next_amd — MI355X-native Krylov hot path for nekStab (Arnoldi / Krylov–Schur / GMRES).

Host mirror of nekStab's vector/operator/solver interfaces driving hand-written gfx950 HIP kernels
through the C ABI in include/nekkrylov.h (libnekkrylov.so, built in-tree).  See DESIGN.md.
"""
from .layout import NekLayout, box3d_layout, cylinder_layout  # noqa: F401
from .config import GmresConfig, KrylovSchurConfig  # noqa: F401

__version__ = "0.1.0"


def __getattr__(name):
    # GPU-facing modules are imported lazily so that `import nekstab_next_amd` works on a
    # build host without a GPU; they raise loudly on first use if the HIP library or the GPU is absent.
    import importlib

    for mod in ("vector", "operators", "arnoldi", "krylov_schur", "gmres", "newton", "sensitivity", "lapack",
                "comm", "synthetic", "lightkrylov", "drivers", "checkpoint", "fld", "boostconv", "seeds", "_lib"):
        if name == mod:
            return importlib.import_module(f".{mod}", __name__)
    raise AttributeError(name)
