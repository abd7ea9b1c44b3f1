"""ifres checkpoint + uparam(2) restart on the device path: a Krylov–Schur run resumed from the
KRY/HES files written at step mstart reproduces the uninterrupted run (restart count, mstart
sequence, Ritz values to 1e-12)."""
import os

import numpy as np
import pytest

from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.checkpoint import ArnoldiCheckpoint, load_restart
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.krylov_schur import krylov_schur
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.operators import DiagOperator
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu


def test_restart_from_checkpoint_matches_uninterrupted(gpu, tmp_path):
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=32)
    d, exact = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    cfg = KrylovSchurConfig(k_dim=16, schur_tgt=5)
    ref = krylov_schur(ctx, op, seed, cfg)

    # first run writes checkpoints; we only need its first factorisation's files up to step 9
    hook = ArnoldiCheckpoint(ctx, str(tmp_path), session="cyl", evop="d")
    cfg0 = KrylovSchurConfig(k_dim=16, schur_tgt=0)
    krylov_schur(ctx, op, seed, cfg0, on_step=hook)
    assert os.path.exists(tmp_path / "HEScyl0009") and os.path.exists(tmp_path / "KRYcyl0.f00010")
    assert os.path.exists(tmp_path / "Spectre_Hd0016.dat")
    mstart = 9
    Q, H = load_restart(ctx, str(tmp_path), "cyl", mstart, 16)
    res = krylov_schur(ctx, op, None, cfg, Q=Q, start=(mstart, H))
    assert res.schur_cnt == ref.schur_cnt and res.mstart_history == ref.mstart_history
    conv = ref.residual < 1e-6
    np.testing.assert_allclose(res.vals[conv], ref.vals[conv], rtol=1e-12)
    np.testing.assert_allclose(np.sort(res.vals[conv].real)[::-1], exact, atol=1e-9)
