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


def test_noise_seeded_restart_keeps_mgs(gpu, tmp_path):
    """The reference's default noise seed leaves Q(1) unnormalised, so the whole solve is modified
    Gram–Schmidt (by default "mgs2-lagged"); a run resumed from its checkpoint (uparam(2) > 0, the same
    seed_mode) must stay MGS too — a classical resume would change the factorisation — and
    reproduces the uninterrupted run."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=32)
    d, exact = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    cfg = KrylovSchurConfig(k_dim=16, schur_tgt=5, seed_mode="noise")
    ref = krylov_schur(ctx, op, seed, cfg)
    hook = ArnoldiCheckpoint(ctx, str(tmp_path), session="cyl", evop="d")
    krylov_schur(ctx, op, seed, KrylovSchurConfig(k_dim=16, schur_tgt=0, seed_mode="noise"), on_step=hook)
    mstart = 9
    Q, H = load_restart(ctx, str(tmp_path), "cyl", mstart, 16)
    res = krylov_schur(ctx, op, None, cfg, Q=Q, start=(mstart, H))
    assert res.schur_cnt == ref.schur_cnt >= 1 and res.mstart_history == ref.mstart_history
    conv = ref.residual < 1e-6
    np.testing.assert_allclose(res.vals[conv], ref.vals[conv], rtol=1e-11)
    classical = krylov_schur(ctx, op, None, KrylovSchurConfig(k_dim=16, schur_tgt=0),
                             Q=load_restart(ctx, str(tmp_path), "cyl", mstart, 16)[0], start=(mstart, H))
    mgs = krylov_schur(ctx, op, None, KrylovSchurConfig(k_dim=16, schur_tgt=0, seed_mode="noise"),
                       Q=load_restart(ctx, str(tmp_path), "cyl", mstart, 16)[0], start=(mstart, H))
    assert np.max(np.abs(classical.H - mgs.H)) > 1e-8 * np.max(np.abs(mgs.H))


def test_outpost_ks_files(gpu, tmp_path):
    """End of the in-tree solver: orthonormality.dat, Spectre_H/NS(_conv) files and the Re/Im
    eigenmode field files (eigensolvers.f90:335-349, 472-640)."""
    from nekstab_next_amd import fld
    from nekstab_next_amd.krylov_schur import outpost_ks

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=32)
    d, exact = syn.diag_spectrum(lay)
    seed = ctx.vector()
    seed.fill_hash(11)
    k = 16
    res = krylov_schur(ctx, DiagOperator(ctx, d), seed, KrylovSchurConfig(k_dim=k, schur_tgt=5))
    out = outpost_ks(ctx, res, str(tmp_path), evop="d", period=2.0, maxmodes=4)
    assert out["modes"] == list(range(min(4, res.converged)))
    lines = open(tmp_path / "orthonormality.dat").read().split("\n")
    norms = [float(l.split("=")[1]) for l in lines if l.startswith("Norm of")]
    orth = [float(l.split("=")[1]) for l in lines if l.startswith("Orthogonality")]
    assert len(norms) == k and len(orth) == k * (k - 1) // 2
    assert max(abs(n - 1.0) for n in norms) < 1e-12 and max(abs(o) for o in orth) < 1e-12
    sh = np.loadtxt(tmp_path / "Spectre_Hd.dat")
    sn = np.loadtxt(tmp_path / "Spectre_NSd.dat")
    assert sh.shape == (k, 3) and sn.shape == (k, 3)
    np.testing.assert_allclose(sh[:, 0], res.vals.real, rtol=1e-6)
    np.testing.assert_allclose(sn[:, 0], np.log(np.abs(res.vals)) / 2.0, rtol=1e-6, atol=1e-7)
    conv = np.atleast_2d(np.loadtxt(tmp_path / "Spectre_NSd_conv.dat"))
    assert conv.shape == (len(out["modes"]), 2)
    for num in range(1, len(out["modes"]) + 1):
        re = ctx.vector().from_packed(fld.vector_from_fld(lay, fld.read_fld(str(tmp_path / fld.fld_name("dRe", "nek", 0, num)))))
        im = ctx.vector().from_packed(fld.vector_from_fld(lay, fld.read_fld(str(tmp_path / fld.fld_name("dIm", "nek", 0, num)))))
        assert abs(ctx.dot(re, re, False) + ctx.dot(im, im, False) - 1.0) < 1e-10


def test_dcgs2_step_hook_sees_final_columns(gpu):
    """DCGS2 with a per-step hook (checkpointing): the hook for step k runs once column k of Q and
    H's columns 0..k-1 are final — every step mstart..k_dim of every Krylov–Schur cycle, in order —
    and what it sees equals the end of the factorisation bit for bit; the hook changes nothing
    (the whole solve equals the hook-free DCGS2 solve bit for bit)."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=32)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    seed = ctx.vector()
    seed.fill_hash(11)
    k = 16
    cfg = KrylovSchurConfig(k_dim=k, schur_tgt=5, mode="dcgs2")
    ref = krylov_schur(ctx, op, seed, cfg)
    Qref = ref.Q.storage.cpu().numpy().copy()
    seen = []

    def hook(mstep, Q, Hd):
        seen.append((mstep, Hd.download()[: mstep + 1, :mstep].copy(), Q.storage[mstep].cpu().numpy().copy()))

    cycles = []
    res = krylov_schur(ctx, op, seed, cfg, on_step=hook,
                       on_restart=lambda cnt, ms: cycles.append((len(seen), ms)))
    assert res.schur_cnt == ref.schur_cnt and res.mstart_history == ref.mstart_history
    np.testing.assert_array_equal(res.H, ref.H)
    np.testing.assert_array_equal(res.Q.storage.cpu().numpy(), Qref)
    # the step sequence: 1..k, then mstart..k after each restart
    starts = [1] + res.mstart_history
    want = [s for m in starts for s in range(m, k + 1)]
    assert [s for s, _, _ in seen] == want
    # within the last factorisation the hook's view is the final state (earlier cycles were rotated)
    last = len(seen) - (k - starts[-1] + 1)
    for mstep, Hs, q in seen[last:]:
        np.testing.assert_array_equal(Hs, res.H[: mstep + 1, :mstep])
        np.testing.assert_array_equal(q, Qref[mstep])
