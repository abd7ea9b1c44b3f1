"""Checkpoint / restart across implementations on the device path (§8 rows a20 and f2;
VERDICT r1 item 3).  The reference writes KRY<session>0.f<k+1> + HES<session><k> after every
Arnoldi step (arnoldi_checkpoint, core/eigensolvers.f90:758-857) and resumes with uparam(2)=mstart
(:240-285, core/IO.f90:12-73).  Here:

* the product resumes from files the ORACLE wrote (oracle/nekio.py: an independent #std writer and
  gfortran-style list-directed HES text), and
* the oracle resumes from files the PRODUCT wrote (checkpoint.ArnoldiCheckpoint),

and both must follow the oracle's uninterrupted trajectory: identical restart count, mstart and
converged-count sequences; Ritz values in the comparison set within 1e-10 relative.  The run is cut
inside the first factorisation: after a Schur condensation the reference does not rewrite
KRY 1..mstart (only Q(k+1) is written per step), so its files only describe the first one."""
import os

import numpy as np
import pytest

import nekio
import oracle as orc
from helpers import match_ritz, olayout, oracle_diag_matvec, oracle_rot2_matvec, ritz_compare_set
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.checkpoint import ArnoldiCheckpoint, load_restart
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.krylov_schur import krylov_schur
from nekstab_next_amd.layout import NekLayout, cylinder_layout
from nekstab_next_amd.operators import DiagOperator, Rot2Operator
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu


class _Killed(Exception):
    pass


def _geom(lay):
    e0, e1 = lay.elem_range()
    return nekio.Geom(lay.ldim, lay.lx1, lay.lx2, lay.nelgv, e0, e1 - e0, lay.n_scalars)


def _problem(kind):
    if kind == "config1":
        lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=1136)
        w = syn.mass_weights(lay)
        d, _ = syn.diag_spectrum(lay)
        L = olayout(lay)
        return dict(lay=lay, w=w, k=16, tgt=5, cut=9, seed=11,
                    prod_op=lambda ctx: DiagOperator(ctx, d),
                    orc_mv=oracle_diag_matvec(L, syn.to_reference_order(lay, d)))
    lay = cylinder_layout(1996)
    w = syn.mass_weights(lay)
    c, s, dr, _ = syn.rot2_operator(lay)
    return dict(lay=lay, w=w, k=24, tgt=4, cut=17, seed=5,
                prod_op=lambda ctx: Rot2Operator(ctx, c, s, dr),
                orc_mv=oracle_rot2_matvec(lay, c, s, dr))


def _check(res_sched, res_cnt, res_mhist, vals, ref, eigen_tol=1e-6):
    assert res_sched == ref["schur_cnt"]
    assert res_mhist == ref["mstart"]
    assert res_cnt == ref["cnt"]
    sel = ritz_compare_set(ref["vals"], ref["residual"], eigen_tol)
    got = match_ritz(ref["vals"][sel], vals)
    err = np.abs(got - ref["vals"][sel]) / np.abs(ref["vals"][sel])
    assert err.max() <= 1e-10, err.max()


@pytest.mark.parametrize("kind", ["config1", "config2"])
def test_product_resumes_from_oracle_files(gpu, tmp_path, kind):
    P = _problem(kind)
    lay, w, k, tgt, cut = P["lay"], P["w"], P["k"], P["tgt"], P["cut"]
    L = olayout(lay)
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, P["seed"])))
    ref = orc.krylov_schur(L, w, P["orc_mv"], q1, k, tgt)
    if kind == "config1":
        assert ref["schur_cnt"] >= 1          # the resumed run goes through real restarts
    cutrun = orc.krylov_schur(L, w, P["orc_mv"], q1, k, tgt, stop_after=cut,
                              on_step=nekio.checkpoint_writer(str(tmp_path), "cyl", _geom(lay)))
    assert cutrun["stopped_at"] == cut
    ctx = NekContext(lay, weights=w, max_cols=k + 8)
    Q, H = load_restart(ctx, str(tmp_path), "cyl", cut, k)
    res = krylov_schur(ctx, P["prod_op"](ctx), None, KrylovSchurConfig(k_dim=k, schur_tgt=tgt), Q=Q, start=(cut, H))
    _check(res.schur_cnt, res.cnt_history, res.mstart_history, res.vals, ref)


@pytest.mark.parametrize("kind", ["config1", "config2"])
def test_oracle_resumes_from_product_files(gpu, tmp_path, kind):
    P = _problem(kind)
    lay, w, k, tgt, cut = P["lay"], P["w"], P["k"], P["tgt"], P["cut"]
    L = olayout(lay)
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, P["seed"])))
    ref = orc.krylov_schur(L, w, P["orc_mv"], q1, k, tgt)
    ctx = NekContext(lay, weights=w, max_cols=k + 8)
    seed = ctx.vector()
    seed.fill_hash(P["seed"])
    ck = ArnoldiCheckpoint(ctx, str(tmp_path), session="cyl", evop="d")

    def hook(mstep, Q, Hd):    # the product's ifres checkpoint, then the job is killed after `cut`
        ck(mstep, Q, Hd)
        if mstep == cut:
            raise _Killed

    with pytest.raises(_Killed):
        krylov_schur(ctx, P["prod_op"](ctx), seed, KrylovSchurConfig(k_dim=k, schur_tgt=tgt), on_step=hook)
    assert os.path.exists(tmp_path / f"HEScyl{cut:04d}") and os.path.exists(tmp_path / nekio.kry_name("cyl", cut + 1))
    H, Qs = nekio.load_restart(str(tmp_path), "cyl", _geom(lay), cut, k)
    res = orc.krylov_schur(L, w, P["orc_mv"], None, k, tgt, start=(cut, H, Qs))
    _check(res["schur_cnt"], res["cnt"], res["mstart"], res["vals"], ref)


def test_product_files_are_the_oracle_basis(gpu, tmp_path):
    """Step by step, the product's checkpoint files hold the oracle's Krylov vectors and H (read
    with the oracle's reader): KRY vectors to 1e-10 in the W-norm (the product's CGS2 vs the
    oracle's MGS2 differ by rounding), H to 1e-12 max|H|."""
    P = _problem("config1")
    lay, w, k = P["lay"], P["w"], 12
    L = olayout(lay)
    q1 = orc.prepare_seed(L, w, syn.to_reference_order(lay, syn.hash_vector(lay, 11)))
    ref = orc.krylov_schur(L, w, P["orc_mv"], q1, k, 0)
    ctx = NekContext(lay, weights=w, max_cols=k + 8)
    seed = ctx.vector()
    seed.fill_hash(11)
    krylov_schur(ctx, P["prod_op"](ctx), seed, KrylovSchurConfig(k_dim=k, schur_tgt=0),
                 on_step=ArnoldiCheckpoint(ctx, str(tmp_path), session="cyl", write_spectra=False))
    g = _geom(lay)
    for num in range(1, k + 2):
        v = nekio.read_std_vector([str(tmp_path / nekio.kry_name("cyl", num))], g)
        dv = v - ref["Q"][num - 1]
        dv[-1] = 0.0
        assert np.sqrt(orc.k_dot(L, w, dv, dv)) < 1e-10, num
    Hk = nekio.read_hes(str(tmp_path / nekio.hes_name("cyl", k)), k, k)
    assert np.abs(Hk - ref["H"]).max() <= 1e-12 * np.abs(ref["H"]).max()
