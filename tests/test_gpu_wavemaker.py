"""GPU parity of ``wave_maker`` (core/sensitivity.f90:3-77) against the oracle's restatement.

The chain is the reference's: a direct and an adjoint Krylov–Schur run on config 5's operator
(D + rank-2 non-normal term and its W-adjoint) write their modes with ``outpost_ks``
(``dRe/dIm<session>0.f#####``, ``aRe/aIm…``); ``wave_maker`` reads the direct mode 1 and the adjoint
mode 2 (the file numbers of :43-58), bi-orthogonalises them (:63-66), forms
sqrt(sum dRe^2 + dIm^2) * sqrt(sum aRe^2 + aIm^2) (:69-71) and writes it as the temperature of
``wm_<session>0.f00001`` (:73-74).

Gates: the pointwise kernel is bit-identical to the oracle's restatement on the same inputs; the
whole chain (files read by the oracle's independent #std reader, its own bi-orthogonalisation)
agrees to 1e-12; the written file reads back through the oracle's reader bit for bit.  At
BASELINE config 5's full N=50,007,232 the size-independent properties are checked."""
import numpy as np
import pytest
import torch

import nekio
import oracle as orc
from helpers import olayout, oracle_rank2_matvec
from nekstab_next_amd import fld
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.config import KrylovSchurConfig
from nekstab_next_amd.krylov_schur import krylov_schur, outpost_ks
from nekstab_next_amd.layout import NekLayout, box3d_layout
from nekstab_next_amd.operators import DiagOperator, RankTwoPerturbed
from nekstab_next_amd.sensitivity import velocity_layout, wave_maker, wavemaker_field
from nekstab_next_amd.vector import NekContext

pytestmark = pytest.mark.gpu


def _vel_olayout(lay):
    return orc.OLayout(lay.n_v, 0, lay.ldim, False, lay.ldim)


def _ref_velocity(lay, x_padded):
    """Reference-order velocity-only vector (vx, vy, [vz], time) of a padded device vector."""
    parts = [x_padded[k * lay.sv: k * lay.sv + lay.n_v] for k in range(lay.ldim)]
    return np.concatenate(parts + [np.zeros(1)])


@pytest.mark.parametrize("ldim,lx1,E", [(2, 6, 37), (3, 8, 11), (3, 5, 1)])
def test_wavemaker_kernel_bit_exact(gpu, ldim, lx1, E):
    """nkv_wavemaker == oracle.wavemaker_pointwise bit for bit on hashed inputs (ragged sizes,
    one element); padding rows give 0."""
    lay = velocity_layout(NekLayout(ldim=ldim, lx1=lx1, lx2=lx1 - 2, nelgv=E))
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=4)
    vs = []
    for s in (31, 32, 33, 34):
        v = ctx.vector()
        v.fill_hash(s)
        vs.append(v)
    out = wavemaker_field(ctx, *vs)
    got = out.cpu().numpy()
    L = _vel_olayout(lay)
    ref = orc.wavemaker_pointwise(L, *(_ref_velocity(lay, v.to_packed()) for v in vs))
    assert np.array_equal(got[: lay.n_v], ref)
    assert not np.any(got[lay.n_v:])
    # argument checks: ncomp outside 2..n_wf, NULL operand
    from nekstab_next_amd import _lib as L_
    rc = ctx.lib.nkv_wavemaker(ctx._Lp, vs[0].ptr, vs[1].ptr, vs[2].ptr, vs[3].ptr, out.data_ptr(), 4, ctx.stream)
    assert rc == L_.NKV_EINVAL
    rc = ctx.lib.nkv_wavemaker(ctx._Lp, vs[0].ptr, None, vs[2].ptr, vs[3].ptr, out.data_ptr(), ldim, ctx.stream)
    assert rc == L_.NKV_EINVAL and "dIm is NULL" in L_.last_error()


def _config5_modes(lay, tmp, m, session, maxmodes_d, maxmodes_a, vecs_host=None):
    """Direct and adjoint Krylov–Schur on config 5's operator; outpost_ks writes the mode files."""
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=m + 1)
    d, _ = syn.diag_spectrum(lay)
    vs = []
    for s5 in (21, 22, 23, 24):
        v = ctx.vector()
        v.fill_hash(s5)
        v.scal(1e-3)
        vs.append(v)
    A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=50.0)
    del d
    seed = ctx.vector()
    seed.fill_hash(11)
    cfg = KrylovSchurConfig(k_dim=m, schur_tgt=2)
    rd = krylov_schur(ctx, A, seed, cfg)
    od = outpost_ks(ctx, rd, str(tmp), evop="d", maxmodes=maxmodes_d, session=session, orthonormality=False)
    del rd
    ra = krylov_schur(ctx, A, seed, cfg, transpose=True)
    oa = outpost_ks(ctx, ra, str(tmp), evop="a", maxmodes=maxmodes_a, session=session, orthonormality=False)
    assert len(od["modes"]) >= 1 and len(oa["modes"]) >= maxmodes_a
    return ctx


def _pair_modes(lay, tmp, m, session):
    """A leading complex pair: config 2's rotation-scaling operator (r e^{±i theta}) plus config
    5's rank-2 non-normal term, direct and adjoint Krylov–Schur, outpost_ks of the first 2 modes."""
    from nekstab_next_amd.operators import Rot2Operator

    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=m + 1)
    c, s, dr, _ = syn.rot2_operator(lay)
    vs = []
    for s5 in (21, 22, 23, 24):
        v = ctx.vector()
        v.fill_hash(s5)
        v.scal(1e-2)
        vs.append(v)
    A = RankTwoPerturbed(Rot2Operator(ctx, c, s, dr), *vs, sigma=1.0)
    seed = ctx.vector()
    seed.fill_hash(5)
    cfg = KrylovSchurConfig(k_dim=m, schur_tgt=2)
    rd = krylov_schur(ctx, A, seed, cfg)
    ra = krylov_schur(ctx, A, seed, cfg, transpose=True)
    for r in (rd, ra):   # the leading pair is complex: mode 1 = lambda (Im > 0), mode 2 = its conjugate
        assert r.converged >= 2 and r.vals[0].imag > 0 and abs(r.vals[1] - np.conj(r.vals[0])) < 1e-10
    outpost_ks(ctx, rd, str(tmp), evop="d", maxmodes=2, session=session, orthonormality=False)
    outpost_ks(ctx, ra, str(tmp), evop="a", maxmodes=2, session=session, orthonormality=False)
    return rd.vals[0]


@pytest.mark.parametrize("case,a_num", [("cfg5", 1), ("cfg5", 2), ("pair", 2)])
def test_wave_maker_vs_oracle(gpu, tmp_path, case, a_num):
    """The product's wave_maker against the oracle's, both from the same mode files (the oracle
    reads them with its own #std reader).  ``cfg5``: config 5's operator (reduced, E=60, 3-D), a
    real leading eigenvalue, so the matched adjoint mode is mode 1; mode 2 belongs to another
    eigenvalue, <a, d>_W is tiny and the rescaling amplifies rounding by 1/|<a, d>| (the gate
    scales with it).  ``pair``: a leading complex pair (2-D cylinder layout); the reference's file
    numbers (direct 1, adjoint 2) pick lambda and the adjoint mode of conj(lambda) — the left
    eigenvector of lambda — so <a, d>_W is O(1)."""
    from nekstab_next_amd.layout import cylinder_layout

    if case == "cfg5":
        lay = box3d_layout(60)
        _config5_modes(lay, tmp_path, 30, "cfg5", 2, 2)
    else:
        lay = cylinder_layout(120)
        _pair_modes(lay, tmp_path, 40, "cfg5")
    vlay = velocity_layout(lay)
    w = syn.mass_weights(vlay)
    vctx = NekContext(vlay, weights=w, max_cols=4)
    res = wave_maker(vctx, str(tmp_path), session="cfg5", d_num=1, a_num=a_num)

    # oracle: independent reader, its own bi-orthogonalisation and pointwise product
    g = nekio.Geom(lay.ldim, lay.lx1, lay.lx2, lay.nelgv)
    L = _vel_olayout(vlay)
    nvel = lay.ldim * lay.n_v

    def load(prefix, num):
        v = nekio.read_std_vector([str(tmp_path / fld.fld_name(prefix, "cfg5", 0, num))], g)
        return np.concatenate([v[:nvel], np.zeros(1)])

    ins = [load("dRe", 1), load("dIm", 1), load("aRe", a_num), load("aIm", a_num)]
    wm_ref, vecs_ref = orc.wave_maker(L, w, *ins)
    scale = np.max(np.abs(wm_ref))
    ip = abs(res["inner_product"])     # |<a, d/||d||>_W| before the rescaling
    if case == "pair" or a_num == 1:
        assert ip > 1e-3               # a matched direct/adjoint pair
    tol = 1e-12 / min(1.0, ip)
    assert scale > 0
    assert np.max(np.abs(res["wavemaker"] - wm_ref)) <= tol * scale
    for x, y in zip(res["vectors"], vecs_ref):
        xr = _ref_velocity(vlay, x.to_packed())
        assert np.max(np.abs(xr - y)) <= tol * max(np.max(np.abs(y)), 1e-300)
    # the pointwise product alone: bit-identical to the oracle's on the product's own vectors
    prod_vecs = [_ref_velocity(vlay, x.to_packed()) for x in res["vectors"]]
    assert np.array_equal(res["wavemaker"], orc.wavemaker_pointwise(L, *prod_vecs))
    # bi-orthogonality of the pair the wave-maker was formed from
    dRe, dIm, aRe, aIm = res["vectors"]
    re = vctx.dot(aRe, dRe, False) + vctx.dot(aIm, dIm, False)
    im = vctx.dot(aRe, dIm, False) - vctx.dot(aIm, dRe, False)
    assert abs(re - 1.0) < tol and abs(im) < tol
    # the file: the oracle's reader sees one T group holding the wave-maker, bit for bit, the time of
    # the last file loaded (aIm, outpost_ks's time = output number) and every element once
    tok, ids, fields = nekio.read_std(res["path"])
    assert res["path"].endswith("wm_cfg50.f00001")
    assert tok[11] == "T" and float(tok[7]) == float(a_num)
    assert np.array_equal(ids, np.arange(1, lay.nelgv + 1)) and set(fields) == {"t"}
    assert np.array_equal(fields["t"].ravel(), res["wavemaker"])
    # and the product's own reader agrees
    f = fld.read_fld(res["path"])
    assert np.array_equal(np.asarray(f.fields["t"]).ravel(), res["wavemaker"])


def test_wave_maker_rejects_full_layout(gpu, tmp_path):
    lay = box3d_layout(2)
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=4)
    with pytest.raises(ValueError, match="velocity-only"):
        wave_maker(ctx, str(tmp_path))


def test_wave_maker_config5_full_size(gpu, tmp_path):
    """BASELINE config 5's full N=50,007,232 (E=22,088, k_dim=96, both bases resident during the
    runs): the whole chain through the mode files; size-independent checks — <a, d>_W = 1 + 0i to
    1e-12, the wave-maker equals the oracle's pointwise restatement of the product's own
    bi-orthogonalised vectors bit for bit, and the file reads back through the oracle's reader."""
    lay = box3d_layout(22088)
    ctx = _config5_modes(lay, tmp_path, 96, "big", 1, 1)
    del ctx
    torch.cuda.empty_cache()
    vlay = velocity_layout(lay)
    vctx = NekContext(vlay, weights=syn.mass_weights(vlay), max_cols=4)
    res = wave_maker(vctx, str(tmp_path), session="big", d_num=1, a_num=1)
    dRe, dIm, aRe, aIm = res["vectors"]
    re = vctx.dot(aRe, dRe, False) + vctx.dot(aIm, dIm, False)
    im = vctx.dot(aRe, dIm, False) - vctx.dot(aIm, dRe, False)
    assert abs(re - 1.0) < 1e-12 and abs(im) < 1e-12
    L = _vel_olayout(vlay)
    prod_vecs = [_ref_velocity(vlay, x.to_packed()) for x in res["vectors"]]
    assert np.array_equal(res["wavemaker"], orc.wavemaker_pointwise(L, *prod_vecs))
    assert res["wavemaker"].size == 22088 * 512 and np.all(res["wavemaker"] >= 0)
    f = fld.read_fld(res["path"])
    assert f.rdcode == "T" and np.array_equal(np.asarray(f.fields["t"]).ravel(), res["wavemaker"])
    tok, ids, fields = nekio.read_std(res["path"])
    assert tok[11] == "T" and ids.size == 22088 and np.array_equal(fields["t"].ravel(), res["wavemaker"])


@pytest.mark.parametrize("part", ["r", "i"])
def test_steady_force_sensitivity_vs_oracle(gpu, tmp_path, part):
    """ts_steady_force_sensitivity (sensitivity.f90:273-346): the forcing's velocity read from
    ``s<part>_<session>0.f00001`` (written by the oracle's own #std writer, pressure and scalars
    present and ignored), GMRES on the mode-4 map q - A^T q of a non-normal operator, sol * alpha
    written as ``fs<part><session>0.f00001``.  GMRES histories 1e-8 and the solution 1e-10 against the
    oracle's restatement; the written file read back by the oracle's reader."""
    from nekstab_next_amd.sensitivity import ts_steady_force_sensitivity

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=120, n_scalars=1)
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=24)
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    d = 0.5 * d
    vs = []
    for s5 in (21, 22, 23, 24):
        v = ctx.vector()
        v.fill_hash(s5)
        v.scal(0.05)
        vs.append(v)
    A = RankTwoPerturbed(DiagOperator(ctx, d), *vs, sigma=2.0)
    adj = oracle_rank2_matvec(lay, d, *(0.05 * syn.hash_vector(lay, s5) for s5 in (21, 22, 23, 24)), 2.0, w,
                              transpose=True)
    g = nekio.Geom(lay.ldim, lay.lx1, lay.lx2, lay.nelgv, 0, lay.nelgv, lay.n_scalars)
    forcing = syn.to_reference_order(lay, syn.hash_vector(lay, 5))
    nekio.write_std(str(tmp_path / f"s{part}_cyl0.f00001"), g, forcing)
    r = ts_steady_force_sensitivity(ctx, A, str(tmp_path), session="cyl", part=part, k_dim=20, tol=1e-14)
    rhs = nekio.read_std_vector([str(tmp_path / f"s{part}_cyl0.f00001")], g)
    nvel = lay.ldim * lay.n_v
    rhs[nvel:] = 0.0                                  # opcopy: velocity only
    sref, hist, alpha = orc.ts_steady_force_sensitivity(L, w, adj, rhs, 20, 1e-14, part=part)
    assert abs(r["alpha"] - alpha) <= 1e-12 * alpha
    assert len(r["info"].outer_residuals) == len(hist["outer"]) >= 1
    assert len(r["info"].inner_residuals) == len(hist["inner"])
    np.testing.assert_allclose(r["info"].inner_residuals, hist["inner"], rtol=1e-8)
    np.testing.assert_allclose(r["info"].outer_residuals, hist["outer"], rtol=1e-8)
    got = syn.to_reference_order(lay, r["solution"].to_packed())
    n = L.n
    assert np.max(np.abs(got[:n] - sref[:n])) <= 1e-10 * np.max(np.abs(sref[:n]))
    back = nekio.read_std_vector([r["path"]], g)
    assert np.max(np.abs(back[:nvel] - got[:nvel])) == 0.0   # 64-bit file, velocity bit for bit
    assert r["path"].endswith(f"fs{part}cyl0.f00001")
