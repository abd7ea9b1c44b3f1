"""GPU parity of every C-ABI entry point against the CPU oracle / numpy on the same inputs.

Tolerances: data movement (zero/copy/fill/rotate of exact values) is bit-exact; BLAS-1 updates
agree to 1 ulp-level (the device contracts a*x+b*y into one FMA, the oracle does not); reductions
are regrouped (tree vs sequential), so dots agree to 1e-13 relative.
"""
import ctypes

import numpy as np
import pytest
import torch

import oracle as orc
from helpers import olayout
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd._lib import NKV_NORM2, NKV_TIME, NkvError, NkvNaNError
from nekstab_next_amd.arnoldi import HessenbergDev, arnoldi_factorization
from nekstab_next_amd.layout import NekLayout
from nekstab_next_amd.operators import DiagOperator, Rot2Operator
from nekstab_next_amd.vector import NekContext, k_matmul, k_normalize

pytestmark = pytest.mark.gpu

LAYOUTS = {
    "2d": NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300),
    "3d_scalar": NekLayout(ldim=3, lx1=5, lx2=3, nelgv=37, n_scalars=1),  # odd sizes, ragged pads
    "2d_nopr": NekLayout(ldim=2, lx1=6, lx2=4, nelgv=150, ifpo=False),   # no pressure segment (.not. ifpo)
    "3d_noscal": NekLayout(ldim=3, lx1=4, lx2=2, nelgv=61),              # three weighted fields
}


def make_ctx(lay, weights=None, **kw):
    w = syn.mass_weights(lay) if weights is None else weights
    return NekContext(lay, weights=w, **kw), w


def dev_vec(ctx, padded):
    return ctx.vector().from_packed(padded)


@pytest.mark.parametrize("name", list(LAYOUTS))
def test_fill_hash_bitexact(gpu, name):
    lay = LAYOUTS[name]
    ctx, _ = make_ctx(lay)
    v = ctx.vector()
    v.fill_hash(1234)
    np.testing.assert_array_equal(v.to_packed(), syn.hash_vector(lay, 1234))
    L = olayout(lay)
    np.testing.assert_array_equal(syn.to_reference_order(lay, v.to_packed()), orc.fill_hash(L, 1234))


@pytest.mark.parametrize("name", list(LAYOUTS))
def test_blas1_vs_oracle(gpu, name):
    lay = LAYOUTS[name]
    ctx, w = make_ctx(lay)
    L = olayout(lay)
    c = ctypes.byref(L.c)
    a = syn.hash_vector(lay, 1)
    b = syn.hash_vector(lay, 2)
    a[lay.time_offset], b[lay.time_offset] = 0.25, -1.5
    ra, rb = syn.to_reference_order(lay, a), syn.to_reference_order(lay, b)
    x, y = dev_vec(ctx, a), dev_vec(ctx, b)

    # real_axpby: time untouched
    x.axpby(0.7, y, -1.3)
    ref = ra.copy()
    orc.lib().orc_real_axpby(c, ref, 0.7, rb, -1.3)
    got = syn.to_reference_order(lay, x.to_packed())
    np.testing.assert_allclose(got, ref, rtol=0, atol=4e-16 * 3)
    assert got[-1] == 0.25
    ref = got.copy()  # continue from the device state: the remaining ops are exact elementwise
    # k_cmult / real_scal incl. time
    x.scal(-2.5)
    orc.lib().orc_k_cmult(c, ref, -2.5)
    np.testing.assert_array_equal(syn.to_reference_order(lay, x.to_packed()), ref)
    # copy / zero
    z = ctx.vector()
    z.copy_from(x)
    np.testing.assert_array_equal(z.to_packed(), x.to_packed())
    z.zero()
    assert not np.any(z.to_packed())
    # sub3 with time (k_sub3)
    from nekstab_next_amd.vector import k_sub3, k_add2, k_sub2
    k_sub3(z, x, y)
    r3 = L.zeros()
    orc.lib().orc_k_sub3(c, r3, ref, rb)
    np.testing.assert_array_equal(syn.to_reference_order(lay, z.to_packed()), r3)
    k_add2(z, y)
    orc.lib().orc_k_add2(c, r3, rb)
    np.testing.assert_array_equal(syn.to_reference_order(lay, z.to_packed()), r3)
    k_sub2(z, x)
    orc.lib().orc_k_sub2(c, r3, ref)
    np.testing.assert_array_equal(syn.to_reference_order(lay, z.to_packed()), r3)
    # padding rows stay zero
    p = z.to_packed()
    for _, s, n in lay.field_slices():
        pad_end = s + (lay.sv if _ != "pr" else lay.sp)
        assert not np.any(p[s + n:pad_end])


@pytest.mark.parametrize("name", list(LAYOUTS))
@pytest.mark.parametrize("time_in_dot", [False, True])
def test_dot_vs_oracle(gpu, name, time_in_dot):
    lay = LAYOUTS[name]
    w = syn.sponge(syn.mass_weights(lay))  # zero weights inside a sponge are allowed
    ctx, _ = make_ctx(lay, weights=w, time_in_dot=time_in_dot)
    L = olayout(lay, time_in_dot)
    a, b = syn.hash_vector(lay, 3), syn.hash_vector(lay, 4)
    a[lay.time_offset], b[lay.time_offset] = 0.5, 3.0
    x, y = dev_vec(ctx, a), dev_vec(ctx, b)
    from nekstab_next_amd.vector import k_dot
    got = k_dot(x, y)
    ref = orc.k_dot(L, w, syn.to_reference_order(lay, a), syn.to_reference_order(lay, b))
    assert abs(got - ref) <= 1e-13 * max(1.0, abs(ref))
    # real_dot always includes time
    got2 = x.dot(y)
    ref2 = orc.real_dot(L, w, syn.to_reference_order(lay, a), syn.to_reference_order(lay, b))
    assert abs(got2 - ref2) <= 1e-13 * max(1.0, abs(ref2))
    # k_normalize
    alpha = k_normalize(x)
    ra = syn.to_reference_order(lay, a)
    alpha_ref = orc.k_normalize(L, w, ra)
    assert abs(alpha - alpha_ref) <= 1e-13 * alpha_ref
    np.testing.assert_allclose(syn.to_reference_order(lay, x.to_packed()), ra, rtol=1e-13, atol=1e-15)


@pytest.mark.parametrize("j", [1, 3, 4, 5, 37, 128])
def test_block_dot_update_vs_numpy(gpu, j):
    lay = LAYOUTS["2d"]
    ctx, w = make_ctx(lay, max_cols=128)
    Q = ctx.basis(j + 1)
    for i in range(j):
        Q[i].fill_hash(100 + i)
    f = ctx.vector()
    f.fill_hash(99)
    Qh = Q.storage.cpu().numpy()[:j]
    fh = f.to_packed()
    wfull = np.zeros(lay.ld)
    for f_ in range(lay.n_wf):
        wfull[f_ * lay.sv: f_ * lay.sv + lay.n_v] = w
    h = ctx.h1[:j]
    ctx.call("nkv_block_dot", ctx.w.data_ptr(), Q.ptr, j, f.ptr, h.data_ptr(), ctx.ws.data_ptr(), 0, ctx.stream)
    href = Qh @ (wfull * fh)
    np.testing.assert_allclose(h.cpu().numpy(), href, rtol=1e-12, atol=1e-12 * np.abs(href).max())
    # f <- f - Q h, fused norm
    nrm = ctx.scal[5:6]
    ctx.call("nkv_block_update", ctx.w.data_ptr(), Q.ptr, j, h.data_ptr(), f.ptr, nrm.data_ptr(),
             ctx.ws.data_ptr(), NKV_NORM2 | NKV_TIME, ctx.stream)
    hh = h.cpu().numpy()
    fref = fh - hh @ Qh
    np.testing.assert_allclose(f.to_packed(), fref, rtol=1e-12, atol=1e-13)
    nref = np.sum(wfull * fref * fref)
    assert abs(nrm.item() - nref) <= 1e-12 * nref
    # overwrite (k_matmul): out = Q y incl. time
    out = ctx.vector()
    Q[0].time = 2.0
    k_matmul(out, Q, hh, j)
    Qh = Q.storage.cpu().numpy()[:j]
    np.testing.assert_allclose(out.to_packed(), hh @ Qh, rtol=1e-12, atol=1e-13)


def test_k_matmul_vs_oracle(gpu):
    lay = LAYOUTS["3d_scalar"]
    ctx, w = make_ctx(lay)
    L = olayout(lay)
    k = 9
    Q = ctx.basis(k)
    Qref = np.zeros((k, L.len))
    for i in range(k):
        v = syn.hash_vector(lay, 50 + i)
        v[lay.time_offset] = 0.1 * i
        Q[i].from_packed(v)
        Qref[i] = syn.to_reference_order(lay, v)
    y = np.linspace(-1, 1, k)
    out = ctx.vector()
    k_matmul(out, Q, y, k)
    ref = L.zeros()
    orc.lib().orc_k_matmul(ctypes.byref(L.c), ref, Qref, y, k)
    np.testing.assert_allclose(syn.to_reference_order(lay, out.to_packed()), ref, rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("k", [1, 7, 16, 64, 100, 129, 200, 256])
def test_rotate_vs_oracle(gpu, k):
    lay = LAYOUTS["2d"]
    ctx, _ = make_ctx(lay)
    L = olayout(lay)
    Q = ctx.basis(k + 1)
    Qref = np.zeros((k + 1, L.len))
    for i in range(k + 1):
        v = syn.hash_vector(lay, 7 + i)
        v[lay.time_offset] = 1.0 + i
        Q[i].from_packed(v)
        Qref[i] = syn.to_reference_order(lay, v)
    V = np.linalg.qr(np.random.default_rng(k).standard_normal((k, k)))[0]
    Vd = torch.as_tensor(V.ravel(order="F").copy()).to(ctx.device)
    ctx.call("nkv_rotate", Q.ptr, k, Vd.data_ptr(), k, ctx.stream)
    Qk = np.ascontiguousarray(Qref[:k])
    orc.set_threads(8 if k > 128 else 1)
    try:
        orc.lib().orc_rotate(ctypes.byref(L.c), Qk, k, np.ascontiguousarray(V.ravel(order="F")))
    finally:
        orc.set_threads(1)
    got = Q.storage.cpu().numpy()
    for i in range(k):
        np.testing.assert_allclose(syn.to_reference_order(lay, got[i]), Qk[i], rtol=1e-12, atol=1e-13)
        assert got[i][lay.time_offset] == 1.0 + i  # time not rotated
    np.testing.assert_array_equal(syn.to_reference_order(lay, got[k]), Qref[k])  # column k untouched


@pytest.mark.parametrize("k,n_out", [(7, 3), (100, 1), (128, 6), (128, 8), (9, 9), (4, 4), (131, 5), (576, 7),
                                     (128, 12), (130, 13), (64, 16), (1000, 11), (128, 20), (129, 17), (256, 255),
                                     (300, 150), (576, 33), (900, 6), (256, 100), (200, 128), (576, 256),
                                     # k_rotate_wide (17-64 kept, V in LDS): every column-block count, whole
                                     # and partial last batches (k % 16), one-batch k, k = n_out
                                     (128, 25), (100, 17), (130, 48), (64, 64), (129, 33), (37, 33), (17, 17),
                                     (200, 40), (18, 18), (250, 64),
                                     # k_rotate_stream two batches ahead (65-128 kept): MB 5..8, zero
                                     # and several steady trips, every tail branch
                                     (83, 70), (128, 65), (96, 96), (128, 128), (150, 100)])
def test_rotate_cols_vs_oracle(gpu, k, n_out):
    """Partial restart rotation: Q[:, :n_out] = Q[:, :k] V[:, :n_out]; columns n_out..k untouched."""
    lay = LAYOUTS["2d"]
    ctx, _ = make_ctx(lay)
    L = olayout(lay)
    Q = ctx.basis(k + 1)
    Qref = np.zeros((k + 1, L.len))
    for i in range(k + 1):
        v = syn.hash_vector(lay, 11 + i)
        Q[i].from_packed(v)
        Qref[i] = syn.to_reference_order(lay, v)
    V = np.linalg.qr(np.random.default_rng(k + n_out).standard_normal((k, k)))[0]
    Vd = torch.as_tensor(np.asfortranarray(V[:, :n_out]).ravel(order="F")).to(ctx.device)
    ctx.call("nkv_rotate_cols", Q.ptr, k, Vd.data_ptr(), k, n_out, ctx.stream)
    Qk = Qref[:k].copy()
    orc.set_threads(8 if k > 128 else 1)
    try:
        orc.lib().orc_rotate(ctypes.byref(L.c), Qk, k, np.ascontiguousarray(V.ravel(order="F")))
    finally:
        orc.set_threads(1)
    got = Q.storage.cpu().numpy()
    for i in range(n_out):
        np.testing.assert_allclose(syn.to_reference_order(lay, got[i]), Qk[i], rtol=1e-12, atol=1e-13)
    for i in range(n_out, k + 1):
        np.testing.assert_array_equal(syn.to_reference_order(lay, got[i]), Qref[i])


@pytest.mark.parametrize("n_out", [6, 12, 16, 17])
def test_rotate_cols_row_bands(gpu, n_out):
    """The few-column rotation issues one dispatch per row band (NKV_ROTF_ROUNDS): at N=2.26e6
    (E=1000, 3-D) a call spans several bands; every band's rows equal Q V to 1e-12 and the
    columns past n_out are untouched (n_out=17 runs the MFMA streaming kernel beside it)."""
    from nekstab_next_amd.layout import box3d_layout

    lay = box3d_layout(1000)
    ctx, _ = make_ctx(lay)
    k = 20
    Q = ctx.basis(k + 1)
    for i in range(k + 1):
        Q[i].fill_hash(300 + i)
    before = Q.storage.cpu().numpy().copy()
    V = np.linalg.qr(np.random.default_rng(n_out).standard_normal((k, k)))[0][:, :n_out]
    Vd = torch.as_tensor(np.asfortranarray(V).ravel(order="F")).to(ctx.device)
    ctx.call("nkv_rotate_cols", Q.ptr, k, Vd.data_ptr(), k, n_out, ctx.stream)
    got = Q.storage.cpu().numpy()
    rows = lay.rows   # streamed rows; the time slot and the padding after it are not rotated
    want = V.T @ before[:k, :rows]
    for i in range(n_out):
        np.testing.assert_allclose(got[i, :rows], want[i], rtol=1e-12, atol=1e-13)
    np.testing.assert_array_equal(got[:n_out, rows:], before[:n_out, rows:])
    np.testing.assert_array_equal(got[n_out:], before[n_out:])


@pytest.mark.parametrize("name", list(LAYOUTS) + ["large"])
def test_native_dcgs2_driver_bit_identical(gpu, name):
    """nkv_arnoldi_dcgs2 (the whole DCGS2 factorisation in one ABI call, operator as a callback)
    gives the Python-driven DCGS2 factorisation bit for bit — from the seed and from mstart > 1 —
    and nkv_arnoldi_factorization (per-column CGS2, or the reference's MGS2 order with NKV_MGS2) the
    Python-driven CGS2 / MGS2 ones; so does nkv_update_hessenberg called per column (with a step
    hook the native per-column modes run column by column)."""
    from nekstab_next_amd.layout import box3d_layout

    lay = box3d_layout(4000) if name == "large" else LAYOUTS[name]
    ctx, _ = make_ctx(lay, max_cols=32)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    m = 20
    out = {}
    modes = ("dcgs2", "dcgs2-native", "cgs2", "cgs2-native", "cgs2-native-hook", "mgs2", "mgs2-native",
             "mgs2-native-hook")
    for mode in modes:
        Q = ctx.basis(m + 1)
        Q[0].fill_hash(5)
        k_normalize(Q[0])
        Hd = HessenbergDev(ctx, m)
        hook = (lambda _s: None) if mode.endswith("-hook") else None
        md = mode.replace("-hook", "")
        arnoldi_factorization(ctx, op, Q, Hd, 1, 12, mode=md, on_step=hook)
        arnoldi_factorization(ctx, op, Q, Hd, 13, m, mode=md, on_step=hook)   # continue from column 12
        out[mode] = (Hd.download(), Q.storage.cpu().numpy())
    for a, b in (("dcgs2", "dcgs2-native"), ("cgs2", "cgs2-native"), ("cgs2", "cgs2-native-hook"),
                 ("mgs2", "mgs2-native"), ("mgs2", "mgs2-native-hook")):
        np.testing.assert_array_equal(out[a][0], out[b][0])
        np.testing.assert_array_equal(out[a][1], out[b][1])


def test_native_dcgs2_driver_callback_errors(gpu):
    """A failing operator callback stops nkv_arnoldi_dcgs2 with the callback's exception (Python)
    and NKV_ECALLBACK (C ABI) after the first call; a NULL matvec is refused (NKV_EINVAL)."""
    from nekstab_next_amd import _lib as L_

    lay = LAYOUTS["2d"]
    ctx, _ = make_ctx(lay, max_cols=8)
    Q = ctx.basis(5)
    Q[0].fill_hash(3)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, 4)

    class Boom(DiagOperator):
        def matvec(self, x, y):
            raise RuntimeError("operator failed")

    d, _ = syn.diag_spectrum(lay)
    with pytest.raises(RuntimeError, match="operator failed"):
        arnoldi_factorization(ctx, Boom(ctx, d), Q, Hd, 1, 4, mode="dcgs2-native")
    f = ctx.vector()
    scratch = torch.zeros(int(ctx.lib.nkv_arnoldi_scratch_doubles(4)), dtype=torch.float64, device=ctx.device)
    rc = ctx.lib.nkv_arnoldi_dcgs2(ctx._Lp, ctx.w.data_ptr(), Q.ptr, 1, 4, Hd.t.data_ptr(), 5, f.ptr,
                                   scratch.data_ptr(), ctx.ws.data_ptr(), L_.MATVEC_FN(), None, L_.ALLREDUCE_FN(),
                                   None, 0, ctx.stream)
    assert rc == L_.NKV_EINVAL and "matvec" in L_.last_error()
    # a callback that reports failure: NKV_ECALLBACK, no further steps
    calls = []

    def bad(_user, x, y, _stream):
        calls.append(x)
        return 7

    rc = ctx.lib.nkv_arnoldi_dcgs2(ctx._Lp, ctx.w.data_ptr(), Q.ptr, 1, 4, Hd.t.data_ptr(), 5, f.ptr,
                                   scratch.data_ptr(), ctx.ws.data_ptr(), L_.MATVEC_FN(bad), None, L_.ALLREDUCE_FN(),
                                   None, 0, ctx.stream)
    assert rc == L_.NKV_ECALLBACK and "returned 7" in L_.last_error() and len(calls) == 1
    # argument checks (no launch): ldh too small, mstart 0, scratch NULL; nkv_update_hessenberg j < 0
    good = L_.MATVEC_FN(lambda *_: 0)
    for args, what in (((1, 4, 4, scratch.data_ptr()), "ldh"), ((0, 4, 5, scratch.data_ptr()), "outside"),
                       ((1, 4, 5, None), "scratch")):
        ms, me, ldh, scr = args
        rc = ctx.lib.nkv_arnoldi_dcgs2(ctx._Lp, ctx.w.data_ptr(), Q.ptr, ms, me, Hd.t.data_ptr(), ldh, f.ptr, scr,
                                       ctx.ws.data_ptr(), good, None, L_.ALLREDUCE_FN(), None, 0, ctx.stream)
        assert rc == L_.NKV_EINVAL and what in L_.last_error(), (args, L_.last_error())
    rc = ctx.lib.nkv_update_hessenberg(ctx._Lp, ctx.w.data_ptr(), Q.ptr, -1, f.ptr, Q.col_ptr(1), Hd.t.data_ptr(),
                                       scratch.data_ptr(), ctx.ws.data_ptr(), L_.ALLREDUCE_FN(), None, 0, ctx.stream)
    assert rc == L_.NKV_EINVAL
    # NULL operands are refused before any launch
    for i, what in ((1, "w"), (4, "f"), (5, "q_out"), (8, "ws"), (2, "Q")):
        a = [ctx._Lp, ctx.w.data_ptr(), Q.ptr, 2, f.ptr, Q.col_ptr(2), Hd.t.data_ptr(), scratch.data_ptr(),
             ctx.ws.data_ptr(), L_.ALLREDUCE_FN(), None, 0, ctx.stream]
        a[i] = None
        rc = ctx.lib.nkv_update_hessenberg(*a)
        assert rc == L_.NKV_EINVAL and f"{what} is NULL" in L_.last_error(), (what, L_.last_error())
    # the per-column one-call factorisation: the same argument checks and callback failure
    for args, what in (((1, 4, 4, scratch.data_ptr()), "ldh"), ((0, 4, 5, scratch.data_ptr()), "outside"),
                       ((1, 4, 5, None), "scratch")):
        ms, me, ldh, scr = args
        rc = ctx.lib.nkv_arnoldi_factorization(ctx._Lp, ctx.w.data_ptr(), Q.ptr, ms, me, Hd.t.data_ptr(), ldh, f.ptr,
                                               scr, ctx.ws.data_ptr(), good, None, L_.ALLREDUCE_FN(), None,
                                               L_.NKV_MGS2, ctx.stream)
        assert rc == L_.NKV_EINVAL and what in L_.last_error(), (args, L_.last_error())
    calls.clear()
    rc = ctx.lib.nkv_arnoldi_factorization(ctx._Lp, ctx.w.data_ptr(), Q.ptr, 1, 4, Hd.t.data_ptr(), 5, f.ptr,
                                           scratch.data_ptr(), ctx.ws.data_ptr(), L_.MATVEC_FN(bad), None,
                                           L_.ALLREDUCE_FN(), None, L_.NKV_MGS2, ctx.stream)
    assert rc == L_.NKV_ECALLBACK and "returned 7" in L_.last_error() and len(calls) == 1


@pytest.mark.parametrize("rank", [3, 5])
def test_native_breakdown_flag_and_mgs2_fallback(gpu, rank):
    """NKV_CHECK_BREAKDOWN on the one-call drivers (include/nekkrylov.h, "Breakdown"): on a
    rank-``rank`` operator nkv_arnoldi_dcgs2 returns NKV_EBREAKDOWN (its message names the column);
    a C host then restores Q(mstart) and H and redoes the factorisation with
    nkv_arnoldi_factorization(NKV_MGS2), without the flag (past the invariant subspace the noise
    columns' ratios are tiny by construction; MGS2 normalises them as the reference does).  The
    fallback's H and basis equal the Python-driven mgs2 factorisation bit for bit.  On a full-rank
    operator the flag adds one synchronisation and returns NKV_OK with the same bits as without it."""
    from nekstab_next_amd import _lib as L_
    from nekstab_next_amd.arnoldi import _native_scratch

    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=300)
    ctx, _ = make_ctx(lay, max_cols=32)
    d = np.zeros(lay.ld)
    for i in range(rank):
        d[7 * (i + 1)] = 0.95 - 0.1 * i
    m = 16
    ops = {"deficient": DiagOperator(ctx, d), "full": DiagOperator(ctx, syn.diag_spectrum(lay)[0])}

    def run_c(op, entry, flags, Q, Hd):
        f = ctx.vector()
        scratch = _native_scratch(ctx, m)
        base, ld8 = Q.ptr, 8 * lay.ld

        def mv(_u, x, y, _s):
            op.matvec(Q[(x - base) // ld8], f)
            return 0

        return getattr(ctx.lib, entry)(ctx._Lp, ctx.w.data_ptr(), Q.ptr, 1, m, Hd.t.data_ptr(), m + 1, f.ptr,
                                       scratch.data_ptr(), ctx.ws.data_ptr(), L_.MATVEC_FN(mv), None,
                                       L_.ALLREDUCE_FN(), None, flags, ctx.stream)

    def fresh():
        Q = ctx.basis(m + 1)
        Q[0].fill_hash(11)
        k_normalize(Q[0])
        return Q, HessenbergDev(ctx, m)

    Q, Hd = fresh()
    seed = Q.storage[0].clone()
    rc = run_c(ops["deficient"], "nkv_arnoldi_dcgs2", L_.NKV_CHECK_BREAKDOWN, Q, Hd)
    assert rc == L_.NKV_EBREAKDOWN, (rc, L_.last_error())
    assert "breakdown" in L_.last_error()
    ctx.check_nan()   # the driver cleared the NaN flag it reported
    Q.storage[0].copy_(seed)   # restore, then the reference-order fallback
    Hd.upload(np.zeros((m + 1, m), order="F"))
    assert run_c(ops["deficient"], "nkv_arnoldi_factorization", L_.NKV_MGS2, Q, Hd) == L_.NKV_OK
    Qp, Hp = fresh()
    arnoldi_factorization(ctx, ops["deficient"], Qp, Hp, 1, m, mode="mgs2")
    np.testing.assert_array_equal(Hd.download(), Hp.download())
    np.testing.assert_array_equal(Q.storage.cpu().numpy(), Qp.storage.cpu().numpy())
    # full rank: the flag returns NKV_OK, results unchanged
    res = []
    for flags in (0, L_.NKV_CHECK_BREAKDOWN):
        Q, Hd = fresh()
        assert run_c(ops["full"], "nkv_arnoldi_dcgs2", flags, Q, Hd) == L_.NKV_OK, L_.last_error()
        res.append((Hd.download(), Q.storage.cpu().numpy()))
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])


@pytest.mark.parametrize("mode", ["cgs2", "mgs2", "dcgs2"])
@pytest.mark.parametrize("name", list(LAYOUTS))
def test_arnoldi_hessenberg_vs_oracle(gpu, mode, name):
    lay = LAYOUTS[name]
    ctx, w = make_ctx(lay, max_cols=32)
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    m = 20
    Q = ctx.basis(m + 1)
    q0 = syn.hash_vector(lay, 5)
    Q[0].from_packed(q0)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, m)
    arnoldi_factorization(ctx, op, Q, Hd, 1, m, mode=mode)
    H = Hd.download()

    Qr = np.zeros((m + 1, L.len))
    Qr[0] = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, Qr[0])
    Hr = np.zeros((m + 1, m))
    dref = syn.to_reference_order(lay, d)
    orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.0),
                              Qr, Hr, 1, m)
    assert np.max(np.abs(H - Hr)) <= 1e-12 * np.max(np.abs(Hr)), np.max(np.abs(H - Hr))
    Qg = Q.storage.cpu().numpy()
    for i in range(m + 1):
        np.testing.assert_allclose(syn.to_reference_order(lay, Qg[i]), Qr[i], rtol=0, atol=1e-10)
    # orthonormality in the W inner product (orthonormality.dat check, eigensolvers.f90:335-345)
    G = np.array([[ctx.dot(Q[a], Q[b], time=False) for b in range(m + 1)] for a in range(m + 1)])
    assert np.max(np.abs(G - np.eye(m + 1))) < 1e-13


def test_rot2_operator_vs_numpy(gpu):
    lay = LAYOUTS["3d_scalar"]
    ctx, _ = make_ctx(lay)
    c, s, dr, _ = syn.rot2_operator(lay)
    op = Rot2Operator(ctx, c, s, dr)
    from helpers import oracle_rot2_matvec
    x = syn.hash_vector(lay, 9)
    xr = syn.to_reference_order(lay, x)
    for tr in (False, True):
        y = ctx.vector()
        (op.rmatvec if tr else op.matvec)(dev_vec(ctx, x), y)
        yr = np.zeros_like(xr)
        oracle_rot2_matvec(lay, c, s, dr, tr)(xr, yr)
        np.testing.assert_allclose(syn.to_reference_order(lay, y.to_packed()), yr, rtol=1e-15, atol=1e-16)


def test_nan_is_reported(gpu):
    lay = LAYOUTS["2d"]
    ctx, _ = make_ctx(lay)
    a = syn.hash_vector(lay, 1)
    a[17] = np.nan
    x = dev_vec(ctx, a)
    with pytest.raises(NkvNaNError):
        x.dot(x)
    ctx.check_nan()  # flag was cleared


def test_shape_errors(gpu):
    lay = LAYOUTS["2d"]
    ctx, _ = make_ctx(lay)
    from nekstab_next_amd._lib import NkvError
    v = ctx.vector()
    with pytest.raises(NkvError):
        ctx.call("nkv_block_dot", ctx.w.data_ptr(), v.ptr, 0, v.ptr, ctx.h1.data_ptr(), ctx.ws.data_ptr(), 0,
                 ctx.stream)
    # more kept columns than the rotation holds in registers (NKV_ROT_MAX_OUT = 256): refused
    with pytest.raises(NkvError, match="NKV_ROT_MAX_OUT"):
        ctx.call("nkv_rotate", v.ptr, 600, ctx.h1.data_ptr(), 600, ctx.stream)
    with pytest.raises(NkvError, match="NKV_ROT_MAX_OUT"):
        ctx.call("nkv_rotate_cols", v.ptr, 300, ctx.h1.data_ptr(), 300, 257, ctx.stream)
    with pytest.raises(NkvError, match="outside"):
        ctx.call("nkv_rotate_cols", v.ptr, 1025, ctx.h1.data_ptr(), 1025, 6, ctx.stream)
    for n_out in (0, 5):   # n_out outside [1, k]
        with pytest.raises(NkvError):
            ctx.call("nkv_rotate_cols", v.ptr, 4, ctx.h1.data_ptr(), 4, n_out, ctx.stream)
    # more columns than a multi-dot's LDS partials hold: refused before any launch
    with pytest.raises(NkvError, match="outside 1..1024"):
        ctx.call("nkv_block_dot", ctx.w.data_ptr(), v.ptr, 1025, v.ptr, ctx.h1.data_ptr(), ctx.ws.data_ptr(), 0,
                 ctx.stream)
    with pytest.raises(NkvError, match="outside 1..1024"):
        ctx.call("nkv_block_dot2", ctx.w.data_ptr(), v.ptr, 1025, v.ptr, v.ptr, ctx.h1.data_ptr(),
                 ctx.ws.data_ptr(), 0, ctx.stream)


@pytest.mark.parametrize("j", [1, 5, 8, 9, 31, 64, 65, 128, 129, 200, 256, 300])
def test_block_update_dot_fused_vs_numpy(gpu, j):
    """nkv_block_update_dot = update then weighted multi-dot, in one pass (all CPW variants +
    the two-pass fallback above 256 columns)."""
    lay = LAYOUTS["3d_scalar"]
    ctx, w = make_ctx(lay, max_cols=300)
    Q = ctx.basis(j)
    for i in range(j):
        Q[i].fill_hash(300 + i)
        Q[i].time = 0.01 * i
    f = ctx.vector()
    f.fill_hash(7)
    f.time = 0.5
    Qh = Q.storage.cpu().numpy()
    fh = f.to_packed()
    wfull = np.zeros(lay.ld)
    for f_ in range(lay.n_wf):
        wfull[f_ * lay.sv: f_ * lay.sv + lay.n_v] = w
    h = torch.as_tensor(np.linspace(-0.3, 0.7, j)).to(ctx.device)
    hout = ctx.h2[:j]
    from nekstab_next_amd._lib import NKV_TIME_DOT
    ctx.call("nkv_block_update_dot", ctx.w.data_ptr(), Q.ptr, j, h.data_ptr(), f.ptr, hout.data_ptr(),
             ctx.ws.data_ptr(), NKV_TIME | NKV_TIME_DOT, ctx.stream)
    fref = fh - h.cpu().numpy() @ Qh  # includes the time slot (NKV_TIME)
    np.testing.assert_allclose(f.to_packed(), fref, rtol=1e-12, atol=1e-13)
    t = lay.time_offset
    href = Qh @ (wfull * fref) + Qh[:, t] * fref[t]
    np.testing.assert_allclose(hout.cpu().numpy(), href, rtol=1e-12, atol=1e-12 * np.abs(href).max())


@pytest.mark.parametrize("time_dot", [True, False])
@pytest.mark.parametrize("mode", ["mgs2", "dcgs2", "mgs2-icwy", "mgs2-lagged", "mgs2-icwy-native"])
def test_arnoldi_with_time_component_vs_oracle(gpu, mode, time_dot):
    """The scalar `time` follows every update and the operator propagates it (time_scale); with
    uparam(1)==2.1 it also enters k_dot (krylov_subspace.f90:52-54), otherwise it is carried but
    kept out of every dot and norm (round 3: the CGS2 norm pass used to add it regardless)."""
    lay = LAYOUTS["3d_scalar"]
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=16, time_in_dot=time_dot)
    L = olayout(lay, time_in_dot=time_dot)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d, time_scale=0.7)
    m = 12
    Q = ctx.basis(m + 1)
    q0 = syn.hash_vector(lay, 5)
    q0[lay.time_offset] = 0.3
    Q[0].from_packed(q0)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, m)
    arnoldi_factorization(ctx, op, Q, Hd, 1, m, mode=mode)
    H = Hd.download()
    Qr = np.zeros((m + 1, L.len))
    Qr[0] = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, Qr[0])
    Hr = np.zeros((m + 1, m))
    dref = syn.to_reference_order(lay, d)
    orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.7), Qr, Hr, 1, m)
    assert np.max(np.abs(H - Hr)) <= 1e-12 * np.max(np.abs(Hr))
    times = Q.storage.cpu().numpy()[:, lay.time_offset]
    np.testing.assert_allclose(times, Qr[:, -1], rtol=1e-10, atol=1e-14)
    assert np.any(np.abs(times) > 1e-3)  # the time component is really carried


@pytest.mark.parametrize("time_dot", [False, True])
@pytest.mark.parametrize("scale", [0.05, 1.0, 7.0])
def test_mgs2_icwy_nonorthonormal_basis_vs_oracle(gpu, scale, time_dot):
    """"mgs2-icwy" (MGS in inverse compact WY form, nkv_mgs_icwy_solve) on the reference's
    non-orthonormal bases: Q(1) NOT normalised (the noise/load seed leaves ||Q(1)|| = ||A s|| != 1,
    eigensolvers.f90:192-223), where classical Gram–Schmidt is a different algorithm.  H and the
    basis against the oracle's MGS2 in the reference's operation order (krylov_decomposition.f90:
    155-186), 12 steps: H to 1e-12 of max|H|, columns to 1e-11; the same factorisation split in two
    calls (the Gram rows of columns before mstart rebuilt by multi-dots) agrees with the single call
    to 1e-13; CGS2 on the same basis is measurably different (so the test can tell the algorithms
    apart)."""
    lay = LAYOUTS["3d_scalar"]
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=16, time_in_dot=time_dot)
    L = olayout(lay, time_in_dot=time_dot)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d, time_scale=0.7)
    m = 12
    q0 = syn.hash_vector(lay, 7)
    q0[lay.time_offset] = 0.3
    q0r = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, q0r)
    q0r *= scale
    q0 = syn.from_reference_order(lay, q0r)
    Qr = np.zeros((m + 1, L.len))
    Qr[0] = q0r
    Hr = np.zeros((m + 1, m))
    dref = syn.to_reference_order(lay, d)
    orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.7), Qr, Hr, 1, m)
    out = {}
    for name, mode, splits in (("one", "mgs2-icwy", [(1, m)]), ("split", "mgs2-icwy", [(1, 5), (6, m)]),
                               ("cgs2", "cgs2", [(1, m)]), ("native", "mgs2-icwy-native", [(1, 5), (6, m)])):
        Q = ctx.basis(m + 1)
        Q[0].from_packed(q0)
        Hd = HessenbergDev(ctx, m)
        for a, b in splits:
            arnoldi_factorization(ctx, op, Q, Hd, a, b, mode=mode)
        ctx.check_nan()
        out[name] = (Hd.download(), np.stack([syn.to_reference_order(lay, Q[i].to_packed()) for i in range(m + 1)]))
    H, Qg = out["one"]
    hmax = np.max(np.abs(Hr))
    assert np.max(np.abs(H - Hr)) <= 1e-12 * hmax, np.max(np.abs(H - Hr)) / hmax
    np.testing.assert_allclose(Qg, Qr, rtol=0, atol=1e-11 * max(1.0, scale))
    assert np.max(np.abs(out["split"][0] - H)) <= 1e-13 * hmax
    # the library's one-call sequence (nkv_arnoldi_factorization, NKV_MGS_ICWY) is the Python one
    np.testing.assert_array_equal(out["native"][0], out["split"][0])
    np.testing.assert_array_equal(out["native"][1], out["split"][1])
    if scale != 1.0:
        assert np.max(np.abs(out["cgs2"][0] - Hr)) > 1e-6 * hmax



@pytest.mark.parametrize("time_dot", [False, True])
@pytest.mark.parametrize("scale", [0.05, 1.0, 7.0])
def test_mgs2_lagged_nonorthonormal_basis_vs_oracle(gpu, scale, time_dot):
    """"mgs2-lagged" (MGS2's coefficients for any basis, the second pass lagged into the next
    step's multi-dot: two reads of Q per step, arnoldi.lagged_coefficients) on the reference's
    non-orthonormal bases (Q(1) = scale x a unit vector, eigensolvers.f90:192-223) against the
    oracle's MGS2 in the reference's operation order, 12 steps: H to 1e-12 of max|H|, columns to
    1e-11; the factorisation split in two calls, or into one-column calls (Gram rows rebuilt, the
    split column finished by the closing pass) agrees with the single call to 1e-12 of max|H|; the library's one-call
    driver (NKV_MGS_LAGGED) reproduces the Python-driven split run bit for bit."""
    lay = LAYOUTS["3d_scalar"]
    w = syn.mass_weights(lay)
    ctx = NekContext(lay, weights=w, max_cols=16, time_in_dot=time_dot)
    L = olayout(lay, time_in_dot=time_dot)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d, time_scale=0.7)
    m = 12
    q0 = syn.hash_vector(lay, 7)
    q0[lay.time_offset] = 0.3
    q0r = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, q0r)
    q0r *= scale
    q0 = syn.from_reference_order(lay, q0r)
    Qr = np.zeros((m + 1, L.len))
    Qr[0] = q0r
    Hr = np.zeros((m + 1, m))
    dref = syn.to_reference_order(lay, d)
    orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.7), Qr, Hr, 1, m)
    out = {}
    for name, mode, splits in (("one", "mgs2-lagged", [(1, m)]), ("split", "mgs2-lagged", [(1, 5), (6, m)]),
                               ("native", "mgs2-lagged-native", [(1, 5), (6, m)]),
                               ("steps", "mgs2-lagged", [(1, 1), (2, 2), (3, 5), (6, m)]),
                               ("native_steps", "mgs2-lagged-native", [(1, 1), (2, 2), (3, 5), (6, m)])):
        Q = ctx.basis(m + 1)
        Q[0].from_packed(q0)
        Hd = HessenbergDev(ctx, m)
        for a, b in splits:
            arnoldi_factorization(ctx, op, Q, Hd, a, b, mode=mode)
        ctx.check_nan()
        out[name] = (Hd.download(), np.stack([syn.to_reference_order(lay, Q[i].to_packed()) for i in range(m + 1)]))
    H, Qg = out["one"]
    hmax = np.max(np.abs(Hr))
    assert np.max(np.abs(H - Hr)) <= 1e-12 * hmax, np.max(np.abs(H - Hr)) / hmax
    np.testing.assert_allclose(Qg, Qr, rtol=0, atol=1e-11 * max(1.0, scale))
    assert np.max(np.abs(out["split"][0] - H)) <= 1e-12 * hmax
    # the library's one-call sequence (nkv_arnoldi_factorization, NKV_MGS_LAGGED) is the Python one
    np.testing.assert_array_equal(out["native"][0], out["split"][0])
    np.testing.assert_array_equal(out["native"][1], out["split"][1])
    # one-column calls (mstart == mend: the first step's stage, then the closing pass at once)
    assert np.max(np.abs(out["steps"][0] - H)) <= 1e-12 * hmax
    np.testing.assert_allclose(out["steps"][1], Qg, rtol=0, atol=1e-11 * max(1.0, scale))
    np.testing.assert_array_equal(out["native_steps"][0], out["steps"][0])
    np.testing.assert_array_equal(out["native_steps"][1], out["steps"][1])


def test_mgs2_icwy_solve_entry(gpu):
    """nkv_mgs_icwy_solve alone: x = (I + L)^{-1} b for a random row-major Gram matrix (the new row
    from grow, stored into G), in place, against numpy's triangular solve; argument checks."""
    from nekstab_next_amd import _lib as lib_mod

    lib = lib_mod.load()
    st = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(3)
    for j in (1, 2, 7, 64, 257):
        ldg = j + 3
        Gh = rng.standard_normal((ldg, ldg)) * (0.5 / j)   # a near-orthonormal basis's Gram entries
        grow = rng.standard_normal(max(j - 1, 1)) * (0.5 / j)
        b = rng.standard_normal(j)
        G = torch.as_tensor(Gh).cuda()
        gr = torch.as_tensor(grow).cuda()
        x = torch.as_tensor(b).cuda()
        lib_mod.check(lib.nkv_mgs_icwy_solve(j, G.data_ptr(), ldg, gr.data_ptr(), x.data_ptr(), x.data_ptr(), st), "icwy")
        torch.cuda.synchronize()
        Lm = np.tril(Gh[:j, :j], -1)
        if j > 1:
            Lm[j - 1, : j - 1] = grow[: j - 1]
        ref = np.linalg.solve(np.eye(j) + Lm, b)
        np.testing.assert_allclose(x.cpu().numpy(), ref, rtol=1e-10, atol=1e-12)
        if j > 1:
            np.testing.assert_array_equal(G.cpu().numpy()[j - 1, : j - 1], grow[: j - 1])
    G = torch.zeros((4, 4), dtype=torch.float64, device="cuda")
    assert lib.nkv_mgs_icwy_solve(0, G.data_ptr(), 4, None, G.data_ptr(), G.data_ptr(), st) != 0
    assert lib.nkv_mgs_icwy_solve(5, G.data_ptr(), 4, None, G.data_ptr(), G.data_ptr(), st) != 0
    assert lib.nkv_mgs_icwy_solve(2, None, 4, None, G.data_ptr(), G.data_ptr(), st) != 0


def test_empty_shard(gpu):
    """A rank that owns no elements (more ranks than elements): every entry point is a no-op on
    its data and contributes zero partials; only the replicated time term is counted (rank 0)."""
    class Solo:
        rank, world, backend = 0, 3, None

        def allreduce_(self, t):
            return t

    g = NekLayout(ldim=2, lx1=4, lx2=2, nelgv=2)
    lay = g.shard(0, 3)  # elements [0*2//3, 1*2//3) = [0, 0)
    assert lay.nelv == 0 and lay.n_v == 0 and lay.sv == 0
    ctx = NekContext(lay, weights=np.zeros(0), comm=Solo(), max_cols=8)
    Q = ctx.basis(5)
    for i in range(5):
        Q[i].fill_hash(i)
    f = ctx.vector()
    f.fill_hash(9)
    h = ctx.h1[:4]
    ctx.call("nkv_block_dot", ctx.w.data_ptr(), Q.ptr, 4, f.ptr, h.data_ptr(), ctx.ws.data_ptr(), 0, ctx.stream)
    assert not np.any(h.cpu().numpy())
    from nekstab_next_amd._lib import NKV_TIME_DOT
    ctx.call("nkv_block_update_dot", ctx.w.data_ptr(), Q.ptr, 4, h.data_ptr(), f.ptr, ctx.h2[:4].data_ptr(),
             ctx.ws.data_ptr(), NKV_TIME | NKV_TIME_DOT, ctx.stream)
    ctx.call("nkv_block_update", ctx.w.data_ptr(), Q.ptr, 4, h.data_ptr(), f.ptr, ctx.scal[4:5].data_ptr(),
             ctx.ws.data_ptr(), NKV_NORM2, ctx.stream)
    assert ctx.scal[4].item() == 0.0 and not np.any(ctx.h2[:4].cpu().numpy())
    V = torch.eye(4, dtype=torch.float64, device=ctx.device).flatten()
    ctx.call("nkv_rotate", Q.ptr, 4, V.data_ptr(), 4, ctx.stream)
    ctx.call("nkv_rotate_cols", Q.ptr, 4, V.data_ptr(), 4, 2, ctx.stream)
    # DCGS2 entry points: zero partials from the empty shard, the time slot still follows the update
    from nekstab_next_amd._lib import NKV_X_IS_LAST
    hd = ctx.hd[:8]
    ctx.call("nkv_block_dot2", ctx.w.data_ptr(), Q.ptr, 4, Q.col_ptr(3), f.ptr, hd.data_ptr(), ctx.ws.data_ptr(),
             NKV_X_IS_LAST, ctx.stream)
    assert not np.any(hd.cpu().numpy())
    coef = np.zeros(3 * 3 + 8)
    coef[2 * 3 + 1] = coef[2 * 3 + 4] = 1.0
    ctx.coef[: coef.size].copy_(torch.as_tensor(coef))
    t0 = Q[3].time
    ctx.call("nkv_dcgs2_update", ctx.w.data_ptr(), Q.ptr, 3, ctx.coef.data_ptr(), Q.col_ptr(3), f.ptr, Q.col_ptr(4),
             ctx.scal[5:6].data_ptr(), ctx.ws.data_ptr(), NKV_TIME, ctx.stream)
    assert ctx.scal[5].item() == 0.0 and Q[3].time == t0
    ctx.call("nkv_dcgs2_update", ctx.w.data_ptr(), Q.ptr, 3, ctx.coef.data_ptr(), Q.col_ptr(3), f.ptr, Q.col_ptr(4),
             None, ctx.ws.data_ptr(), NKV_TIME, ctx.stream)
    assert Q[3].time == t0
    # the banded launches (NKV_DC_ROUNDS) still run once on an empty shard: the replicated time slot
    # follows the update (s = 2: qbar.time = 2 u.time, f.time = 2 (A u).time)
    coef[2 * 3 + 4] = 2.0
    ctx.coef[: coef.size].copy_(torch.as_tensor(coef))
    Q[3].time, f.time, Q[4].time = 0.25, 0.5, 9.0
    ctx.call("nkv_dcgs2_update", ctx.w.data_ptr(), Q.ptr, 3, ctx.coef.data_ptr(), Q.col_ptr(3), f.ptr, Q.col_ptr(4),
             None, ctx.ws.data_ptr(), NKV_TIME, ctx.stream)
    assert Q[3].time == 0.5 and Q[4].time == 1.0
    torch.cuda.synchronize()


# ---- DCGS2 entry points, each against numpy on the same inputs (small- and large-tile paths) ----
from nekstab_next_amd.layout import box3d_layout  # noqa: E402

DC_LAYOUTS = {"small": LAYOUTS["3d_scalar"], "large": box3d_layout(4000),   # large: >= 2048 4096-row tiles
              # large tiles with three weighted fields and no pressure segment (.not. ifpo)
              "large_3f_nopr": NekLayout(ldim=3, lx1=8, lx2=6, nelgv=6000, ifpo=False)}


def _wfull(lay, w):
    wf = np.zeros(lay.ld)
    for f_ in range(lay.n_wf):
        wf[f_ * lay.sv: f_ * lay.sv + lay.n_v] = w
    return wf


@pytest.mark.parametrize("name", list(DC_LAYOUTS))
@pytest.mark.parametrize("j", [1, 2, 7, 33])
@pytest.mark.parametrize("x_last", [False, True])
def test_block_dot2_vs_numpy(gpu, name, j, x_last):
    from nekstab_next_amd._lib import NKV_X_IS_LAST
    lay = DC_LAYOUTS[name]
    ctx, w = make_ctx(lay, max_cols=40)
    Q = ctx.basis(j + 1)
    for i in range(j):
        Q[i].fill_hash(500 + i)
        Q[i].time = 0.02 * i
    x, y = (Q[j - 1] if x_last else Q[j]), ctx.vector()
    x.fill_hash(8)
    y.fill_hash(9)
    x.time, y.time = 0.3, -0.7
    h = ctx.hd[: 2 * j]
    ctx.call("nkv_block_dot2", ctx.w.data_ptr(), Q.ptr, j, x.ptr, y.ptr, h.data_ptr(), ctx.ws.data_ptr(),
             NKV_TIME | (NKV_X_IS_LAST if x_last else 0), ctx.stream)
    Qh = Q.storage.cpu().numpy()[:j]
    wf = _wfull(lay, w)
    t = lay.time_offset
    xh, yh = x.to_packed(), y.to_packed()
    ref = np.concatenate([Qh @ (wf * xh) + Qh[:, t] * xh[t], Qh @ (wf * yh) + Qh[:, t] * yh[t]])
    np.testing.assert_allclose(h.cpu().numpy(), ref, rtol=1e-12, atol=1e-12 * np.abs(ref).max())
    if not x_last and j > 1:   # the flag is refused when x is not column j-1
        with pytest.raises(NkvError):
            ctx.call("nkv_block_dot2", ctx.w.data_ptr(), Q.ptr, j, x.ptr, y.ptr, h.data_ptr(), ctx.ws.data_ptr(),
                     NKV_X_IS_LAST, ctx.stream)


def _dcgs2_coef_ref(m, hq, hw, H, beta=None):
    """numpy restatement of k_dcgs2_coef (same algebra as tests/test_dist_gloo._dcgs2_arnoldi):
    raw dots of u = beta q_j, pending subdiagonal H(m, m-1) = beta."""
    H = H.copy()
    b_ = 1.0 if beta is None else beta
    if beta is not None and m > 0:
        H[m, m - 1] = beta
    a = hq[:m] / b_
    r2 = hq[m] / b_ ** 2 - a @ a
    r = np.sqrt(r2)
    row = H[m, :m].copy()
    Hold = H[:m, :m].copy()
    H[:m, :m] += np.outer(a, row)
    H[m, :m] = row * r
    out = dict(H=H, r2s=r2 * b_ ** 2, rinv=1.0 / r, a=a, s=1.0 / b_)
    if hw is not None:
        b = hw[:m] / b_
        t = row @ a
        g = np.concatenate([Hold @ a + a * t, [r * t]])
        c = np.concatenate([(b - g[:m]) / r, [((hw[m] / b_ ** 2 - a @ b) / r - g[m]) / r]])
        H[: m + 1, m] = c
        out.update(H=H, c=c, x=g[:m] / r + c[:m], y=g[m] / r + c[m])
    return out


@pytest.mark.parametrize("m", [0, 1, 5, 40])
@pytest.mark.parametrize("with_hw", [True, False])
@pytest.mark.parametrize("beta", [None, 1.3])
def test_dcgs2_coef_vs_numpy(gpu, m, with_hw, beta):
    rng = np.random.default_rng(m)
    k = 48
    ctx, _ = make_ctx(LAYOUTS["2d"], max_cols=k)
    H = np.zeros((k + 1, k))
    H[: m + 1, :m] = np.triu(rng.standard_normal((m + 1, m)), -1)
    b_ = 1.0 if beta is None else beta
    hq = np.concatenate([1e-9 * rng.standard_normal(m) * b_, [(1.0 + 1e-3) * b_ ** 2]])
    hw = rng.standard_normal(m + 1)
    Hd = HessenbergDev(ctx, k)
    Hd.upload(H)
    hqd = torch.as_tensor(hq).to(ctx.device)
    hwd = torch.as_tensor(hw).to(ctx.device)
    nrm = torch.tensor([b_ ** 2], dtype=torch.float64, device=ctx.device)
    ctx.call_nl("nkv_dcgs2_coef", m, hqd.data_ptr(), hwd.data_ptr() if with_hw else None,
                None if beta is None else nrm.data_ptr(), Hd.t.data_ptr(), k + 1, ctx.coef.data_ptr(),
                ctx.ws.data_ptr(), ctx.stream)
    ref = _dcgs2_coef_ref(m, hq, hw if with_hw else None, H, beta)
    coef = ctx.coef.cpu().numpy()
    np.testing.assert_allclose(Hd.download(), ref["H"], rtol=1e-13, atol=1e-14)
    np.testing.assert_allclose(coef[2 * m + 1], ref["rinv"], rtol=1e-14)
    np.testing.assert_allclose(coef[2 * m + 3], ref["r2s"], rtol=1e-14)
    np.testing.assert_allclose(coef[2 * m + 4], ref["s"], rtol=1e-15)
    np.testing.assert_allclose(coef[2 * m + 5: 3 * m + 5], ref["a"], rtol=1e-14, atol=1e-30)
    if with_hw:
        np.testing.assert_allclose(coef[:m], ref["x"], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(coef[m: 2 * m + 1], ref["c"], rtol=1e-12, atol=1e-14)
        np.testing.assert_allclose(coef[2 * m + 2], ref["y"], rtol=1e-12, atol=1e-14)
    ctx.check_nan()


def test_dcgs2_coef_flags_breakdown(gpu):
    """alpha - a.a <= 0 (q_j in the span of the basis) sets the NaN flag."""
    ctx, _ = make_ctx(LAYOUTS["2d"], max_cols=8)
    Hd = HessenbergDev(ctx, 8)
    hq = torch.as_tensor(np.array([1.0, 1.0])).to(ctx.device)   # a = [1], alpha = 1 -> r2 = 0
    ctx.call_nl("nkv_dcgs2_coef", 1, hq.data_ptr(), hq.data_ptr(), None, Hd.t.data_ptr(), 9, ctx.coef.data_ptr(),
                ctx.ws.data_ptr(), ctx.stream)
    with pytest.raises(NkvNaNError):
        ctx.check_nan()


@pytest.mark.parametrize("with_norm", [True, False])
@pytest.mark.parametrize("name", list(DC_LAYOUTS))
@pytest.mark.parametrize("m", [0, 1, 6, 31])
def test_dcgs2_update_vs_numpy(gpu, name, m, with_norm):
    lay = DC_LAYOUTS[name]
    ctx, w = make_ctx(lay, max_cols=40)
    Q = ctx.basis(m + 2)
    for i in range(m + 1):
        Q[i].fill_hash(700 + i)
        Q[i].time = 0.05 * (i + 1)
    f = ctx.vector()
    f.fill_hash(77)
    f.time = 0.4
    rng = np.random.default_rng(m)
    a = rng.standard_normal(m) * 1e-2
    x = rng.standard_normal(m) * 0.3
    rinv, yc, sc = 1.0 / 1.0003, 0.27, 1.0 / 1.7
    coef = np.zeros(3 * m + 8)
    coef[:m] = x
    coef[2 * m + 1], coef[2 * m + 2], coef[2 * m + 4] = rinv, yc, sc
    coef[2 * m + 5: 3 * m + 5] = a
    ctx.coef[: coef.size].copy_(torch.as_tensor(coef))
    Qh = Q.storage.cpu().numpy()
    fh = f.to_packed()
    nrm = ctx.scal[3:4]
    nrm.fill_(-1.0)
    ctx.call("nkv_dcgs2_update", ctx.w.data_ptr(), Q.ptr, m, ctx.coef.data_ptr(), Q.col_ptr(m), f.ptr,
             Q.col_ptr(m + 1), nrm.data_ptr() if with_norm else None, ctx.ws.data_ptr(), NKV_TIME, ctx.stream)
    qbar = (Qh[m] * sc - a @ Qh[:m]) * rinv          # every row incl. the time slot (NKV_TIME)
    fref = fh * sc * rinv - x @ Qh[:m] - qbar * yc
    np.testing.assert_allclose(Q.storage[m].cpu().numpy(), qbar, rtol=1e-12, atol=1e-13)
    np.testing.assert_allclose(Q.storage[m + 1].cpu().numpy(), fref, rtol=1e-12, atol=1e-13)
    np.testing.assert_array_equal(f.to_packed(), fh)   # the matvec output is only read
    wf = _wfull(lay, w)
    if with_norm:
        np.testing.assert_allclose(nrm.item(), np.sum(wf * fref * fref), rtol=1e-12)
    else:
        assert nrm.item() == -1.0   # no norm requested: nothing reduced, nothing written


@pytest.mark.parametrize("mode", ["cgs2", "dcgs2"])
def test_arnoldi_long_vs_oracle(gpu, mode):
    """m = 300 > 256: the two-pass fallback of the fused cgs2 middle pass, DCGS2's 2j-wide dots and
    its coefficient kernel at large j, against the reference-order MGS2 oracle."""
    lay = LAYOUTS["2d"]
    m = 300
    ctx, w = make_ctx(lay, max_cols=m + 1)
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    Q = ctx.basis(m + 1)
    q0 = syn.hash_vector(lay, 5)
    Q[0].from_packed(q0)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, m)
    arnoldi_factorization(ctx, op, Q, Hd, 1, m, mode=mode)
    H = Hd.download()
    Qr = np.zeros((m + 1, L.len))
    Qr[0] = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, Qr[0])
    Hr = np.zeros((m + 1, m))
    dref = syn.to_reference_order(lay, d)
    orc.set_threads(8)
    try:
        orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.0),
                                  Qr, Hr, 1, m)
    finally:
        orc.set_threads(1)
    assert np.max(np.abs(H - Hr)) <= 1e-11 * np.max(np.abs(Hr)), np.max(np.abs(H - Hr))
    idx = [0, 1, 150, 299, 300]
    G = np.array([[ctx.dot(Q[a], Q[b], time=False) for b in idx] for a in idx])
    assert np.max(np.abs(G - np.eye(len(idx)))) < 1e-12


def test_c_host_example_runs(gpu):
    """examples/c_host/arnoldi_c: 24 DCGS2 Arnoldi steps driven from plain C through the ABI (the
    integration a Fortran/C host performs), W-orthonormality and the Arnoldi relation to 1e-12."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "c_host", "arnoldi_c")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True, timeout=300)
    p = subprocess.run([exe, "512", "24"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "arnoldi_c: OK" in p.stdout


def test_fortran_host_example_runs(gpu):
    """examples/fortran_host/arnoldi_f: the DCGS2 loop of INTEGRATION.md §2b from Fortran through the
    bind(C) interface (the reference's language): W-orthonormality and Arnoldi relation to 1e-12;
    and the default noise seed's unnormalised Q(1) through nkv_arnoldi_factorization with NKV_MGS2 and
    with NKV_MGS_ICWY, equal to 1e-12 of max|H|."""
    import os
    import subprocess

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = os.path.join(root, "examples", "fortran_host", "arnoldi_f")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(exe)], check=True, timeout=300)
    p = subprocess.run([exe, "512", "24"], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "arnoldi_f: OK" in p.stdout
    assert "unnormalised Q(1)" in p.stdout


@pytest.mark.parametrize("mode", ["dcgs2"])
def test_arnoldi_at_max_columns(gpu, mode):
    """m = 1000 steps, max_cols = 1001: the widest factorisation the ABI takes (NKV_MAX_COLS = 1024
    bounds the closing multi-dot; the two-vector dot keeps 8j partials in LDS, the coefficient
    kernel its j-vectors).  Checks:
    W-orthonormality of all 1001 columns, the Arnoldi relation, and the first 20 columns of H
    against the reference-order oracle."""
    lay = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=60)   # N_w = 4,320 > m
    m = 1000
    ctx, w = make_ctx(lay, max_cols=m + 1)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    Q = ctx.basis(m + 1)
    q0 = syn.hash_vector(lay, 5)
    Q[0].from_packed(q0)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, m)
    arnoldi_factorization(ctx, op, Q, Hd, 1, m, mode=mode)
    ctx.check_nan()
    H = Hd.download()
    Qh = Q.storage.cpu().numpy()
    wf = _wfull(lay, w)
    G = Qh @ (wf[None, :] * Qh).T
    assert np.max(np.abs(G - np.eye(m + 1))) < 1e-12
    f = ctx.vector()
    for jcol in (0, 499, m - 1):   # A q_j - Q[:, :j+2] H[:j+2, j]
        op.matvec(Q[jcol], f)
        r = f.to_packed() - H[: jcol + 2, jcol] @ Qh[: jcol + 2]
        assert np.sqrt(np.sum(wf * r * r)) <= 1e-12 * np.max(np.abs(H)), jcol
    L = olayout(lay)
    Qr = np.zeros((21, L.len))
    Qr[0] = syn.to_reference_order(lay, q0)
    orc.k_normalize(L, w, Qr[0])
    Hr = np.zeros((21, 20))
    dref = syn.to_reference_order(lay, d)
    orc.arnoldi_factorization(L, w, lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.0),
                              Qr, Hr, 1, 20)
    assert np.max(np.abs(H[:21, :20] - Hr)) <= 1e-12 * np.max(np.abs(Hr))


def test_legacy_krylov_vector_api_vs_oracle(gpu):
    """The free-subroutine krylov_vector API (krylov_subspace.f90:94-161) over the device vectors —
    k_zero, k_copy (fields and time), k_cmult, k_add2, k_sub2, k_sub3 — against the oracle's C
    restatement on the same data, every op carrying the time slot."""
    from nekstab_next_amd.vector import k_add2, k_cmult, k_copy, k_sub2, k_sub3, k_zero

    lay = LAYOUTS["3d_scalar"]
    ctx, _ = make_ctx(lay)
    L = olayout(lay)
    c = ctypes.byref(L.c)
    a, b = syn.hash_vector(lay, 41), syn.hash_vector(lay, 42)
    a[lay.time_offset], b[lay.time_offset] = 0.75, -0.5
    p, q, r = dev_vec(ctx, a), dev_vec(ctx, b), ctx.vector()
    rp, rq, rr = syn.to_reference_order(lay, a), syn.to_reference_order(lay, b), np.zeros(L.len)

    def same(v, ref):
        np.testing.assert_array_equal(syn.to_reference_order(lay, v.to_packed()), ref)

    k_copy(r, p)
    orc.lib().orc_k_copy(c, rr, rp)
    same(r, rr)
    assert r.time == 0.75
    k_cmult(r, 1.5)
    orc.lib().orc_k_cmult(c, rr, 1.5)
    same(r, rr)
    k_add2(r, q)
    orc.lib().orc_k_add2(c, rr, rq)
    same(r, rr)
    k_sub2(r, p)
    orc.lib().orc_k_sub2(c, rr, rp)
    same(r, rr)
    k_sub3(r, q, p)
    orc.lib().orc_k_sub3(c, rr, rq, rp)
    same(r, rr)
    k_zero(r)
    orc.lib().orc_k_zero(c, rr)
    same(r, rr)
    assert r.time == 0.0


@pytest.mark.parametrize("k,tgt", [(16, 5), (24, 2), (40, 4)])
def test_schur_condensation_vs_oracle(gpu, k, tgt):
    """One Krylov–Schur restart (eigensolvers.f90:363-468) on the same factorisation, the product's
    host chain on OpenBLAS against the oracle's on MKL: mstart and the selected set identical; the
    Schur vectors of the two libraries may differ by a sign (or a rotation inside a 2x2 block), so
    the kept columns are compared through the orthogonal S with Q_gpu = Q_oracle S: S orthogonal to
    1e-10, the rotated kept columns (every stored row) to 1e-11, the condensed H's kept block
    S^T T S and its b^T Z row to 1e-11 of max|H|, its spectrum to 1e-12, the rows below it zero, and
    Q(mstart) <- Q(k+1) exact."""
    from nekstab_next_amd.krylov_schur import schur_condensation

    lay = LAYOUTS["2d"]
    ctx, w = make_ctx(lay, max_cols=48)
    L = olayout(lay)
    d, _ = syn.diag_spectrum(lay)
    op = DiagOperator(ctx, d)
    Q = ctx.basis(k + 1)
    q0 = syn.hash_vector(lay, 9)
    Q[0].from_packed(q0)
    k_normalize(Q[0])
    Hd = HessenbergDev(ctx, k)
    arnoldi_factorization(ctx, op, Q, Hd, 1, k, mode="dcgs2")
    H = np.array(Hd.download(), order="F")
    Qh = Q.storage.cpu().numpy()
    Qr = np.array([syn.to_reference_order(lay, Qh[i]) for i in range(k + 1)])
    Hr = H.copy(order="F")
    from nekstab_next_amd.config import KrylovSchurConfig
    ms_d, sel_d = schur_condensation(ctx, H, Q, k, KrylovSchurConfig(k_dim=k, schur_tgt=tgt))
    assert orc.lapack_name() == "mkl"
    ms_r, sel_r = orc.schur_condensation(L, Hr, Qr, k, 0.1, tgt)
    assert ms_d == ms_r
    np.testing.assert_array_equal(sel_d, sel_r)
    ms = ms_d - 1   # kept columns
    got = Q.storage.cpu().numpy()
    Qd = np.array([syn.to_reference_order(lay, got[i])[: L.n] for i in range(ms)])
    Qo = Qr[:ms, : L.n]
    S = np.linalg.lstsq(Qo.T, Qd.T, rcond=None)[0]        # Qd = S^T Qo  (columns: Q_gpu = Q_oracle S)
    assert np.max(np.abs(S.T @ S - np.eye(ms))) < 1e-10
    assert np.max(np.abs(S.T @ Qo - Qd)) < 1e-11
    hmax = np.max(np.abs(Hr))
    assert np.max(np.abs(H[:ms, :ms] - S.T @ Hr[:ms, :ms] @ S)) <= 1e-11 * hmax
    assert np.max(np.abs(H[ms, :ms] - Hr[ms, :ms] @ S)) <= 1e-11 * hmax
    np.testing.assert_allclose(np.sort_complex(np.linalg.eigvals(H[:ms, :ms])),
                               np.sort_complex(np.linalg.eigvals(Hr[:ms, :ms])), rtol=1e-12, atol=1e-14)
    assert not H[ms + 1:].any() and not Hr[ms + 1:].any() and not H[:ms, ms:].any()
    gi = syn.to_reference_order(lay, got[ms])   # Q(mstart) <- Q(k+1), fields only
    np.testing.assert_array_equal(gi[: L.n], Qr[ms, : L.n])


@pytest.mark.parametrize("time_dot", [False, True])
def test_mgs2_step_combine_normalize_store_vs_oracle(gpu, time_dot):
    """SURVEY §8(b)'s remaining entry points: nkv_mgs2_step (the whole update_hessenberg_matrix in
    the reference's operation order, one process) against the oracle's update_hessenberg on the same
    basis and f — H column to 1e-13·max, q_out to 1e-13; nkv_combine = Q y; nkv_normalize_store =
    f/||f|| with beta returned."""
    from nekstab_next_amd._lib import NKV_TIME, NKV_TIME_DOT

    lay = LAYOUTS["3d_scalar"]
    ctx, w = make_ctx(lay, max_cols=16)
    L = olayout(lay, time_in_dot=time_dot)
    d, _ = syn.diag_spectrum(lay)
    dref = syn.to_reference_order(lay, d)
    j = 7
    Qr = np.zeros((j + 1, L.len))
    Qr[0] = syn.to_reference_order(lay, syn.hash_vector(lay, 21))
    Qr[0, -1] = 0.3 if time_dot else 0.0
    orc.k_normalize(L, w, Qr[0])
    Hr = np.zeros((j + 1, j))
    mv = lambda x, y: orc.lib().orc_op_diag(ctypes.byref(L.c), dref, x, y, 0.5)  # noqa: E731
    orc.arnoldi_factorization(L, w, mv, Qr, Hr, 1, j - 1)    # Q[0:j] orthonormal
    f_ref = np.zeros(L.len)
    mv(Qr[j - 1], f_ref)
    Q = ctx.basis(j + 1)
    for i in range(j):
        Q[i].from_packed(syn.from_reference_order(lay, Qr[i]))
    f = ctx.vector().from_packed(syn.from_reference_order(lay, f_ref))
    hcol = torch.zeros(j + 1, dtype=torch.float64, device=ctx.device)
    q_out = ctx.vector()
    ctx.call("nkv_mgs2_step", ctx.w.data_ptr(), Q.ptr, j, f.ptr, q_out.ptr, hcol.data_ptr(), ctx.ws.data_ptr(),
             NKV_TIME_DOT if time_dot else 0, ctx.stream)
    col = np.zeros(j + 1)
    wrk = L.zeros()
    fr = f_ref.copy()
    orc.lib().orc_update_hessenberg(ctypes.byref(L.c), w, col, fr, np.ascontiguousarray(Qr[:j]), j, wrk)
    h = hcol.cpu().numpy()
    np.testing.assert_allclose(h, col, rtol=0, atol=1e-13 * np.max(np.abs(col)))
    np.testing.assert_allclose(syn.to_reference_order(lay, q_out.to_packed()), fr, rtol=0, atol=1e-13)
    # nkv_combine: out = Q[:, :j] y (fields and time)
    y = np.random.default_rng(1).standard_normal(j)
    yd = torch.as_tensor(y).to(ctx.device)
    out = ctx.vector()
    ctx.call("nkv_combine", Q.ptr, j, yd.data_ptr(), out.ptr, NKV_TIME, ctx.stream)
    want = y @ Q.storage[:j].cpu().numpy()
    np.testing.assert_allclose(out.to_packed(), want, rtol=1e-13, atol=1e-14)
    # nkv_normalize_store: q_next = f / sqrt(nrm2), beta returned
    nrm2 = torch.tensor([4.0], dtype=torch.float64, device=ctx.device)
    beta = torch.zeros(1, dtype=torch.float64, device=ctx.device)
    qn = ctx.vector()
    ctx.call("nkv_normalize_store", out.ptr, nrm2.data_ptr(), qn.ptr, beta.data_ptr(), 0, ctx.stream)
    np.testing.assert_array_equal(qn.to_packed(), out.to_packed() * 0.5)
    assert beta.item() == 2.0


@pytest.mark.parametrize("name", ["2d", "3d_scalar"])
def test_inner_product_norm_normalize_vs_oracle(gpu, name):
    """The in-tree solver's inner_product / norm / normalize (eigensolvers.f90:3-116): weighted
    fields only, pressure and time never enter — even on a context with time inside k_dot
    (uparam(1)==2.1); normalize scales pressure too (nopcmult) and leaves time alone."""
    from nekstab_next_amd.vector import inner_product, norm, normalize

    lay = LAYOUTS[name]
    ctx, w = make_ctx(lay, time_in_dot=True)
    L = olayout(lay, time_in_dot=False)
    p_h, q_h = syn.hash_vector(lay, 3), syn.hash_vector(lay, 4)
    p_h[lay.time_offset], q_h[lay.time_offset] = 0.7, -1.3
    p, q = dev_vec(ctx, p_h), dev_vec(ctx, q_h)
    pr, qr = syn.to_reference_order(lay, p_h), syn.to_reference_order(lay, q_h)
    ref = orc.k_dot(L, w, pr, qr)
    assert abs(inner_product(p, q) - ref) <= 1e-13 * abs(ref)
    nref = np.sqrt(orc.k_dot(L, w, qr, qr))
    assert abs(norm(q) - nref) <= 1e-13 * nref
    a = normalize(q)
    assert abs(a - nref) <= 1e-13 * nref
    got = syn.to_reference_order(lay, q.to_packed())
    np.testing.assert_allclose(got[:-1], qr[:-1] / nref, rtol=1e-14, atol=1e-16)
    assert got[-1] == -1.3
    assert abs(inner_product(q, q) - 1.0) < 1e-14
