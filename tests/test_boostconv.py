"""BoostConv (fixedp.f90:218-403): the oracle restatement stabilises a fixed-point iteration with
unstable modes and converges to the exact fixed point (CPU); the device implementation follows
the oracle step for step (GPU)."""
import numpy as np
import pytest

import oracle as orc
from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout


def _problem(lay):
    n = lay.ldim * lay.n_v
    u = syn.hash_uniform(17, 500, np.arange(n, dtype=np.uint64))
    a = 0.8 * u
    a[:2] = (1.05, 1.02)  # two unstable modes: plain iteration diverges
    b = 2.0 * syn.hash_uniform(17, 501, np.arange(n, dtype=np.uint64)) - 1.0
    return a, b, b / (1.0 - a)


def _oracle_run(lay, w, a, b, iters, boost=True, tol=1e-22):
    """v <- v + boostconv(G(v) - v); stops once the W-norm^2 of the residual is below tol, as
    BoostConv sets ifbfcv (fixedp.f90:247-250) — qr_dec has no guard on its first column, so the
    iteration must not continue past exact convergence."""
    v = np.zeros(lay.ldim * lay.n_v)
    st = {"n": 10}
    hist = []
    W = np.tile(w, lay.ldim)
    for _ in range(iters):
        vnew = a * v + b
        rb = vnew - v
        residu = float(np.sum(W * rb * rb))
        if boost:
            orc.boostconv_core(st, rb, w, rb.size)
        v = v + rb
        hist.append(v.copy())
        if residu < tol:
            break
    return hist


def test_boostconv_oracle_converges_to_fixed_point():
    lay = NekLayout(ldim=2, lx1=4, lx2=2, nelgv=30, ifpo=False)
    w = syn.mass_weights(lay)
    a, b, vstar = _problem(lay)
    plain = _oracle_run(lay, w, a, b, 200, boost=False)
    assert np.max(np.abs(plain[-1] - vstar)) > 1.0  # diverges
    hist = _oracle_run(lay, w, a, b, 200)
    assert np.max(np.abs(hist[-1] - vstar)) < 1e-8


@pytest.mark.gpu
def test_boostconv_device_matches_oracle(gpu):
    from nekstab_next_amd.boostconv import BoostConv, velocity_layout
    from nekstab_next_amd.vector import NekContext

    lay = velocity_layout(NekLayout(ldim=2, lx1=4, lx2=2, nelgv=30))
    w = syn.mass_weights(lay)
    a, b, vstar = _problem(lay)
    ctx = NekContext(lay, weights=w, max_cols=16)

    def pad(x):
        out = np.zeros(lay.ld)
        for f in range(lay.ldim):
            out[f * lay.sv: f * lay.sv + lay.n_v] = x[f * lay.n_v:(f + 1) * lay.n_v]
        return out

    def unpad(p):
        return np.concatenate([p[f * lay.sv: f * lay.sv + lay.n_v] for f in range(lay.ldim)])

    A = ctx.vector().from_packed(pad(a))
    B = ctx.vector().from_packed(pad(b))
    v, vnew, rb = ctx.vector(), ctx.vector(), ctx.vector()
    bc = BoostConv(ctx, 10)
    ref = _oracle_run(lay, w, a, b, 60)
    for it in range(60):
        ctx.call("nkv_op_diag", A.ptr, v.ptr, vnew.ptr, 0.0, ctx.stream)
        vnew.axpby(1.0, B, 1.0)
        rb.copy_from(vnew)
        rb.axpby(1.0, v, -1.0)
        bc.core(rb)
        v.axpby(1.0, rb, 1.0)
        got = unpad(v.to_packed())
        assert np.max(np.abs(got - ref[it])) <= 1e-9 * max(1.0, np.max(np.abs(ref[it]))), it
    assert np.max(np.abs(unpad(v.to_packed()) - vstar)) < 1e-6


@pytest.mark.gpu
def test_boostconv_qr_device_equals_host_and_guard(gpu):
    """The device-resident MGS QR (one host synchronisation) gives the host-scalar QR's dd and Q,
    and a numerically zero column (the reference's guard, fixedp.f90:371-376: Q(j) = 0,
    dd(j,j) = 1) sends the QR to the host form."""
    from nekstab_next_amd.boostconv import BoostConv, velocity_layout
    from nekstab_next_amd.vector import NekContext

    lay = velocity_layout(NekLayout(ldim=2, lx1=4, lx2=2, nelgv=30))
    ctx = NekContext(lay, weights=syn.mass_weights(lay), max_cols=16)
    n = 6
    bc = BoostConv(ctx, n)
    for j in range(n):
        bc.Y[j].fill_hash(900 + j)
    assert bc._qr_dec_device()
    dd_dev, Q_dev = bc.dd.copy(), bc.Q.storage.cpu().numpy().copy()
    bc._qr_dec_host()
    np.testing.assert_allclose(dd_dev, bc.dd, rtol=1e-14, atol=1e-15)
    np.testing.assert_allclose(Q_dev, bc.Q.storage.cpu().numpy(), rtol=0, atol=1e-14)
    bc.Y[3].zero()   # a zero column: the guard
    assert not bc._qr_dec_device()
    bc.qr_dec()
    assert bc.dd[3, 3] == 1.0 and not np.any(bc.Q[3].to_packed())
    G = np.array([[ctx.dot(bc.Q[a], bc.Q[b], time=False) for b in range(n)] for a in range(n)])
    keep = [0, 1, 2, 4, 5]
    np.testing.assert_allclose(G[np.ix_(keep, keep)], np.eye(5), atol=1e-13)
    ctx.check_nan()   # the device pass's 0 * inf on the zero column leaves no NaN flag behind
