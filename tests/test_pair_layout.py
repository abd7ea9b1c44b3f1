"""Complex vectors as re/im pair vectors (PairLayout, CPU): element-range sharding consistent with
the base layout at any world size, pack/unpack round trip, and the synthetic resolvent's exact
singular values."""
import numpy as np

from nekstab_next_amd import synthetic as syn
from nekstab_next_amd.layout import NekLayout, PairLayout, pair_layout


def test_pair_layout_shards_with_the_base():
    b = NekLayout(ldim=3, lx1=4, lx2=2, nelgv=11, n_scalars=1)
    for world in (1, 2, 3, 4, 7):
        tot = 0
        for r in range(world):
            bs = b.shard(r, world)
            p = pair_layout(bs)
            assert isinstance(p, PairLayout) and p.nelv == 2 * bs.nelv and p.n_p == 2 * bs.n_p
            assert p.shard(r, world) == p and p.base == bs
            tot += p.nelv
        assert tot == 2 * b.nelgv


def test_pack_unpack_round_trip():
    b = NekLayout(ldim=2, lx1=6, lx2=4, nelgv=9)
    p = pair_layout(b)
    rng = np.random.default_rng(0)
    re, im = rng.standard_normal(b.ld), rng.standard_normal(b.ld)
    r2, i2 = p.unpack(p.pack(re, im))
    for _, s, n in b.field_slices():
        np.testing.assert_array_equal(r2[s: s + n], re[s: s + n])
        np.testing.assert_array_equal(i2[s: s + n], im[s: s + n])
    assert r2[b.time_offset] == re[b.time_offset]


def test_resolvent_diag_exact_values():
    p = pair_layout(NekLayout(ldim=2, lx1=6, lx2=4, nelgv=50))
    cr, ci, sv = syn.resolvent_diag(p, omega=0.3)
    rre, _ = p.unpack(cr)
    ire, _ = p.unpack(ci)
    b = p.base
    mod = np.abs(rre[: b.n_v] + 1j * ire[: b.n_v])   # |R| on the first weighted field
    top = np.sort(np.concatenate([np.abs(rre[s: s + n] + 1j * ire[s: s + n]) for _, s, n in b.field_slices()]))[::-1]
    np.testing.assert_allclose(top[: len(sv)], sv, rtol=1e-14)
    assert mod.max() <= sv[0] * (1 + 1e-14)
