"""Sharded table: every shard answers its owned queries exactly as the whole table
would (exact halos), with global node indices. CPU: the answers come from the oracle."""
import numpy as np
import pytest

import oracle as O
from opendht_amd import synth as S
from opendht_amd.metrics import window_radii
from opendht_amd.sharded import ShardSpec, build_shard


@pytest.mark.parametrize("good,exp", [(80, 10), (30, 40)])
def test_shards_answer_like_the_whole_table(good, exp):
    spec = ShardSpec(n_shards=8, depth=11, mean_per_bucket=6.0, good_pct=good, expired_pct=exp, seed=77)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    for s in range(spec.n_shards):
        sh = build_shard(spec, s)
        assert sh.b0 <= sh.lo and sh.hi <= sh.b1
        assert sh.index_base == int(goff[sh.b0])
        np.testing.assert_array_equal(sh.ids, gids[goff[sh.b0]:goff[sh.b1]])
        tg = spec.targets_for(s, 1500, seed=5 + s)
        for k in (1, 8, 14, 32):
            a, ac = O.flat_rt_closest(sh.ids, sh.status, sh.first, sh.off, tg, k)
            a = np.where(a != 0xFFFFFFFF, a + np.uint32(sh.index_base), a)
            b, bc = O.flat_rt_closest(gids, gst, gfirst, goff, tg, k)
            np.testing.assert_array_equal(ac, bc)
            np.testing.assert_array_equal(a, b)


def test_window_radii_matches_oracle_rounds():
    spec = ShardSpec(n_shards=1, depth=9, mean_per_bucket=3.0, good_pct=50, expired_pct=20, seed=3)
    ids, st, off = spec.bucket_range(0, spec.n_buckets)
    good = np.diff(np.concatenate([[0], np.cumsum(st & 1)])[off.astype(np.int64)])
    for count in (1, 8, 32):
        R = window_radii(good, count)
        B = good.shape[0]
        for b in range(0, B, 7):
            lo, hi = max(0, b - 1), b
            g = good[lo:hi + 1].sum()
            r = 0
            while g < count and (lo > 0 or hi < B - 1):
                r += 1
                if hi < B - 1:
                    hi += 1
                    g += good[hi]
                if lo > 0:
                    lo -= 1
                    g += good[lo]
            assert R[b] == r


def test_halo_ok_detects_a_shrunk_halo():
    """The halo is sized from the build-time good counts; turning the owned edge buckets' nodes bad makes
    windows run past it, which halo_ok must report (ShardTable raises HaloError on it)."""
    from opendht_amd.sharded import halo_ok

    spec = ShardSpec(n_shards=4, depth=10, mean_per_bucket=6.0, seed=91)
    sh = build_shard(spec, 1)
    assert halo_ok(sh, sh.status)
    st = sh.status.copy()
    lo_node = int(sh.off[sh.lo - sh.b0])
    st[lo_node:lo_node + 400] = 0  # the first owned buckets go dubious: their windows grow leftwards
    assert not halo_ok(sh, st)


@pytest.mark.gpu
def test_shard_table_raises_on_halo_overrun(gpu):
    from opendht_amd.sharded import HaloError, ShardTable

    spec = ShardSpec(n_shards=4, depth=10, mean_per_bucket=6.0, seed=92)
    sh = build_shard(spec, 2)
    T = ShardTable(sh, device=0)
    st = sh.status.copy()
    T.patch_status(np.arange(5, dtype=np.uint32), st[:5])  # no change: fine
    lo_node = int(sh.off[sh.lo - sh.b0])
    nodes = np.arange(lo_node, lo_node + 400, dtype=np.uint32)
    with pytest.raises(HaloError):
        T.patch_status(nodes, np.zeros(400, np.uint8))
    T.close()
