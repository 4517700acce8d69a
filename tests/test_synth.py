"""The config-3 generator (kad_synth_recipe_range) is SURVEY.md §8d's recipe: random_ids(n) / random_status(n)
(kad_synth_ids / kad_synth_status, the generator of configs 1, 2 and 4) restricted to a bucket range, sorted, with
the global index of the range's first node -- checked here on small tables, bucket range by bucket range."""
import numpy as np
import pytest

from opendht_amd import synth as S
from opendht_amd.sharded import ShardSpec, build_shard


@pytest.mark.parametrize("depth,lo,hi", [(10, 0, 1024), (10, 100, 300), (10, 1000, 1024), (12, 7, 8)])
def test_recipe_range_is_the_recipe(depth, lo, hi):
    n = 40_000
    ids = S.random_ids(n)
    st = S.random_status(n)
    bucket = ids[:, :8].copy().view(">u8").reshape(-1) >> np.uint64(64 - depth)
    sel = np.flatnonzero((bucket >= lo) & (bucket < hi))
    order = sel[np.lexsort(ids[sel].T[::-1])]
    want_ids, want_st = ids[order], st[order]
    want_off = np.searchsorted(bucket[order], np.arange(lo, hi + 1)).astype(np.uint32)
    got_ids, got_st, got_off, below = S.recipe_range(n, depth, lo, hi)
    np.testing.assert_array_equal(got_ids, want_ids)
    np.testing.assert_array_equal(got_st, want_st)
    np.testing.assert_array_equal(got_off, want_off)
    assert below == int((bucket < lo).sum())


def test_recipe_shards_tile_the_table():
    """Shards of a recipe spec (with their halos cut off) concatenate to the whole sorted table, and each shard's
    index_base is its first held node's global index."""
    spec = ShardSpec(n_shards=4, depth=10, recipe_n=30_000, k_max=16)
    whole, wst, woff, below = spec.bucket_range_below(0, spec.n_buckets)
    assert below == 0 and whole.shape[0] == 30_000
    for s in range(spec.n_shards):
        sh = build_shard(spec, s)
        g0 = int(woff[sh.b0])
        assert sh.index_base == g0
        np.testing.assert_array_equal(sh.ids, whole[g0:int(woff[sh.b1])])
        np.testing.assert_array_equal(sh.status, wst[g0:int(woff[sh.b1])])
        assert spec.nodes_below(sh.b0) == g0
