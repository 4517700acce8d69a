"""NodeCache mutation mirror (kad_nc_apply): a NodeCache family map (std::map<InfoHash, weak_ptr<Node>>,
node_cache.h:42-50) changes on every message -- NodeMap::getNode(id, addr, now, confirm) emplaces new IDs,
getNode(id) erases an entry whose node died, clearBadNodes erases the dead ones and resets the rest
(node_cache.cpp:79-115). The device copy follows with a sorted merge instead of a re-snapshot. After random
batches the device array equals the model map (a sorted list), the remap / new indices are right, and
getCachedNodes equals the oracle on the model for counts 1..32, 48, 64."""
import numpy as np
import pytest
import torch

import oracle as O
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd._lib import KadError

pytestmark = pytest.mark.gpu

COUNTS = tuple(range(1, 33)) + (48, 64)


def _key(ids):
    return [bytes(r) for r in ids]


def _check(T, ids, st, gpu, rng, counts=COUNTS):
    gids, gst, _, _ = T.export()
    np.testing.assert_array_equal(gids, ids)
    np.testing.assert_array_equal(gst, st)
    targets = np.concatenate([rng.integers(0, 256, (3000, 20), dtype=np.uint8), ids[rng.choice(ids.shape[0], 500)]])
    tg = torch.from_numpy(np.ascontiguousarray(targets)).to(gpu)
    for k in counts:
        idx, cnt = T.nc_closest(tg, k)
        torch.cuda.synchronize()
        want, wcnt = O.flat_nc_closest(ids, st, targets, k, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"k={k} counts")
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"k={k} rows")


@pytest.mark.parametrize("n0", [20_000, 200_000])
def test_nc_apply_batches(gpu, n0):
    rng = np.random.default_rng(n0)
    ids, _ = S.sort_ids(S.random_ids(n0, 0x4E43 + n0))
    st = (rng.random(n0) < 0.15).astype(np.uint8) * 2  # expired bit
    T = DeviceTable(ids, st, device=0, sorted=True)
    erased_pool = []
    for batch in range(4):
        n = ids.shape[0]
        ne, ni = int(n * 0.02), int(n * 0.03)
        erase = rng.choice(n, size=ne, replace=False).astype(np.uint32)
        new = S.random_ids(ni, 0x77 + batch * 1000 + n0)
        near = ids[rng.choice(n, size=ni // 4)].copy()  # IDs next to existing ones (same top 15 bytes)
        near[:, 15:] = rng.integers(0, 256, (near.shape[0], 5), dtype=np.uint8)
        cand = np.concatenate([new, near] + ([np.array(erased_pool[:50])] if erased_pool else []))
        keep = np.ones(n, bool)
        keep[erase] = False
        existing = set(_key(ids[keep]))
        seen, ins = set(), []
        for r in cand:
            b = bytes(r)
            if b not in existing and b not in seen:
                seen.add(b)
                ins.append(r)
        ins = np.array(ins, np.uint8)
        ist = (rng.random(ins.shape[0]) < 0.1).astype(np.uint8) * 2
        erased_pool = list(ids[erase[:100]])
        remap, new_index = T.nc_apply(erase, ins, ist)
        # the model: kept old entries + new ones, sorted
        allk = np.concatenate([ids[keep], ins])
        alls = np.concatenate([st[keep], ist])
        order = np.lexsort(allk.T[::-1])
        ids2, st2 = np.ascontiguousarray(allk[order]), np.ascontiguousarray(alls[order])
        pos = np.empty(order.shape[0], np.int64)
        pos[order] = np.arange(order.shape[0])
        want_remap = np.full(n, 0xFFFFFFFF, np.uint32)
        want_remap[np.flatnonzero(keep)] = pos[:keep.sum()]
        np.testing.assert_array_equal(remap, want_remap)
        np.testing.assert_array_equal(new_index, pos[keep.sum():].astype(np.uint32))
        ids, st = ids2, st2
        _check(T, ids, st, gpu, rng, counts=COUNTS if batch == 3 else (1, 8, 14, 16, 17, 32, 64))
    # clearBadNodes (node_cache.cpp:68-77, 105-115): dead entries erased, every live node reset (not expired)
    dead = rng.choice(ids.shape[0], size=100, replace=False).astype(np.uint32)
    T.nc_apply(dead)
    keep = np.ones(ids.shape[0], bool)
    keep[dead] = False
    ids = np.ascontiguousarray(ids[keep])
    st = np.zeros(ids.shape[0], np.uint8)
    T.update_status(st)
    _check(T, ids, st, gpu, rng, counts=(1, 8, 14, 32))
    T.close()


def test_nc_apply_rejects_and_keeps_table(gpu):
    rng = np.random.default_rng(3)
    ids, _ = S.sort_ids(S.random_ids(5000, 0x4E44))
    st = np.zeros(5000, np.uint8)
    with DeviceTable(ids, st, device=0, sorted=True) as T:
        with pytest.raises(KadError):  # an ID already in the map
            T.nc_apply(None, ids[10:11], np.zeros(1, np.uint8))
        with pytest.raises(KadError):  # erase listed twice
            T.nc_apply(np.array([3, 3], np.uint32))
        with pytest.raises(KadError):  # out of range
            T.nc_apply(np.array([5000], np.uint32))
        _check(T, ids, st, gpu, rng, counts=(1, 14, 32))
        # erasing an ID and re-inserting it in the same batch is allowed
        remap, ni = T.nc_apply(np.array([10], np.uint32), ids[10:11], np.full(1, 2, np.uint8))
        assert ni[0] == 10 and remap[10] == 0xFFFFFFFF
        st[10] = 2
        _check(T, ids, st, gpu, rng, counts=(1, 14))
        # everything erased, then refilled
        T.nc_apply(np.arange(5000, dtype=np.uint32))
        assert T.info()["n_nodes"] == 0
        T.nc_apply(None, ids, st)
        _check(T, ids, st, gpu, rng, counts=(1, 14, 32))


def test_nc_apply_needs_nodecache_table(gpu):
    ids, _ = S.sort_ids(S.random_ids(3000, 0x4E45))
    first, off = S.uniform_buckets(ids, 8)
    with DeviceTable(ids, np.ones(3000, np.uint8), first, off, device=0, sorted=True) as T:
        with pytest.raises(KadError):
            T.nc_apply(np.array([1], np.uint32))
