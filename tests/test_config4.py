"""BASELINE config 4 at the survey's size: two families, a v4 and a v6 table of 1M nodes
each (independent IDs, 80/10/10 good/expired/dubious), 1M queries with `af` alternating, every query
checked against the oracle: RoutingTable::findClosestNodes for k = 8, 16, 32 (kad_rt_closest_batch_dual,
Dht::onGetValues asks both tables, dht.cpp:3216-3217) and NodeCache::getCachedNodes for 8, 14 (refill's
SEARCH_NODES, dht.cpp:1650) and 32 (kad_nc_closest_batch_dual). Plus row properties: every RoutingTable
answer is good in its family, lies inside its window W(R) and ascends in XOR distance; every NodeCache
answer is not expired."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable, nc_closest_dual, rt_closest_dual
from opendht_amd.metrics import good_counts, window_radii

pytestmark = pytest.mark.gpu

N, Q = 1_000_000, 1 << 20


@pytest.fixture(scope="module")
def fams(gpu):
    t4 = TB.uniform_config(N, 17, seed=0xC4F4)
    t6 = TB.uniform_config(N, 17, seed=0xC4F6)
    rng = np.random.default_rng(0xC4)
    targets = rng.integers(0, 256, (Q, 20), dtype=np.uint8)
    targets[:2048] = t4["ids"][rng.choice(N, 2048)]  # targets equal to node IDs of either family
    targets[2048:4096] = t6["ids"][rng.choice(N, 2048)]
    af = (np.arange(Q) % 2).astype(np.uint8)
    T4 = DeviceTable(t4["ids"], t4["status"], t4["first"], t4["off"], device=0, sorted=True)
    T6 = DeviceTable(t6["ids"], t6["status"], t6["first"], t6["off"], device=0, sorted=True)
    yield t4, t6, T4, T6, targets, af
    T4.close()
    T6.close()


def _split(targets, af):
    return np.flatnonzero(af == 0), np.flatnonzero(af == 1)


@pytest.mark.parametrize("k", [8, 16, 32])
def test_config4_rt_every_query(gpu, fams, k):
    t4, t6, T4, T6, targets, af = fams
    tg, afd = torch.from_numpy(targets).to(gpu), torch.from_numpy(af).to(gpu)
    idx, cnt = rt_closest_dual(T4, T6, tg, afd, k)
    torch.cuda.synchronize()
    idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
    for sel, t in zip(_split(targets, af), (t4, t6)):
        want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets[sel], k, nthreads=16)
        np.testing.assert_array_equal(cnt[sel], wcnt, err_msg=f"{t['name']} k={k} counts")
        np.testing.assert_array_equal(idx[sel], want, err_msg=f"{t['name']} k={k} rows")
        # properties of every row: good, inside W(R), ascending XOR distance (top 64 bits)
        rows, c = idx[sel], cnt[sel]
        valid = np.arange(k)[None, :] < c[:, None]
        assert (rows[~valid] == 0xFFFFFFFF).all()
        r = np.where(valid, rows, 0).astype(np.int64)
        assert (t["status"][r][valid] & 1).all()
        g = good_counts(t["status"], t["off"])
        R = window_radii(g, k)
        b = (targets[sel, :8].copy().view(">u8").reshape(-1) >> np.uint64(64 - 17)).astype(np.int64)
        lo, hi = np.maximum(0, b - 1 - R[b]), np.minimum(g.shape[0] - 1, b + R[b])
        off = t["off"].astype(np.int64)
        assert ((r >= off[lo][:, None]) | ~valid).all() and ((r < off[hi + 1][:, None]) | ~valid).all()
        key = t["ids"][:, :8].copy().view(">u8").reshape(-1)
        th = targets[sel, :8].copy().view(">u8").reshape(-1)
        d = key[r] ^ th[:, None]
        d = np.where(valid, d, np.uint64(0xFFFFFFFFFFFFFFFF))
        assert (d[:, 1:] >= d[:, :-1]).all()


@pytest.mark.parametrize("k", [8, 14, 32])
def test_config4_nc_every_query(gpu, fams, k):
    t4, t6, T4, T6, targets, af = fams
    tg, afd = torch.from_numpy(targets).to(gpu), torch.from_numpy(af).to(gpu)
    idx, cnt = nc_closest_dual(T4, T6, tg, afd, k)
    torch.cuda.synchronize()
    idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
    for sel, t in zip(_split(targets, af), (t4, t6)):
        want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets[sel], k, nthreads=16)
        np.testing.assert_array_equal(cnt[sel], wcnt, err_msg=f"{t['name']} nc k={k} counts")
        np.testing.assert_array_equal(idx[sel], want, err_msg=f"{t['name']} nc k={k} rows")
        rows, c = idx[sel], cnt[sel]
        valid = np.arange(k)[None, :] < c[:, None]
        assert (c == k).all()
        assert not (t["status"][np.where(valid, rows, 0).astype(np.int64)][valid] & 2).any()


def test_dual_nc_missing_family(gpu):
    """A missing family (NULL table) is an empty map: zero results for its queries."""
    t = TB.uniform_config(20_000, 11, seed=0xC4A)
    rng = np.random.default_rng(1)
    targets = rng.integers(0, 256, (5000, 20), dtype=np.uint8)
    af = (np.arange(5000) % 2).astype(np.uint8)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=True) as T:
        for k in (8, 14, 32):
            idx, cnt = nc_closest_dual(T, None, torch.from_numpy(targets).to(gpu), torch.from_numpy(af).to(gpu), k)
            torch.cuda.synchronize()
            idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
            assert (cnt[1::2] == 0).all() and (idx[1::2] == 0xFFFFFFFF).all()
            want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets[0::2], k, nthreads=8)
            np.testing.assert_array_equal(idx[0::2], want)
            np.testing.assert_array_equal(cnt[0::2], wcnt)
