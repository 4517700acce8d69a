"""384-byte NodeCache lines, counts 17..32 (nc32_line_kernel): 8 lanes per query, the walk's
first 64 steps as one bitonic merge, the two-pass wave path for the rest. Every test compares with the oracle
(NodeCache::getCachedNodes, node_cache.cpp:36-66) bit for bit, and with the wave path (KAD_NC_KERNEL=two_pass)."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable, nc_closest_dual
from opendht_amd import synth as S
from opendht_amd._lib import KAD_INFO_NODECACHE_LINES32

pytestmark = pytest.mark.gpu

COUNTS = (17, 20, 24, 31, 32)


def _check(t, gpu, targets, monkeypatch, counts=COUNTS):
    tg = torch.from_numpy(np.ascontiguousarray(targets)).to(gpu)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=True, eager=True) as T:
        assert T.info()["flags"] & KAD_INFO_NODECACHE_LINES32
        for k in counts:
            idx, cnt = T.nc_closest(tg, k)
            monkeypatch.setenv("KAD_NC_KERNEL", "two_pass")
            idx2, cnt2 = T.nc_closest(tg, k)
            monkeypatch.delenv("KAD_NC_KERNEL")
            torch.cuda.synchronize()
            want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets, k, nthreads=8)
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} k={k} counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k}")
            np.testing.assert_array_equal(idx2.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k} wave")
            np.testing.assert_array_equal(cnt2.cpu().numpy(), wcnt)


@pytest.mark.parametrize("n,expired", [(20_000, 10), (50_000, 45), (5_000, 80), (130, 10), (300, 30)])
def test_densities(gpu, n, expired, monkeypatch):
    """Expired-heavy maps (walks that emit fewer than `count` in 64 steps: wave path), maps barely larger
    than a line's window (clamped lines: wave path)."""
    t = TB.uniform_config(n, 8, seed=0x3200 + n, good=100 - expired, expired=expired)
    t["name"] = f"n{n}_e{expired}"
    _check(t, gpu, TB.adversarial_targets(t, extra=8192), monkeypatch)


def test_clustered(gpu, monkeypatch):
    """Clusters of IDs sharing 56 and 72 bits (adjacent nodes equal in key24: deferred lines) among random IDs."""
    rng = np.random.default_rng(0xC3)
    base = S.random_ids(20_000, 0xC3C3)
    c1 = np.repeat(base[:1], 400, 0)
    c1[:, 7:] = rng.integers(0, 256, (400, 13), dtype=np.uint8)
    c2 = np.repeat(base[1:2], 150, 0)
    c2[:, 9:] = rng.integers(0, 256, (150, 11), dtype=np.uint8)
    ids = np.unique(np.concatenate([base, c1, c2]), axis=0)
    first, off = S.uniform_buckets(ids, 8)
    t = TB.table(ids, S.random_status(ids.shape[0], 0xC4, 70, 20), first, off, sorted_=True, name="clustered32")
    near = np.concatenate([c1[:128], c2[:64]]).copy()
    near[:, 19] ^= 0x5A
    _check(t, gpu, np.concatenate([TB.adversarial_targets(t, extra=4096), near]), monkeypatch)


def test_after_status_patch(gpu):
    """The 384-byte lines carry expired bits: incremental patches rebuild the slots whose window holds a node."""
    t = TB.uniform_config(60_000, 12, seed=0x3277)
    rng = np.random.default_rng(9)
    targets = TB.adversarial_targets(t, extra=8192)
    tg = torch.from_numpy(targets).to(gpu)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=True) as T:
        st = t["status"].copy()
        for frac in (0.001, 0.02):
            nodes = rng.choice(st.shape[0], size=int(frac * st.shape[0]), replace=False).astype(np.uint32)
            st[nodes] = rng.choice(np.array([0, 1, 2, 3], np.uint8), size=nodes.shape[0])
            T.patch_status(nodes, st[nodes])
            for k in (17, 32):
                idx, cnt = T.nc_closest(tg, k)
                torch.cuda.synchronize()
                want, wcnt = O.flat_nc_closest(t["ids"], st, targets, k, nthreads=8)
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"frac {frac} k={k}")
                np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"frac {frac} k={k}")


def test_dual(gpu):
    """Dual-family batch (af per query) with the 384-byte lines in both families."""
    t4 = TB.uniform_config(30_000, 10, seed=0x3241)
    t6 = TB.uniform_config(20_000, 10, seed=0x3261, good=60, expired=30)
    targets = TB.adversarial_targets(t4, extra=4096)
    af = (np.arange(targets.shape[0]) % 3 == 1).astype(np.uint8)
    tg = torch.from_numpy(targets).to(gpu)
    with DeviceTable(t4["ids"], t4["status"], t4["first"], t4["off"], device=gpu.index or 0, sorted=True) as T4, \
            DeviceTable(t6["ids"], t6["status"], t6["first"], t6["off"], device=gpu.index or 0, sorted=True) as T6:
        for k in (17, 32):
            idx, cnt = nc_closest_dual(T4, T6, tg, torch.from_numpy(af).to(gpu), k)
            torch.cuda.synchronize()
            w4, c4 = O.flat_nc_closest(t4["ids"], t4["status"], targets, k, nthreads=8)
            w6, c6 = O.flat_nc_closest(t6["ids"], t6["status"], targets, k, nthreads=8)
            want = np.where(af[:, None] == 1, w6, w4)
            wcnt = np.where(af == 1, c6, c4)
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt)
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want)
