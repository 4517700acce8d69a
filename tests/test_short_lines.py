"""Short (64-byte) window lines, the count <= 8 path of uniform-depth tables (rt_ws_kernel).

A short line answers from 19 slots of 16-bit keys; a query it cannot answer (fallback line: 16-bit key
collision inside a bucket, offsets >= 64, a window needing more than 19 slots) reads the 128-byte line, and
from there the exact path. Each test drives one of those branches and must equal the oracle bit for bit
(indices, counts, order), and the 128-byte path (KAD_RT_KERNEL=wl) on the same queries.
"""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd._lib import KAD_INFO_SHORT_LINES, KAD_INFO_WINDOW_LINES

pytestmark = pytest.mark.gpu


def _make(t, gpu):
    return DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=t["sorted"])


def _check(t, gpu, targets, counts=range(1, 9), monkeypatch=None):
    tg = torch.from_numpy(np.ascontiguousarray(targets)).to(gpu)
    with _make(t, gpu) as T:
        assert T.info()["flags"] & KAD_INFO_SHORT_LINES, "uniform table without short lines"
        for k in counts:
            idx, cnt = T.rt_closest(tg, k)
            monkeypatch.setenv("KAD_RT_KERNEL", "wl")
            idx2, cnt2 = T.rt_closest(tg, k)
            monkeypatch.delenv("KAD_RT_KERNEL")
            torch.cuda.synchronize()
            want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k, nthreads=8)
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} k={k} counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k}")
            np.testing.assert_array_equal(idx2.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k} wl")
            np.testing.assert_array_equal(cnt2.cpu().numpy(), wcnt)


def _collision_table(n=40_000, depth=10, keys_per_bucket=3, seed=0xC011):
    """U(depth) whose nodes take their ID bits [depth, depth+16) from a few values per bucket: most buckets
    hold 16-bit key collisions (fallback short lines), bits [depth+16, depth+21) decide some of them (the
    128-byte line answers), and the rest tie on all 21 bits (the exact path)."""
    rng = np.random.default_rng(seed)
    ids = S.random_ids(n, seed)
    hi = np.frombuffer(ids[:, :8].tobytes(), dtype=">u8").astype(np.uint64)
    bucket = hi >> np.uint64(64 - depth)
    vals = rng.integers(0, 1 << 16, size=(1 << depth, keys_per_bucket), dtype=np.uint64)
    pick = vals[bucket.astype(np.int64), rng.integers(0, keys_per_bucket, size=n)]
    sh = np.uint64(64 - depth - 16)
    mask = np.uint64(0xFFFF) << sh
    hi = (hi & ~mask) | (pick << sh)
    # a quarter of the nodes also copy bits [depth+16, depth+21) of a bucket-wide value: 21-bit ties
    tie = rng.random(n) < 0.25
    sh5 = np.uint64(64 - depth - 21)
    m5 = np.uint64(0x1F) << sh5
    hi = np.where(tie, (hi & ~m5) | ((bucket & np.uint64(0x1F)) << sh5), hi)
    ids = ids.copy()
    ids[:, :8] = np.frombuffer(hi.astype(">u8").tobytes(), dtype=np.uint8).reshape(n, 8)
    ids, _ = S.sort_ids(ids)
    st = S.random_status(n, S.SEED_STATUS ^ seed, 80, 10)
    first, off = S.uniform_buckets(ids, depth)
    return TB.table(ids, st, first, off, sorted_=True, name="collisions")


def test_flags(gpu):
    u = TB.uniform_config(5000, 9)
    s = TB.split_config(5000)
    with _make(u, gpu) as T:
        f = T.info()["flags"]
        assert f & KAD_INFO_WINDOW_LINES and f & KAD_INFO_SHORT_LINES
    with _make(s, gpu) as T:
        assert not T.info()["flags"] & KAD_INFO_SHORT_LINES


def test_key_collisions(gpu, monkeypatch):
    t = _collision_table()
    _check(t, gpu, TB.adversarial_targets(t, extra=8192), monkeypatch=monkeypatch)


@pytest.mark.parametrize("n,depth,good", [(10_000, 8, 80), (40_000, 10, 30), (60_000, 14, 80), (30_000, 13, 12),
                                          (200, 3, 70), (5, 1, 80)])
def test_densities(gpu, n, depth, good, monkeypatch):
    """Dense buckets (more than 19 slots and offsets >= 64: fallback), sparse ones (R_c < R_8 for small
    counts, windows past R_8 = 2), tiny tables whose windows are the whole table."""
    t = TB.uniform_config(n, depth, seed=0x5400 + depth, good=good, expired=(100 - good) // 2)
    t["name"] = f"U{depth}_{n}_g{good}"
    _check(t, gpu, TB.adversarial_targets(t, extra=8192), monkeypatch=monkeypatch)


def test_after_status_patch(gpu, monkeypatch):
    """Short lines follow an incremental status change (transcoded from the rebuilt 128-byte lines)."""
    t = TB.uniform_config(50_000, 13, seed=0x5E9)
    rng = np.random.default_rng(5)
    targets = TB.adversarial_targets(t, extra=8192)
    tg = torch.from_numpy(targets).to(gpu)
    with _make(t, gpu) as T:
        st = t["status"].copy()
        for frac in (0.001, 0.01, 0.1):
            nodes = rng.choice(st.shape[0], size=max(1, int(frac * st.shape[0])), replace=False).astype(np.uint32)
            st[nodes] = rng.choice(np.array([0, 1, 2], np.uint8), size=nodes.shape[0])
            T.patch_status(nodes, st[nodes])
            for k in (1, 5, 8):
                idx, cnt = T.rt_closest(tg, k)
                torch.cuda.synchronize()
                want, wcnt = O.flat_rt_closest(t["ids"], st, t["first"], t["off"], targets, k, nthreads=8)
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"frac {frac} k={k}")
                np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"frac {frac} k={k}")
