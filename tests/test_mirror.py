"""Incremental device mirror: kad_table_apply replays RoutingTable mutations
(Dht::expireBuckets removals, onNewNode's expired-slot replacement and emplace_front insertion,
RoutingTable::split) on the device. Checked against the same ops on the oracle's structure-faithful
std::list table: the exported table (ids, status, firsts, offsets), every old node's new index and
every new node's index, then queries on the mutated table against the oracle."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable
from opendht_amd._lib import KAD_OP_INSERT, KAD_OP_REMOVE, KAD_OP_REPLACE, KAD_OP_SPLIT


def test_oracle_split_known_answer():
    """One bucket [0, 2^160) with nodes 0x10.., 0x90.., 0x20..: split at bit 0 -> [0x00.., 0x80..)
    holds 0x20.., 0x10.. (spliced to the front: reversed) and [0x80.., ..) holds 0x90.."""
    ids = np.zeros((3, 20), np.uint8)
    ids[0, 0], ids[1, 0], ids[2, 0] = 0x10, 0x90, 0x20
    F = O.FaithfulTable(ids, np.ones(3, np.uint8), np.zeros((1, 20), np.uint8), np.array([0, 3], np.uint32))
    out_ids, st, first, off, remap, nidx = F.apply(np.array([[KAD_OP_SPLIT, 0, 0]]), [], [])
    assert first[1, 0] == 0x80 and list(off) == [0, 2, 3]
    assert [r[0] for r in out_ids] == [0x20, 0x10, 0x90] and list(remap) == [1, 2, 0]
    F.close()


def _random_ops(t, rng, n_ops, allow_split=True):
    """A random batch: removals, in-bucket replacements, insertions, splits (old nodes used once)."""
    n = t["ids"].shape[0]
    B = t["first"].shape[0]
    order = rng.permutation(n)
    used = 0
    ops, new_ids, new_st = [], [], []
    existing = {bytes(x) for x in t["ids"]}
    cur_B = B
    for _ in range(n_ops):
        r = rng.random()
        if r < 0.3 and used < n:
            ops.append((KAD_OP_REMOVE, int(order[used]), 0))
            used += 1
        elif r < 0.55 and used < n:
            a = int(order[used])
            used += 1
            nid = t["ids"][a].copy()
            nid[12:] = rng.integers(0, 256, 8, dtype=np.uint8)  # same bucket (depth <= 96)
            if bytes(nid) in existing:
                continue
            existing.add(bytes(nid))
            ops.append((KAD_OP_REPLACE, a, len(new_ids)))
            new_ids.append(nid)
            new_st.append(rng.integers(0, 3))
        elif r < 0.9 or not allow_split:
            nid = rng.integers(0, 256, 20, dtype=np.uint8)
            if bytes(nid) in existing:
                continue
            existing.add(bytes(nid))
            ops.append((KAD_OP_INSERT, len(new_ids), 0))
            new_ids.append(nid)
            new_st.append(rng.integers(0, 3))
        else:
            ops.append((KAD_OP_SPLIT, int(rng.integers(0, cur_B)), 0))
            cur_B += 1
    new_ids = np.array(new_ids, np.uint8).reshape(-1, 20)
    return np.array(ops, np.uint32).reshape(-1, 3), new_ids, np.array(new_st, np.uint8)


def _mirror_tables():
    out = [TB.split_config(3000, seed=0x3131), TB.uniform_config(6000, 9, seed=0x3132), TB.tie_table()[0]]
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("t", _mirror_tables(), ids=lambda t: t["name"])
@pytest.mark.parametrize("split", [False, True], ids=["no_split", "split"])
def test_mirror_parity(gpu, t, split):
    rng = np.random.default_rng(len(t["name"]) + 7 * split)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=t["sorted"]) as T:
        F = O.FaithfulTable(t["ids"], t["status"], t["first"], t["off"])
        cur = dict(t)
        for batch in range(3):
            ops, nid, nst = _random_ops(cur, rng, 300, allow_split=split)
            n_old = cur["ids"].shape[0]
            remap = torch.empty(max(n_old, 1), dtype=torch.int32, device=gpu)
            got_new = T.apply(ops, nid, nst, remap=remap)
            ids, st, first, off = T.export()
            w_ids, w_st, w_first, w_off, w_remap, w_new = F.apply(ops, nid, nst)
            np.testing.assert_array_equal(first, w_first, err_msg=f"batch {batch} firsts")
            np.testing.assert_array_equal(off, w_off, err_msg=f"batch {batch} offsets")
            np.testing.assert_array_equal(ids, w_ids, err_msg=f"batch {batch} ids")
            np.testing.assert_array_equal(st, w_st, err_msg=f"batch {batch} status")
            np.testing.assert_array_equal(remap.cpu().numpy().view(np.uint32)[:n_old], w_remap)
            np.testing.assert_array_equal(got_new, w_new)
            cur = dict(t, ids=w_ids, status=w_st, first=w_first, off=w_off)
            F.close()
            F = O.FaithfulTable(w_ids, w_st, w_first, w_off)
            # queries on the mutated device table
            targets = TB.adversarial_targets(cur, extra=1500)
            tg = torch.from_numpy(targets).to(gpu)
            for k in (1, 8, 14, 32):
                idx, cnt = T.rt_closest(tg, k)
                torch.cuda.synchronize()
                want, wcnt = O.flat_rt_closest(w_ids, w_st, w_first, w_off, targets, k)
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"batch {batch} k={k}")
                np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"batch {batch} k={k}")
        F.close()
