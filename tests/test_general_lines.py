"""General window lines (rt_gl_kernel, rt_gl16_kernel for counts 9..16, rt_gl32_kernel) and their slot lines
(rt_sl_kernel, count <= 8):
RoutingTable::findClosestNodes on tables of any
bucket shape -- the reference split policy (dht.cpp:903-934, routing_table.cpp:137-163) at 10k..300k
nodes, a mostly-bad one and a clustered one (neighbouring buckets of very different depths) -- bit-exact
against the oracle for every count 1..32, with the tables confirmed to carry the general lines (so the
new path is the one under test), before and after status changes and mirror mutations."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd._lib import (KAD_INFO_GENERAL_LINES, KAD_INFO_GENERAL_LINES16, KAD_INFO_GENERAL_LINES32,
                              KAD_INFO_SLOT_LINES, KAD_INFO_SLOT_LINES16, KAD_INFO_WINDOW_LINES, KAD_NO_NODE,
                              KAD_OP_SPLIT)

pytestmark = pytest.mark.gpu

ALL = tuple(range(1, 33))


def _check(T, t, targets, gpu, counts=ALL, status=None, mp=None):
    """Every count against the oracle; with `mp` (monkeypatch) the count <= 8 queries also through the
    128-byte general lines alone (KAD_RT_KERNEL=gl), so the slot lines and their fallback are compared, and
    counts 9..16 through the 128-byte gl16 lines without their slot-indexed copies (KAD_RT_KERNEL=gl) and through
    the 256-byte lines (KAD_RT_KERNEL=gl32) as well as the default slot lines."""
    st = t["status"] if status is None else status
    tg = torch.from_numpy(np.ascontiguousarray(targets)).to(gpu)
    for k in counts:
        idx, cnt = T.rt_closest(tg, k)
        torch.cuda.synchronize()
        want, wcnt = O.flat_rt_closest(t["ids"], st, t["first"], t["off"], targets, k, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} k={k} counts")
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k}")
        if mp is not None and k <= 8:
            mp.setenv("KAD_RT_KERNEL", "gl")
            idx2, cnt2 = T.rt_closest(tg, k)
            mp.delenv("KAD_RT_KERNEL")
            np.testing.assert_array_equal(idx2.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k} gl")
        if mp is not None and 8 < k <= 16:
            for env in ("gl", "gl32"):  # the gl16 lines without their slot-indexed copies; the 256-byte lines
                mp.setenv("KAD_RT_KERNEL", env)
                idx2, cnt2 = T.rt_closest(tg, k)
                mp.delenv("KAD_RT_KERNEL")
                np.testing.assert_array_equal(idx2.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} k={k} {env}")
                np.testing.assert_array_equal(cnt2.cpu().numpy(), wcnt, err_msg=f"{t['name']} k={k} {env} counts")


def _s_tables():
    out = [TB.split_config(10_000, seed=0x61), TB.split_config(100_000, seed=0x62),
           TB.split_config(300_000, seed=0x63, good=60, expired=25)]
    # mostly bad: windows grow past the lines' rounds, the table keeps the lane kernel (no general lines)
    bad = TB.split_config(20_000, seed=0x69, good=15, expired=40)
    bad["name"] = "S20000_mostly_bad"
    bad["lane"] = True
    out.append(bad)
    # a split table of clustered IDs: neighbouring buckets of very different depths
    rng = np.random.default_rng(0x64)
    base = S.random_ids(20_000, 0x64)
    cl = np.repeat(base[:8], 500, 0)
    cl[:, 3:] = rng.integers(0, 256, (4000, 17), dtype=np.uint8)
    ids = np.unique(np.concatenate([base, cl]), axis=0)
    rng.shuffle(ids)
    perm, first, off = S.split_table(ids)
    out.append(TB.table(ids[perm], S.random_status(perm.shape[0], 0x65), first, off, name="S_clustered"))
    return out


@pytest.mark.parametrize("t", _s_tables(), ids=lambda t: t["name"])
def test_general_lines_parity(gpu, t, monkeypatch):
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, eager=True) as T:
        f = T.info()["flags"]
        assert not (f & KAD_INFO_WINDOW_LINES)
        if not t.get("lane"):
            assert f & KAD_INFO_GENERAL_LINES and f & KAD_INFO_GENERAL_LINES32 and f & KAD_INFO_SLOT_LINES, hex(f)
            assert f & KAD_INFO_GENERAL_LINES16 and f & KAD_INFO_SLOT_LINES16, hex(f)
        _check(T, t, TB.adversarial_targets(t, extra=4000), gpu, mp=monkeypatch)


def test_general_lines_after_status_patch(gpu, monkeypatch):
    t = TB.split_config(50_000, seed=0x66)
    rng = np.random.default_rng(0x67)
    targets = TB.adversarial_targets(t, extra=3000)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0) as T:
        st = t["status"].copy()
        for frac in (0.001, 0.01, 0.2):
            m = int(st.shape[0] * frac)
            nodes = rng.choice(st.shape[0], size=m, replace=False).astype(np.uint32)
            st[nodes] = rng.choice(np.array([0, 1, 1, 2], np.uint8), size=m)
            T.patch_status(nodes, st[nodes])
            _check(T, t, targets, gpu, counts=(1, 5, 8, 9, 14, 16, 20, 32), status=st, mp=monkeypatch)


def test_uniform_table_switches_to_general_lines_after_split(gpu):
    """A U(d) table answers from uniform lines; a split breaks the uniform depth and the mirror moves it to
    general lines (kad_table_apply), still bit-exact."""
    t = TB.uniform_config(30_000, 11, seed=0x68)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0) as T:
        assert T.info()["flags"] & KAD_INFO_WINDOW_LINES
        T.apply(np.array([[KAD_OP_SPLIT, 100, 0], [KAD_OP_SPLIT, 7, 0]], np.uint32))
        ids, st, first, off = T.export()
        T.prepare()  # the count 9..32 sets of the new shape (otherwise built by their first query)
        f = T.info()["flags"]
        assert not (f & KAD_INFO_WINDOW_LINES) and f & KAD_INFO_GENERAL_LINES and f & KAD_INFO_SLOT_LINES, hex(f)
        assert f & KAD_INFO_GENERAL_LINES16 and f & KAD_INFO_SLOT_LINES16, hex(f)
        t2 = TB.table(ids, st, first, off, name="U11_split")
        _check(T, t2, TB.adversarial_targets(t2, extra=3000), gpu, counts=(1, 7, 8, 9, 16, 17, 32))


def test_dual_family_general_lines(gpu):
    """kad_rt_closest_batch_dual on two split-policy families (af per query): counts <= 8 through
    rt_dual_sl_kernel, 9..16 through rt_dual_sl16_kernel (each lane reads its family's slot line), 17..32 through
    the general-line kernels; bit-exact against the oracle per family. Then one family empty (routing_table.cpp:73):
    its queries get empty rows from the same slot-line kernels."""
    from opendht_amd import rt_closest_dual
    t4 = TB.split_config(100_000, seed=0x6B4)
    t6 = TB.split_config(60_000, seed=0x6B6, good=60, expired=25)
    rng = np.random.default_rng(0x6B)
    targets = np.ascontiguousarray(np.concatenate([TB.adversarial_targets(t4, extra=3000),
                                                   TB.adversarial_targets(t6, extra=3000)]))
    af = rng.integers(0, 2, targets.shape[0]).astype(np.uint8)
    with DeviceTable(t4["ids"], t4["status"], t4["first"], t4["off"], device=0, eager=True) as T4, \
            DeviceTable(t6["ids"], t6["status"], t6["first"], t6["off"], device=0, eager=True) as T6:
        for T in (T4, T6):
            f = T.info()["flags"]
            assert f & KAD_INFO_GENERAL_LINES and f & KAD_INFO_GENERAL_LINES16 and f & KAD_INFO_GENERAL_LINES32, hex(f)
            assert f & KAD_INFO_SLOT_LINES and f & KAD_INFO_SLOT_LINES16, hex(f)
        tg, afd = torch.from_numpy(targets).to(gpu), torch.from_numpy(af).to(gpu)
        for k in (1, 5, 8, 9, 14, 16, 17, 24, 27, 28, 32):  # 24 / 28 / 32: the quad kernel (rt_dual_wl32q_kernel<true>)
            idx, cnt = rt_closest_dual(T4, T6, tg, afd, k)
            torch.cuda.synchronize()
            idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
            for fam, t in ((0, t4), (1, t6)):
                sel = np.flatnonzero(af == fam)
                want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets[sel], k, nthreads=8)
                np.testing.assert_array_equal(cnt[sel], wcnt, err_msg=f"af={fam} k={k} counts")
                np.testing.assert_array_equal(idx[sel], want, err_msg=f"af={fam} k={k}")
        sel = np.flatnonzero(af == 0)
        for k in (1, 8, 9, 16):
            idx, cnt = rt_closest_dual(T4, None, tg, afd, k)
            torch.cuda.synchronize()
            idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
            want, wcnt = O.flat_rt_closest(t4["ids"], t4["status"], t4["first"], t4["off"], targets[sel], k, nthreads=8)
            np.testing.assert_array_equal(idx[sel], want, err_msg=f"empty IPv6 k={k}")
            np.testing.assert_array_equal(cnt[sel], wcnt, err_msg=f"empty IPv6 k={k} counts")
            assert (cnt[af == 1] == 0).all() and (idx[af == 1] == KAD_NO_NODE).all(), k


def test_general_lines_full_size_split_table(gpu):
    """The reference split policy at the per-GPU size of config 3 (12.5M nodes, ~2M buckets of mixed depth):
    1M random targets, EVERY query bit-exact against the oracle's closed form for k = 8 (slot lines), 14 and 16
    (gl16 slot copies) and 32 (256-byte lines), plus the row properties (good, ascending XOR distance)."""
    t = TB.split_config(12_500_000, seed=0x6C)
    q = 1 << 20
    g = torch.Generator(device=gpu).manual_seed(0x6C)
    tg = torch.randint(0, 256, (q, 20), dtype=torch.uint8, device=gpu, generator=g)
    targets = tg.cpu().numpy()
    key = t["ids"][:, :8].copy().view(">u8").reshape(-1)
    th = targets[:, :8].copy().view(">u8").reshape(-1)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, eager=True) as T:
        f = T.info()["flags"]
        assert f & KAD_INFO_SLOT_LINES and f & KAD_INFO_SLOT_LINES16 and f & KAD_INFO_GENERAL_LINES32, hex(f)
        for k in (8, 14, 16, 32):
            idx, cnt = T.rt_closest(tg, k)
            idx, cnt = idx.cpu().numpy().view(np.uint32), cnt.cpu().numpy()
            want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k, nthreads=16)
            np.testing.assert_array_equal(cnt, wcnt, err_msg=f"k={k} counts")
            np.testing.assert_array_equal(idx, want, err_msg=f"k={k}")
            assert (cnt == k).all()
            assert (t["status"][idx] & 1).all()
            d = key[idx] ^ th[:, None]
            assert (d[:, 1:] >= d[:, :-1]).all()
