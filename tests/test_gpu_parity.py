"""GPU parity: the HIP engine (through the C ABI) against the CPU oracle and the golden fixtures.
Bit-exact on indices and counts, including result order. Run with `pytest -m gpu`."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable, rt_closest_dual
from opendht_amd import synth as S
from opendht_amd._lib import KAD_NO_NODE, KadError

pytestmark = pytest.mark.gpu

COUNTS = (0, 1, 7, 8, 9, 14, 16, 17, 32)


def dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def u32(t):
    return t.cpu().numpy().view(np.uint32)


def make(t, gpu, index_base=0):
    return DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0,
                       index_base=index_base, sorted=t["sorted"])


def check_rt(T, t, targets, gpu, counts=COUNTS):
    tg = dev(targets, gpu)
    for k in counts:
        idx, cnt = T.rt_closest(tg, k)
        torch.cuda.synchronize()
        want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} k={k} counts")
        np.testing.assert_array_equal(u32(idx), want, err_msg=f"{t['name']} k={k} indices")


def check_nc(T, t, targets, gpu, counts=(0, 1, 8, 14, 32, 64)):
    tg = dev(targets, gpu)
    for k in counts:
        idx, cnt = T.nc_closest(tg, k)
        torch.cuda.synchronize()
        want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets, k, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} nc k={k} counts")
        np.testing.assert_array_equal(u32(idx), want, err_msg=f"{t['name']} nc k={k} indices")


@pytest.mark.parametrize("t", TB.all_small_tables(), ids=lambda t: t["name"])
def test_rt_closest_parity(gpu, t):
    with make(t, gpu) as T:
        check_rt(T, t, TB.adversarial_targets(t, extra=2048), gpu)


@pytest.mark.parametrize("t", [x for x in TB.all_small_tables() if x["sorted"]], ids=lambda t: t["name"])
def test_nc_closest_parity(gpu, t):
    with make(t, gpu) as T:
        check_nc(T, t, TB.adversarial_targets(t, extra=2048), gpu)


@pytest.mark.parametrize("t", TB.all_small_tables(), ids=lambda t: t["name"])
def test_find_bucket_parity(gpu, t):
    if t["first"].shape[0] == 0:
        pytest.skip("no buckets")
    targets = TB.adversarial_targets(t, extra=2048)
    F = O.FaithfulTable(t["ids"], t["status"], t["first"], t["off"])
    with make(t, gpu) as T:
        got = u32(T.find_bucket(dev(targets, gpu)))
    np.testing.assert_array_equal(got, F.find_bucket(targets))


def test_golden_config1(gpu):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "config1.npz"), allow_pickle=False)
    for shape in ("S", "U"):
        t = TB.table(g[f"{shape}_ids"], g[f"{shape}_status"], g[f"{shape}_first"], g[f"{shape}_off"],
                     sorted_=shape == "U", name=shape)
        tg = dev(g[f"{shape}_targets"], gpu)
        with make(t, gpu) as T:
            for k in (8, 16, 32):
                idx, cnt = T.rt_closest(tg, k)
                np.testing.assert_array_equal(u32(idx), g[f"{shape}_rt_idx_k{k}"])
                np.testing.assert_array_equal(cnt.cpu().numpy(), g[f"{shape}_rt_cnt_k{k}"])
            if shape == "U":
                for k in (8, 14, 32):
                    idx, cnt = T.nc_closest(tg, k)
                    np.testing.assert_array_equal(u32(idx), g[f"U_nc_idx_k{k}"])
                    np.testing.assert_array_equal(cnt.cpu().numpy(), g[f"U_nc_cnt_k{k}"])


def _wl_tables():
    """U(d) tables for the window-line kernel (count <= 8): dense buckets (offsets > 255, buckets
    with > 24 good nodes), low good fractions (R_c < R_8 for small counts, R_8 > 2), tiny tables
    whose windows are the whole table."""
    out = []
    for n, depth, good, name in ((10_000, 8, 80, "dense_U8"), (20_000, 12, 40, "U12_g40"),
                                 (20_000, 12, 60, "U12_g60"), (50_000, 14, 80, "U14_g80"),
                                 (60_000, 13, 15, "U13_g15"), (200, 3, 70, "U3_tiny"), (5, 1, 80, "U1_five")):
        t = TB.uniform_config(n, depth, seed=0x3100 + depth, good=good, expired=(100 - good) // 2)
        t["name"] = name
        out.append(t)
    return out


@pytest.mark.parametrize("t", _wl_tables(), ids=lambda t: t["name"])
def test_window_lines(gpu, t):
    """Every count the window-line kernels serve (1..8, 9..16, 17..32) on U(d) tables of every density."""
    with make(t, gpu) as T:
        check_rt(T, t, TB.adversarial_targets(t, extra=4096), gpu, counts=tuple(range(1, 33)))


def test_host_entry_points(gpu):
    t = TB.split_config(10_000)
    targets = TB.adversarial_targets(t)
    with make(t, gpu) as T:
        idx, cnt = T.rt_closest_host(targets, 8)
    want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, 8)
    np.testing.assert_array_equal(idx, want)
    np.testing.assert_array_equal(cnt, wcnt)
    u = TB.uniform_config(10_000, 10)
    with make(u, gpu) as T:
        idx, cnt = T.nc_closest_host(targets, 14)
    want, wcnt = O.flat_nc_closest(u["ids"], u["status"], targets, 14)
    np.testing.assert_array_equal(idx, want)


def test_host_entry_points_pipelined(gpu):
    """Host-pointer batches large enough for the chunked pipeline (several chunks per worker, uneven splits, the
    last chunk partial), repeated calls reusing the table's buffers, counts above 32 (smaller chunks): equal to the
    device-pointer batch and the oracle."""
    u = TB.uniform_config(200_000, 14)
    rng = np.random.default_rng(0x405)
    targets = rng.integers(0, 256, (300_001, 20), dtype=np.uint8)
    with make(u, gpu) as T:
        for k in (8, 32, 8):
            idx, cnt = T.rt_closest_host(targets, k)
            want, wcnt = O.flat_rt_closest(u["ids"], u["status"], u["first"], u["off"], targets, k, nthreads=8)
            np.testing.assert_array_equal(idx, want, err_msg=f"k={k}")
            np.testing.assert_array_equal(cnt, wcnt, err_msg=f"k={k} counts")
        for k in (14, 100):
            idx, cnt = T.nc_closest_host(targets[:150_000], k)
            di, dc = T.nc_closest(dev(targets[:150_000], gpu), k)
            np.testing.assert_array_equal(idx, u32(di), err_msg=f"nc k={k}")
            np.testing.assert_array_equal(cnt, dc.cpu().numpy(), err_msg=f"nc k={k} counts")
        want, wcnt = O.flat_nc_closest(u["ids"], u["status"], targets[:150_000], 14, nthreads=8)
        idx, cnt = T.nc_closest_host(targets[:150_000], 14)
        np.testing.assert_array_equal(idx, want)


def test_index_base_and_padding(gpu):
    t = TB.split_config(257, seed=99)
    targets = TB.adversarial_targets(t)
    with make(t, gpu, index_base=1_000_000) as T:
        idx, cnt = T.rt_closest(dev(targets, gpu), 32)
    idx, cnt = u32(idx), cnt.cpu().numpy()
    want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, 32)
    for i in range(targets.shape[0]):
        np.testing.assert_array_equal(idx[i, : cnt[i]], want[i, : cnt[i]] + 1_000_000)
        assert (idx[i, cnt[i]:] == KAD_NO_NODE).all()


def test_count_limits(gpu):
    """Any count for findClosestNodes (test_rt_closest_any_count); the wire step still takes at most
    KAD_MAX_COUNT candidates per query and says so."""
    t = TB.split_config(257, seed=98)
    with make(t, gpu) as T:
        tg = dev(TB.adversarial_targets(t), gpu)
        idx, cnt = T.rt_closest(tg, 33)
        torch.cuda.synchronize()
        assert idx.shape[1] == 33
        T.set_addrs(np.zeros((t["ids"].shape[0], 6), np.uint8))
        with pytest.raises(KadError):
            T.buffer_nodes(tg, torch.zeros((tg.shape[0], 33), dtype=torch.int32, device=gpu))


def test_status_update_and_refresh_from_times(gpu):
    """kad_table_update_status and the device-side Node::isGood(now) refresh (node.cpp:34-40)."""
    t = TB.split_config(10_000)
    targets = TB.adversarial_targets(t)
    rng = np.random.default_rng(5)
    with make(t, gpu) as T:
        st2 = rng.choice(np.array([0, 1, 1, 1, 2], np.uint8), size=t["ids"].shape[0])
        T.update_status(st2)
        t2 = dict(t, status=st2)
        check_rt(T, t2, targets, gpu, counts=(8, 32))
        assert T.info()["n_good"] == int((st2 & 1).sum())
        # times: steady_clock ns; now = 10 h
        now = 10 * 3600 * 10**9
        n = t["ids"].shape[0]
        m = 60 * 10**9
        time_ns = now - rng.integers(0, 20, n) * m            # 0..19 min ago
        reply_ns = now - rng.integers(0, 200, n) * m          # 0..199 min ago
        reply_ns[rng.random(n) < 0.05] = np.iinfo(np.int64).min  # never replied
        expired = (rng.random(n) < 0.1).astype(np.uint8)
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        torch.cuda.synchronize()
        good = (expired == 0) & (reply_ns >= now - 120 * m) & (time_ns >= now - 10 * m)
        st3 = (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)
        check_rt(T, dict(t, status=st3), targets, gpu, counts=(8, 14))


@pytest.mark.parametrize("pair", ["uniform_split", "uniform_uniform"])
def test_dual_family(gpu, pair):
    """Config 4: v4 and v6 tables, per-query af, k = 8/14/16/32. uniform_split: one family with window
    lines, one without (the lane path); uniform_uniform: both families answered from window lines."""
    t4 = TB.uniform_config(20_000, 11, seed=41)
    t6 = TB.split_config(20_000, seed=61) if pair == "uniform_split" else TB.uniform_config(30_000, 12, seed=62)
    targets = S.random_targets(4096, seed=9)
    af = (np.random.default_rng(3).random(4096) < 0.5).astype(np.uint8)
    with make(t4, gpu) as T4, make(t6, gpu) as T6:
        for k in (8, 14, 16, 32):
            idx, cnt = rt_closest_dual(T4, T6, dev(targets, gpu), dev(af, gpu), k)
            idx, cnt = u32(idx), cnt.cpu().numpy()
            w4, c4 = O.flat_rt_closest(t4["ids"], t4["status"], t4["first"], t4["off"], targets, k)
            w6, c6 = O.flat_rt_closest(t6["ids"], t6["status"], t6["first"], t6["off"], targets, k)
            np.testing.assert_array_equal(idx, np.where(af[:, None] == 0, w4, w6))
            np.testing.assert_array_equal(cnt, np.where(af == 0, c4, c6))


def test_primitives_batch(gpu):
    from opendht_amd import ops
    rng = np.random.default_rng(11)
    n = 5000
    a = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    b = a.copy()
    k = rng.integers(0, 21, n)
    for i in range(n):  # shared prefixes of every length, incl. equal IDs
        if k[i] < 20:
            b[i, k[i]:] = rng.integers(0, 256, 20 - k[i], dtype=np.uint8)
    a[0] = 0
    t = rng.integers(0, 256, (n, 20), dtype=np.uint8)
    xc = ops.xor_cmp(dev(t, gpu), dev(a, gpu), dev(b, gpu)).cpu().numpy()
    cb = ops.common_bits(dev(a, gpu), dev(b, gpu)).cpu().numpy().view(np.uint32)
    lb = ops.lowbit(dev(a, gpu)).cpu().numpy().view(np.uint32)
    for i in range(n):
        tb, ab, bb = t[i].tobytes(), a[i].tobytes(), b[i].tobytes()
        assert xc[i] == O.xor_cmp(tb, ab, bb)
        assert cb[i] == O.common_bits(ab, bb)
        assert lb[i] == O.lowbit(ab)


def test_config2_uniform_1M(gpu):
    """Config 2: 1M-node table U(17) x 64k queries, k = 8 (and the config 4 sweep's 16 and 32 on the
    same table), bit-exact on every query."""
    n, q = 1_000_000, 65_536
    t = TB.uniform_config(n, 17)
    targets = S.random_targets(q)
    with make(t, gpu) as T:
        check_rt(T, t, targets, gpu, counts=(8, 16, 32))
        check_nc(T, t, targets[:16384], gpu, counts=(14,))


@pytest.mark.parametrize("shard", [0, 3, 7])
def test_config3_full_shard_every_query(gpu, shard):
    """Config 3 at full per-GPU size: a 1/8 shard of the 100M-node U(24) table (~12.5M nodes plus halo;
    the first, a middle and the last shard), 1M owned queries, EVERY query bit-exact against the oracle's
    closed form (16 threads) for k = 8, 16, 32 and NodeCache k = 14, 32 (shard 0), plus the row properties
    (good, ascending XOR distance)."""
    from opendht_amd.sharded import build_shard, config3_spec
    spec = config3_spec()
    sh = build_shard(spec, shard)
    q = 1 << 20
    targets = spec.targets_for(shard, q, seed=1234 + shard)
    key = sh.ids[:, :8].copy().view(">u8").reshape(-1)
    th = targets[:, :8].copy().view(">u8").reshape(-1)
    with DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=gpu.index or 0, sorted=True) as T:
        for k in (8, 16, 32):
            idx, cnt = T.rt_closest(dev(targets, gpu), k)
            idx, cnt = u32(idx), cnt.cpu().numpy()
            assert (cnt == k).all()
            want, wcnt = O.flat_rt_closest(sh.ids, sh.status, sh.first, sh.off, targets, k, nthreads=16)
            np.testing.assert_array_equal(cnt, wcnt, err_msg=f"shard {shard} k={k} counts")
            np.testing.assert_array_equal(idx, want, err_msg=f"shard {shard} k={k}")
            assert (sh.status[idx] & 1).all()
            d = key[idx] ^ th[:, None]
            assert (d[:, 1:] >= d[:, :-1]).all()
        if shard == 0:
            for k in (14, 32):
                idx, cnt = T.nc_closest(dev(targets, gpu), k)
                want, wcnt = O.flat_nc_closest(sh.ids, sh.status, targets, k, nthreads=16)
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"nc k={k} counts")
                np.testing.assert_array_equal(u32(idx), want, err_msg=f"nc k={k}")


def _nc_tables():
    """Sorted tables for the NodeCache lines: U(d) tables of every density and good/expired mix,
    and a clustered table (300 IDs sharing their top 56 bits, 80 sharing the top 72: windows whose
    common prefix is deeper than the 24-bit line keys reach, and top-64 ties)."""
    out = _wl_tables()
    rng = np.random.default_rng(0xC1)
    base = S.random_ids(3000, 0xC1C1)
    c1 = np.repeat(base[:1], 300, 0)
    c1[:, 7:] = rng.integers(0, 256, (300, 13), dtype=np.uint8)
    c2 = np.repeat(base[1:2], 80, 0)
    c2[:, 9:] = rng.integers(0, 256, (80, 11), dtype=np.uint8)
    ids = np.unique(np.concatenate([base, c1, c2]), axis=0)
    first, off = S.uniform_buckets(ids, 8)
    t = TB.table(ids, S.random_status(ids.shape[0], 0xC2, 70, 20), first, off, sorted_=True, name="clustered")
    t["near"] = np.concatenate([c1[:64], c2[:32]])
    out.append(t)
    return out


def _nc_targets(t):
    parts = [TB.adversarial_targets(t, extra=4096)]
    if "near" in t:  # cluster members with their last byte changed: targets inside the clusters
        near = t["near"].copy()
        near[:, 19] ^= 0x5A
        parts.append(near)
    return np.ascontiguousarray(np.concatenate(parts))


@pytest.mark.parametrize("kernel", ["lines", "multi2", "wave64"])
@pytest.mark.parametrize("t", _nc_tables(), ids=lambda t: t["name"])
def test_nc_lines(gpu, t, kernel, monkeypatch):
    """NodeCache::getCachedNodes for every count 1..16 (the line kernel, default; KAD_NC_KERNEL=multi2:
    the wave-per-query kernel), 17..32, 40, 48, 63 and 64 (default: 32-node runs first, 64-node runs for the queries that
    leave them; KAD_NC_KERNEL=wave64: 64-node runs only; KAD_NC_KERNEL=multi2: 32-node runs up to 32, the
    serial walk for 40)."""
    if kernel != "lines":
        monkeypatch.setenv("KAD_NC_KERNEL", kernel)
    with make(t, gpu) as T:
        check_nc(T, t, _nc_targets(t), gpu, counts=tuple(range(1, 33)) + (40, 48, 63, 64))


def test_nc_lines_after_status_change(gpu):
    """The lines carry the expired bits: kad_table_update_status and the device isGood/isExpired
    refresh rebuild them."""
    t = TB.uniform_config(20_000, 11, seed=0x57A7)
    targets = TB.adversarial_targets(t, extra=4096)
    rng = np.random.default_rng(6)
    n = t["ids"].shape[0]
    with make(t, gpu) as T:
        st2 = rng.choice(np.array([0, 1, 2, 2, 3], np.uint8), size=n)
        T.update_status(st2)
        check_nc(T, dict(t, status=st2), targets, gpu, counts=(8, 14, 32))
        now, m = 10 * 3600 * 10**9, 60 * 10**9
        time_ns = now - rng.integers(0, 20, n) * m
        reply_ns = now - rng.integers(0, 200, n) * m
        expired = (rng.random(n) < 0.3).astype(np.uint8)
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        torch.cuda.synchronize()
        good = (expired == 0) & (reply_ns >= now - 120 * m) & (time_ns >= now - 10 * m)
        st3 = (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)
        check_nc(T, dict(t, status=st3), targets, gpu, counts=(8, 14, 32))


BIG_COUNTS = (33, 48, 64, 100, 255, 300, 1000)


def _rows_len(rows):
    """Entries before the first KAD_NO_NODE of each row (the result length for count > 255)."""
    pad = rows == KAD_NO_NODE
    return np.where(pad.any(axis=1), pad.argmax(axis=1), rows.shape[1])


@pytest.mark.parametrize("t", TB.all_small_tables() + [TB.split_config(20_000, seed=0xB16)],
                         ids=lambda t: t["name"])
def test_rt_closest_any_count(gpu, t):
    """RoutingTable::findClosestNodes takes any size_t count (routing_table.h:48, routing_table.cpp:67-111):
    counts above the line kernels' 32 run one wave per query (window from the prefix sums, every good node of
    it ranked tile against tile). Bit-exact rows for counts 33 .. 1000 on uniform, split-policy, tiny, all-bad
    and mostly-bad tables (windows that cover the whole table); the count byte saturates at 255 and the row
    padding gives the length beyond it. The same through the dual-family batch and the host-pointer batch."""
    targets = TB.adversarial_targets(t, extra=600)
    tg = dev(targets, gpu)
    with make(t, gpu) as T:
        for k in BIG_COUNTS:
            idx, cnt = T.rt_closest(tg, k)
            torch.cuda.synchronize()
            want, _ = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k, nthreads=8)
            got = u32(idx)
            np.testing.assert_array_equal(got, want, err_msg=f"{t['name']} k={k} indices")
            m = _rows_len(want)
            np.testing.assert_array_equal(cnt.cpu().numpy(), np.minimum(m, 255), err_msg=f"{t['name']} k={k} counts")
            if k in (33, 255):
                af = torch.zeros(targets.shape[0], dtype=torch.uint8, device=gpu)
                af[1::2] = 1
                di, dc = rt_closest_dual(T, None, tg, af, k)
                torch.cuda.synchronize()
                even = np.arange(targets.shape[0]) % 2 == 0
                np.testing.assert_array_equal(u32(di)[even], want[even], err_msg=f"{t['name']} dual k={k}")
                assert (dc.cpu().numpy()[~even] == 0).all() and (u32(di)[~even] == KAD_NO_NODE).all()
                hi, hc = T.rt_closest_host(targets, k)
                np.testing.assert_array_equal(hi, want, err_msg=f"{t['name']} host k={k}")
                np.testing.assert_array_equal(hc, np.minimum(m, 255))


@pytest.mark.parametrize("t", [x for x in TB.all_small_tables() if x["sorted"]] + [TB.uniform_config(20_000, 11, seed=0xB17)],
                         ids=lambda t: t["name"])
def test_nc_closest_any_count(gpu, t):
    """NodeCache::getCachedNodes takes any size_t count (node_cache.h:32, node_cache.cpp:36-66): counts above 64
    run the serial walk (a lane per query). Bit-exact rows for counts 65 .. 1000 and one above the map's size; the
    count byte saturates at 255 and the row padding gives the length beyond it. The same through the dual-family
    batch and the host-pointer batch."""
    from opendht_amd import nc_closest_dual

    targets = TB.adversarial_targets(t, extra=400)
    tg = dev(targets, gpu)
    with make(t, gpu) as T:
        for k in (65, 100, 255, 300, 1000, t["ids"].shape[0] + 3):
            idx, cnt = T.nc_closest(tg, k)
            torch.cuda.synchronize()
            want, _ = O.flat_nc_closest(t["ids"], t["status"], targets, k, nthreads=8)
            np.testing.assert_array_equal(u32(idx), want, err_msg=f"{t['name']} nc k={k} indices")
            m = _rows_len(want)
            np.testing.assert_array_equal(cnt.cpu().numpy(), np.minimum(m, 255), err_msg=f"{t['name']} nc k={k} counts")
            if k in (65, 300):
                af = torch.zeros(targets.shape[0], dtype=torch.uint8, device=gpu)
                af[1::2] = 1
                di, dc = nc_closest_dual(T, None, tg, af, k)
                torch.cuda.synchronize()
                even = np.arange(targets.shape[0]) % 2 == 0
                np.testing.assert_array_equal(u32(di)[even], want[even], err_msg=f"{t['name']} nc dual k={k}")
                assert (dc.cpu().numpy()[~even] == 0).all() and (u32(di)[~even] == KAD_NO_NODE).all()
                hi, hc = T.nc_closest_host(targets, k)
                np.testing.assert_array_equal(hi, want, err_msg=f"{t['name']} nc host k={k}")
                np.testing.assert_array_equal(hc, np.minimum(m, 255))


def test_host_batch_small_and_large(gpu):
    """kad_rt_closest_batch_host: batches of 1 .. 1024 queries with count <= 64 take the one-launch path on mapped
    pinned memory, larger ones the chunked pipeline; both equal the device batch."""
    t = TB.uniform_config(60_000, 13, seed=0x5A11)
    targets = TB.adversarial_targets(t, extra=5000)
    with make(t, gpu) as T:
        for q in (1, 2, 64, 1024, 1025, targets.shape[0]):
            for k in (8, 14, 32, 64, 65):
                hi, hc = T.rt_closest_host(targets[:q], k)
                want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets[:q], k)
                np.testing.assert_array_equal(hi, want, err_msg=f"q={q} k={k}")
                np.testing.assert_array_equal(hc, wcnt, err_msg=f"q={q} k={k} counts")
            ni, nc = T.nc_closest_host(targets[:q], 14)
            want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets[:q], 14)
            np.testing.assert_array_equal(ni, want, err_msg=f"nc q={q}")
            np.testing.assert_array_equal(nc, wcnt)
