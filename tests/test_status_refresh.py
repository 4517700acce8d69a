"""Incremental status refresh (kad_table_patch_status / update_status / patch_times + refresh_status):
after isGood / isExpired flips (Node::received, setExpired, ageing past NODE_EXPIRE_TIME; node.cpp:34-40,
82-108) only the flipped buckets' masks and the lines whose window reaches them are rebuilt. Every result
must equal the oracle on the new status: RoutingTable counts 1..32 (window lines of all three kinds and the
lane kernel) and NodeCache counts 1..32 (NodeCache lines), after 0.1 % and 1 % flips, repeated patches,
and a moving `now`."""
import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable

pytestmark = pytest.mark.gpu

RT_COUNTS = (1, 2, 3, 5, 7, 8, 9, 12, 14, 16, 17, 20, 24, 31, 32)
NC_COUNTS = (1, 2, 8, 13, 14, 16, 17, 24, 32)


def _dev(a, gpu):
    return torch.from_numpy(np.ascontiguousarray(a)).to(gpu)


def _check(T, t, status, targets, gpu, rt=RT_COUNTS, nc=NC_COUNTS):
    tg = _dev(targets, gpu)
    for k in rt:
        idx, cnt = T.rt_closest(tg, k)
        torch.cuda.synchronize()
        want, wcnt = O.flat_rt_closest(t["ids"], status, t["first"], t["off"], targets, k, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} rt k={k} counts")
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} rt k={k}")
    if t["sorted"]:
        for k in nc:
            idx, cnt = T.nc_closest(tg, k)
            torch.cuda.synchronize()
            want, wcnt = O.flat_nc_closest(t["ids"], status, targets, k, nthreads=8)
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{t['name']} nc k={k} counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{t['name']} nc k={k}")


def _tables():
    return [TB.uniform_config(60_000, 13, seed=0x5E1), TB.uniform_config(20_000, 10, seed=0x5E2),
            TB.split_config(20_000, seed=0x5E3)]


def _flip(rng, status, frac):
    n = status.shape[0]
    m = max(1, int(n * frac))
    nodes = rng.choice(n, size=m, replace=False).astype(np.uint32)
    new = rng.choice(np.array([0, 1, 1, 2, 3], np.uint8), size=m)
    st = status.copy()
    st[nodes] = new
    return nodes, new, st


@pytest.mark.parametrize("frac", [0.001, 0.01])
@pytest.mark.parametrize("t", _tables(), ids=lambda t: t["name"])
def test_patch_status(gpu, t, frac):
    rng = np.random.default_rng(int(frac * 1e4) + t["ids"].shape[0])
    targets = TB.adversarial_targets(t, extra=3000)
    st = t["status"].copy()
    with DeviceTable(t["ids"], st, t["first"], t["off"], device=0, sorted=t["sorted"]) as T:
        for rep in range(3):  # repeated patches: the flags must be cleared and the state consistent
            nodes, new, st = _flip(rng, st, frac)
            T.patch_status(nodes, new)
            assert T.info()["n_good"] == int((st & 1).sum())
            _check(T, t, st, targets, gpu, rt=RT_COUNTS if rep == 2 else (1, 8, 16, 32),
                   nc=NC_COUNTS if rep == 2 else (1, 14, 32))


def test_patch_status_neighbourhood(gpu):
    """Flips concentrated in one region (every node of 40 consecutive buckets): windows that grow or
    shrink by several rounds, lines deferred and un-deferred, targets right there."""
    t = TB.uniform_config(40_000, 12, seed=0x5E4)
    off = t["off"]
    b0 = 1000
    nodes = np.arange(off[b0], off[b0 + 40], dtype=np.uint32)
    near = t["ids"][off[b0 - 10]:off[b0 + 50]]
    targets = np.ascontiguousarray(np.concatenate([TB.adversarial_targets(t, extra=1000), near]))
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=True) as T:
        st = t["status"].copy()
        st[nodes] = 0  # the region goes dubious
        T.patch_status(nodes, st[nodes])
        _check(T, t, st, targets, gpu)
        st[nodes] = 1  # and comes back good
        T.patch_status(nodes, st[nodes])
        _check(T, t, st, targets, gpu)


def test_update_status_full_array_incremental(gpu):
    t = TB.uniform_config(30_000, 12, seed=0x5E5)
    rng = np.random.default_rng(9)
    targets = TB.adversarial_targets(t, extra=2000)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=True) as T:
        _, _, st = _flip(rng, t["status"], 0.01)
        T.update_status(st)
        _check(T, t, st, targets, gpu)


def test_moving_now(gpu):
    """Node times on the device, `now` advancing: nodes age past 10 min (time) and 120 min (reply_time),
    then some are heard again (patch_times) and some expire."""
    t = TB.uniform_config(50_000, 13, seed=0x5E6)
    n = t["ids"].shape[0]
    rng = np.random.default_rng(11)
    targets = TB.adversarial_targets(t, extra=2000)
    MIN = 60 * 10**9
    now = 100 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)         # all heard within the last 10 min
    reply_ns = now - rng.integers(0, 120 * MIN, n)       # all replied within 120 min
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=True) as T:
        T.set_times(time_ns, reply_ns, expired)
        for dt in (1, 5 * 10**8, 10 * 10**9, 60 * 10**9, 3 * MIN):  # small steps: ~0.01 % .. 30 % flips
            now += dt
            T.refresh_status(now)
            torch.cuda.synchronize()
            _check(T, t, status_at(now), targets, gpu, rt=(1, 8, 14, 32), nc=(1, 14, 32))
        # 1 % of the nodes answer now; 0.5 % get expired (setExpired); refresh at the same now
        heard = rng.choice(n, size=n // 100, replace=False).astype(np.uint32)
        time_ns[heard] = now
        reply_ns[heard] = now
        gone = rng.choice(n, size=n // 200, replace=False).astype(np.uint32)
        expired[gone] = 1
        sel = np.unique(np.concatenate([heard, gone])).astype(np.uint32)
        T.patch_times(sel, time_ns[sel], reply_ns[sel], expired[sel])
        T.refresh_status(now)
        torch.cuda.synchronize()
        _check(T, t, status_at(now), targets, gpu)


def test_patch_rejects_bad_index(gpu):
    t = TB.uniform_config(2000, 8, seed=0x5E7)
    from opendht_amd._lib import KadError

    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0) as T:
        with pytest.raises(KadError):
            T.patch_status(np.array([t["ids"].shape[0]], np.uint32), np.array([1], np.uint8))
        with pytest.raises(KadError):  # no times uploaded yet
            T.patch_times(np.array([0], np.uint32), np.array([0]), np.array([0]), np.array([0], np.uint8))


def test_now_walk_across_deadlines(gpu):
    """kad_table_refresh_status follows `now` through the nodes' isGood deadlines (node.cpp:34-40: good while
    now <= min(time + 10 min, reply_time + 120 min)): steps of 1 ns, steps landing exactly on a deadline (the
    node is still good) and 1 ns past it, steps across thousands of deadlines, a refresh at the same `now`,
    patch_times in between (nodes heard again turn good at the next refresh whatever `now`; setExpired), a
    step back in time (every node re-derived) and forward again. After every step the status bytes equal
    isGood / isExpired at that `now`, and at some steps every query equals the oracle."""
    t = TB.uniform_config(40_000, 12, seed=0x5E8)
    n = t["ids"].shape[0]
    rng = np.random.default_rng(0x5E8)
    targets = TB.adversarial_targets(t, extra=1500)
    MIN = 60 * 10**9
    now0 = now = 500 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    time_ns[:300] = now - 5 * MIN  # 300 nodes share one deadline
    reply_ns[:300] = now
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    def deadlines():
        d = np.minimum(time_ns + 10 * MIN, reply_ns + 120 * MIN)
        return np.sort(d[(expired == 0) & (d >= now)])

    def step(tnow, check_queries=False):
        T.refresh_status(tnow)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(T.export_status(), status_at(tnow), err_msg=f"now={tnow}")
        if check_queries:
            _check(T, t, status_at(tnow), targets, gpu, rt=(1, 8, 14, 32), nc=(1, 14, 32))

    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=True) as T:
        T.set_times(time_ns, reply_ns, expired)
        step(now)
        for j in range(40):
            d = deadlines()
            kind = j % 5
            if kind == 0:
                now += 1
            elif kind == 1:
                now = int(d[min(len(d) - 1, 7)])  # exactly on a deadline: that node is still good
            elif kind == 2:
                now += 1  # ... and 1 ns later it is not
            elif kind == 3:
                now = int(d[min(len(d) - 1, 2000)]) + 1  # across ~2000 deadlines
            else:
                pass  # the same `now` again
            step(now, check_queries=(j % 10 == 3))
            if j == 12 and now < now0 + 5 * MIN:  # the 300 nodes sharing a deadline: on it, then past it
                now = now0 + 5 * MIN
                step(now)
                now += 1
                step(now)
            if j in (15, 25):  # some nodes are heard again (good again at once), some expire
                heard = rng.choice(n, size=n // 50, replace=False).astype(np.uint32)
                time_ns[heard] = now
                reply_ns[heard] = now - rng.integers(0, 3 * MIN, heard.shape[0])
                gone = rng.choice(n, size=n // 400, replace=False).astype(np.uint32)
                expired[gone] = 1
                sel = np.unique(np.concatenate([heard, gone])).astype(np.uint32)
                T.patch_times(sel, time_ns[sel], reply_ns[sel], expired[sel])
                step(now, check_queries=True)
            if j == 30:  # back in time: every node re-derived, then forward again
                now -= 4 * MIN
                step(now, check_queries=True)
        now += 30 * MIN  # most good nodes age out
        step(now, check_queries=True)


def test_host_batch_ordered_after_async_refresh(gpu):
    """kad_table_refresh_status on a non-blocking torch stream, then at once a host-pointer batch (which runs on the
    table's own streams): the batch must see the refreshed status (kadgpu.h: host batches are ordered after the
    table's last asynchronous refresh), for the one-launch small batch and the chunked pipeline."""
    t = TB.uniform_config(60_000, 13, seed=0x5E9)
    n = t["ids"].shape[0]
    rng = np.random.default_rng(0x5E9)
    targets = TB.adversarial_targets(t, extra=3000)
    MIN = 60 * 10**9
    now = 900 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    side = torch.cuda.Stream(gpu)
    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=True) as T:
        T.set_times(time_ns, reply_ns, expired)
        for dt in (0, 4 * MIN, 3 * MIN, 2 * MIN):  # the first: every node; then ~40 % / 30 % / 20 % age out
            now += dt
            T.refresh_status(now, stream=side.cuda_stream)  # no synchronisation before the host batches
            st = status_at(now)
            for q in (7, 1024, targets.shape[0]):
                idx, cnt = T.rt_closest_host(targets[:q], 8)
                want, wcnt = O.flat_rt_closest(t["ids"], st, t["first"], t["off"], targets[:q], 8, nthreads=8)
                np.testing.assert_array_equal(idx, want, err_msg=f"dt={dt} q={q}")
                np.testing.assert_array_equal(cnt, wcnt)


@pytest.mark.parametrize("nosl", [False, True], ids=["", "nosl"])
@pytest.mark.parametrize("t", [TB.uniform_config(50_000, 12, seed=0x5EA), TB.split_config(30_000, seed=0x5EB)],
                         ids=lambda t: t["name"])
def test_small_refresh_every_line_set(gpu, t, nosl):
    """The small refresh path (at most 2,048 nodes to re-derive: rf_nodes_kernel lists the changed buckets and the
    lines whose windows reach them, the builders rebuild only those) on tables holding every line set (uniform:
    short, 128-byte, 9..16, 17..32 and NodeCache lines; split policy: slot, general 8 / 16 / 32 lines and their
    slot copies), then across the 2,048 boundary to the flag path: `now` passes exactly k deadlines for
    k = 1, 2, 7, 100, 2047, 2048, 2049, 5000; patch_times of a few nodes (heard again, expired: NodeCache ranges)
    refreshed at the same `now`; patch_status of a few nodes, including the first and last buckets' (windows
    clamped at the table's ends). After every step the status bytes equal isGood / isExpired and every query
    equals the oracle."""
    if nosl and t["sorted"]:  # the split table without slot lines: the fused general-line refresh
        pytest.skip("uniform tables have no slot lines")
    n = t["ids"].shape[0]
    off = t["off"]
    rng = np.random.default_rng(n)
    targets = TB.adversarial_targets(t, extra=2500)
    MIN = 60 * 10**9
    now = 700 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    def passed_after(k):  # the `now` at which exactly k more (distinct) deadlines have passed
        d = np.minimum(time_ns + 10 * MIN, reply_ns + 120 * MIN)
        d = np.unique(d[(expired == 0) & (d >= now)])
        return int(d[min(len(d) - 1, k - 1)]) + 1

    rt, nc = (1, 8, 14, 16, 32), (1, 14, 32)
    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                     slot_lines=not nosl) as T:
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        for k in (1, 2, 7, 100, 2047, 2048, 2049, 5000):
            now = passed_after(k)
            T.refresh_status(now)
            torch.cuda.synchronize()
            st = status_at(now)
            np.testing.assert_array_equal(T.export_status(), st, err_msg=f"k={k}")
            if k in (1, 7, 2048, 2049):
                _check(T, t, st, targets, gpu, rt=rt, nc=nc)
        # a few nodes heard again or expired (the NodeCache lines' ranges), refreshed at the same `now`
        sel = np.unique(np.concatenate([rng.choice(n, 40, replace=False), [0, n - 1]])).astype(np.uint32)
        time_ns[sel[::2]] = now
        reply_ns[sel[::2]] = now
        expired[sel[1::2]] = 1
        T.patch_times(sel, time_ns[sel], reply_ns[sel], expired[sel])
        T.refresh_status(now)
        torch.cuda.synchronize()
        st = status_at(now)
        np.testing.assert_array_equal(T.export_status(), st)
        _check(T, t, st, targets, gpu, rt=rt, nc=nc)
        # direct status patches of a few nodes: the first and last buckets' nodes and random ones
        nodes = np.unique(np.concatenate([np.arange(off[0], off[2]), np.arange(off[-3], off[-1]),
                                          rng.choice(n, 60, replace=False)])).astype(np.uint32)
        vals = rng.choice(np.array([0, 1, 1, 2, 3], np.uint8), size=nodes.shape[0])
        st = st.copy()
        st[nodes] = vals
        T.patch_status(nodes, vals)
        np.testing.assert_array_equal(T.export_status(), st)
        assert T.info()["n_good"] == int((st & 1).sum())
        _check(T, t, st, targets, gpu, rt=rt, nc=nc)


@pytest.mark.parametrize("t", [x for x in TB.all_small_tables() if x["ids"].shape[0] >= 50], ids=lambda t: t["name"])
def test_small_refresh_shapes(gpu, t):
    """The one-launch small refresh (rf_nodes_kernel with the count <= 8 lines built in the same block: window lines
    and their short copies, or general lines where no slot lines exist) and its multi-block form on every small
    table shape: `now` passes 1, 3, 40 and 300 deadlines, then nodes are heard again and refreshed at the same
    `now`."""
    n = t["ids"].shape[0]
    rng = np.random.default_rng(n + 17)
    targets = TB.adversarial_targets(t, extra=500)
    MIN = 60 * 10**9
    now = 300 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=t["sorted"]) as T:
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        for k in (1, 3, 40, 300):
            d = np.unique(np.minimum(time_ns + 10 * MIN, reply_ns + 120 * MIN)[expired == 0])
            d = d[d >= now]
            if d.size == 0:
                break
            now = int(d[min(d.size - 1, k - 1)]) + 1
            T.refresh_status(now)
            torch.cuda.synchronize()
            st = status_at(now)
            np.testing.assert_array_equal(T.export_status(), st, err_msg=f"k={k}")
            _check(T, t, st, targets, gpu, rt=(1, 8, 16, 32), nc=(1, 14, 32))
        sel = rng.choice(n, min(n, 30), replace=False).astype(np.uint32)
        time_ns[sel] = now
        reply_ns[sel] = now
        T.patch_times(sel, time_ns[sel], reply_ns[sel], expired[sel])
        T.refresh_status(now)
        torch.cuda.synchronize()
        st = status_at(now)
        np.testing.assert_array_equal(T.export_status(), st)
        _check(T, t, st, targets, gpu, rt=(1, 8, 16, 32), nc=(1, 14, 32))


LINESETS = ("WL", "WS", "WL16", "WL32", "GL", "GL16", "GL32", "SL", "SL16", "NCL", "NCL32", "GCNT", "DIR")


@pytest.mark.parametrize("nosl", [False, True], ids=["", "nosl"])
@pytest.mark.parametrize("t", [TB.uniform_config(40_000, 12, seed=0x5EC), TB.split_config(20_000, seed=0x5ED),
                               TB.uniform_config(6_000, 12, seed=0x5EE)], ids=lambda t: t["name"])
def test_incremental_lines_equal_fresh_build(gpu, t, nosl):
    """Every derived array an incremental refresh maintains (window, short, general and slot lines of every count,
    NodeCache lines, per-bucket good counts, the directory's masks) is bit for bit what a table built from scratch
    on the same status holds: after refreshes passing 1, 2, 5, 9, 30 and 3000 deadlines (the one-launch path whose
    lines a wave builds, the single-block and multi-block lists, the flag path), a patch of times and one of status
    bytes. The U(12) 6,000-node table has sparse buckets (windows of several rounds, deferred lines). nosl: the
    split table without slot lines (KAD_TABLE_NO_SLOT_LINES), so the count <= 8 general lines are rebuilt in the fused
    launch (block 0 publishes the list to the builder blocks)."""
    from opendht_amd import _lib

    if nosl and t["sorted"]:
        pytest.skip("uniform tables have no slot lines")

    n = t["ids"].shape[0]
    rng = np.random.default_rng(n ^ 0x5EC)
    MIN = 60 * 10**9
    now = 800 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    def compare(T, st, what):
        with DeviceTable(t["ids"], st, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                         slot_lines=not nosl) as F:
            for name in LINESETS:
                k = getattr(_lib, f"KAD_LINESET_{name}")
                a, b = T.export_lines(k), F.export_lines(k)
                assert (a is None) == (b is None), f"{what}: {name} present in one table only"
                if a is not None:
                    np.testing.assert_array_equal(a, b, err_msg=f"{what}: {name}")

    with DeviceTable(t["ids"], status_at(now), t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                     slot_lines=not nosl) as T:
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        for k in (1, 2, 5, 9, 30, 3000):
            d = np.unique(np.minimum(time_ns + 10 * MIN, reply_ns + 120 * MIN)[expired == 0])
            d = d[d >= now]
            now = int(d[min(d.size - 1, k - 1)]) + 1
            T.refresh_status(now)
            torch.cuda.synchronize()
            compare(T, status_at(now), f"k={k}")
        sel = rng.choice(n, 8, replace=False).astype(np.uint32)
        time_ns[sel[:4]] = now
        reply_ns[sel[:4]] = now
        expired[sel[4:]] = 1
        T.patch_times(sel, time_ns[sel], reply_ns[sel], expired[sel])
        T.refresh_status(now)
        torch.cuda.synchronize()
        compare(T, status_at(now), "patch_times")
        st = status_at(now).copy()
        nodes = rng.choice(n, 5, replace=False).astype(np.uint32)
        st[nodes] ^= np.uint8(1)
        T.patch_status(nodes, st[nodes])
        compare(T, st, "patch_status")
