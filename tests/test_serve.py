"""Resident query service (kad_table_serve): the single-request path of the boundary
(RoutingTableMirror::findClosestNodes -> kad_rt_closest_batch_host, the per-request calls of
dht.cpp:3196-3217 and NodeCache::getCachedNodes of dht.cpp:1650) answered by a workgroup that stays on
the GPU. Bit-exact against the oracle on every small table shape, across idle exits and relaunches,
across table mutations (which end the service first), beside a device batch on another stream."""
import time

import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd._lib import KAD_OP_INSERT, KAD_OP_REMOVE, KAD_SERVE_MAX_Q, KadError

pytestmark = pytest.mark.gpu


def make(t, gpu):
    return DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=t["sorted"])


def served(T, targets, k, nc=False, q=KAD_SERVE_MAX_Q):
    """Host batches of at most q queries (the service's request size), concatenated."""
    f = T.nc_closest_host if nc else T.rt_closest_host
    parts = [f(targets[i:i + q], k) for i in range(0, targets.shape[0], q)]
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts])


def check(T, t, targets, counts, nc=False, q=KAD_SERVE_MAX_Q, tag=""):
    for k in counts:
        idx, cnt = served(T, targets, k, nc, q)
        if nc:
            want, wcnt = O.flat_nc_closest(t["ids"], t["status"], targets, k)
        else:
            want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k)
        np.testing.assert_array_equal(cnt, wcnt, err_msg=f"{t['name']}{tag} {'nc' if nc else 'rt'} k={k} counts")
        np.testing.assert_array_equal(idx, want, err_msg=f"{t['name']}{tag} {'nc' if nc else 'rt'} k={k} indices")


@pytest.mark.parametrize("prepared", [False, True], ids=["lazy", "prepared"])
@pytest.mark.parametrize("t", TB.all_small_tables(), ids=lambda t: t["name"])
def test_serve_parity(gpu, t, prepared):
    """The service runs the launch path's kernel bodies for the line sets the table has when it starts (lazy: the
    count <= 8 lines only; prepared: every set), the wave paths beyond."""
    targets = TB.adversarial_targets(t, extra=160)
    with make(t, gpu) as T:
        if prepared:
            T.prepare()
        T.serve(20_000)
        check(T, t, targets, (0, 1, 7, 8, 14, 16, 17, 32, 33, 64))
        check(T, t, targets[:40], (8, 14), q=1, tag=" q=1")
        if t["sorted"]:
            check(T, t, targets, (0, 1, 8, 14, 16, 32, 64), nc=True)
            check(T, t, targets[:40], (14,), nc=True, q=1, tag=" q=1")


def test_serve_idle_exit_and_relaunch(gpu):
    """A launch that went idle has ended; the next request launches it again (same answers)."""
    t = TB.split_config(3000, seed=0x5E1)
    targets = TB.adversarial_targets(t, extra=64)
    with make(t, gpu) as T:
        T.serve(200)  # 0.2 ms
        for rep in range(5):
            check(T, t, targets, (8,), tag=f" rep {rep}")
            time.sleep(0.01)  # 50 idle periods: the launch has ended
        st = T.serve_stats()
        assert st["idle_us"] == 200 and st["launches"] >= 5, st  # one launch per rep (the first by serve())
        assert st["requests"] == 5 * -(-targets.shape[0] // 64), st
        T.serve(0)  # off: the launch path answers
        check(T, t, targets, (8, 14), tag=" off")
        T.serve(5_000)
        check(T, t, targets, (8,), tag=" on again")


def test_serve_follows_mutations(gpu):
    """Status patches, refreshes at a moving `now` (async, another stream), the incremental mirror: every
    answer after a change is the oracle's on the changed table."""
    t = TB.uniform_config(4000, 9, seed=0x5E2)
    n = t["ids"].shape[0]
    targets = TB.adversarial_targets(t, extra=128)
    rng = np.random.default_rng(5)
    with make(t, gpu) as T:
        T.serve(50_000)
        check(T, t, targets, (8, 32))
        st = t["status"].copy()
        nodes = rng.choice(n, 300, replace=False).astype(np.uint32)
        st[nodes] = rng.integers(0, 3, nodes.shape[0]).astype(np.uint8)
        T.patch_status(nodes, st[nodes])
        t = dict(t, status=st)
        check(T, t, targets, (8, 32), tag=" patched")
        check(T, t, targets, (14,), nc=True, tag=" patched")
        # node times on the device, `now` moving across the 10-minute edge on a side stream
        now = 10**15
        age = rng.integers(0, 12 * 60 * 10**9, n)
        tm, rp = now - age, np.full(n, now, np.int64)
        ex = np.zeros(n, np.uint8)
        T.set_times(tm, rp, ex)
        side = torch.cuda.Stream(device=gpu)
        for dt in (0, 30, 90, 200):
            now2 = now + dt * 10**9
            T.refresh_status(now2, stream=side)
            good = (tm >= now2 - 600 * 10**9) & (rp >= now2 - 7200 * 10**9)
            t = dict(t, status=good.astype(np.uint8))
            check(T, t, targets, (8, 16), tag=f" now+{dt}s")
        torch.cuda.synchronize()
        # the incremental mirror: removals and insertions (new arrays: the service must not read the old ones)
        new_ids = S.random_ids(50, 0x5E3)
        ops = np.array([(KAD_OP_REMOVE, int(a), 0) for a in rng.choice(n, 40, replace=False)] +
                       [(KAD_OP_INSERT, j, 0) for j in range(50)], np.uint32)
        T.apply(ops, new_ids, np.ones(50, np.uint8))
        ids, st2, first, off = T.export()
        t = dict(t, ids=ids, status=st2, first=first, off=off, sorted=False)
        check(T, t, targets, (8, 14, 32), tag=" applied")


def test_serve_beside_device_batch(gpu):
    """A large device batch on a torch stream and served requests at the same time: both exact."""
    t = TB.uniform_config(200_000, 15, seed=0x5E4)
    big = S.random_targets(1 << 18, seed=0x5E5)
    small = TB.adversarial_targets(t, extra=64)
    with make(t, gpu) as T:
        T.serve(20_000)
        s = torch.cuda.Stream(device=gpu)
        with torch.cuda.stream(s):
            tg = torch.from_numpy(big).to(gpu)
            idx, cnt = T.rt_closest(tg, 8, stream=s)
        check(T, t, small, (8, 14))
        s.synchronize()
        want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], big, 8, nthreads=8)
        np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt)
        np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want)


def test_serve_limits_and_close(gpu):
    """Requests above the service's size take the launch path; closing a serving table ends the service."""
    t = TB.split_config(2000, seed=0x5E6)
    targets = TB.adversarial_targets(t, extra=300)
    T = make(t, gpu)
    T.serve(20_000)
    check(T, t, targets, (8, 65, 100), q=200, tag=" large")  # q > 64 or count > 64: the launch path
    check(T, t, targets, (8,), tag=" small")
    with pytest.raises(KadError):
        T.serve(2_000_000)  # idle above the limit
    check(T, t, targets[:64], (8,), tag=" after refused serve")
    T.close()  # ends the running launch, then frees the table


def test_serve_refresh_latency_many_streams(gpu):
    """A refresh that flips many nodes, then a served request, with more streams alive than the process has
    hardware queues (GPU_MAX_HW_QUEUES = 4): the refresh ends the resident launch first, so neither the refresh nor
    the request waits behind it for its idle period (50 ms here); the answers follow the refreshed table."""
    t = TB.uniform_config(20_000, 11, seed=0x5E7)
    n = t["ids"].shape[0]
    targets = TB.adversarial_targets(t, extra=32)[:64]
    rng = np.random.default_rng(7)
    streams = [torch.cuda.Stream(device=gpu) for _ in range(8)]
    for s in streams:  # every stream used once, so each holds a hardware queue slot
        with torch.cuda.stream(s):
            torch.ones(1024, device=gpu).sum()
    torch.cuda.synchronize()
    with make(t, gpu) as T:
        now = 10**15
        age = rng.integers(0, 20 * 60 * 10**9, n)
        tm, rp, ex = now - age, np.full(n, now, np.int64), np.zeros(n, np.uint8)
        T.set_times(tm, rp, ex)
        T.refresh_status(now)
        good = (tm >= now - 600 * 10**9) & (rp >= now - 7200 * 10**9)
        t = dict(t, status=good.astype(np.uint8))
        T.serve(50_000)
        check(T, t, targets, (8,))
        worst = 0.0
        for dt in (60, 120, 300):  # seconds of ageing: thousands of nodes flip each time
            now2 = now + dt * 10**9
            t0 = time.perf_counter()
            T.refresh_status(now2)
            good = (tm >= now2 - 600 * 10**9) & (rp >= now2 - 7200 * 10**9)
            t = dict(t, status=good.astype(np.uint8))
            idx, cnt = served(T, targets, 8)
            worst = max(worst, time.perf_counter() - t0)
            want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, 8)
            np.testing.assert_array_equal(cnt, wcnt, err_msg=f"now+{dt}s counts")
            np.testing.assert_array_equal(idx, want, err_msg=f"now+{dt}s indices")
        assert worst < 0.030, f"refresh + served request took {worst * 1e3:.1f} ms (idle period 50 ms)"
