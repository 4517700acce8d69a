"""Shared cases of the small-refresh limit tests (tests/test_refresh_limits.py and the delayed-block-0 worker
tests/rf_delay_worker.py): node times built so that one refresh passes exactly the chosen nodes' isGood deadlines
(node.cpp:34-40: good while now <= min(time + 10 min, reply_time + 120 min)), and the check that every derived
array then equals a fresh build on the same status."""
from __future__ import annotations

import numpy as np

MIN = 60 * 10**9
LINESETS = ("WL", "WS", "WL16", "WL32", "GL", "GL16", "GL32", "SL", "SL16", "NCL", "NCL32", "GCNT", "DIR")


def runs_layout(B: int, runs):
    """Buckets of the given runs [(first, m)]: m consecutive buckets each. The host's line runs of the fused
    refresh follow them: a run of buckets [f, f + m) lists lines [f - 2, f + m + 2] and the bucket offsets
    [f - 5, f + m + 5] (clamped to [0, B]), so an interior run takes m + 11 offsets and one at either end m + 6."""
    out = []
    for f, m in runs:
        assert 0 <= f and f + m <= B
        out.extend(range(f, f + m))
    return np.array(out, np.int64)


def hoff_entries(B: int, runs) -> int:
    tot = 0
    for f, m in runs:
        lo, hi = max(0, f - 2), min(B - 1, f + m - 1 + 3)
        tot += min(B, hi + 3) + 1 - max(0, lo - 3)
    return tot


def times_for(t, buckets, nnodes, now0, seed):
    """(time_ns, reply_ns, expired, chosen): every node heard recently enough that no deadline falls in
    (now0, now0 + 10^4]; `nnodes` chosen good nodes, at least one in each of `buckets`, whose deadlines are
    now0 + 1 .. now0 + nnodes (distinct). A refresh at now0, then one at now0 + 10^4 passes exactly those."""
    rng = np.random.default_rng(seed)
    off = t["off"]
    n = t["ids"].shape[0]
    time_ns = now0 - rng.integers(0, 5 * MIN, n)     # deadlines >= now0 + 5 min
    reply_ns = np.full(n, now0, np.int64)
    expired = np.zeros(n, np.uint8)
    chosen = []
    for b in buckets:
        if off[b + 1] > off[b]:
            chosen.append(int(rng.integers(off[b], off[b + 1])))
    pool = np.setdiff1d(np.concatenate([np.arange(off[b], off[b + 1]) for b in buckets]), chosen)
    extra = nnodes - len(chosen)
    assert extra >= 0, (len(chosen), nnodes)
    chosen.extend(rng.choice(pool, extra, replace=False).tolist())
    chosen = np.array(sorted(chosen), np.int64)
    assert chosen.size == nnodes and np.unique(chosen).size == nnodes
    time_ns[chosen] = now0 - 10 * MIN + 1 + rng.permutation(nnodes)
    return time_ns, reply_ns, expired, chosen


def status_at(time_ns, reply_ns, expired, tnow):
    good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
    return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)


def compare_fresh(DeviceTable, _lib, T, t, st, what, slot_lines=True):
    """Every derived array of T equals a table built from scratch on status st."""
    with DeviceTable(t["ids"], st, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                     slot_lines=slot_lines) as F:
        for name in LINESETS:
            k = getattr(_lib, f"KAD_LINESET_{name}")
            a, b = T.export_lines(k), F.export_lines(k)
            assert (a is None) == (b is None), f"{what}: {name} present in one table only"
            if a is not None:
                np.testing.assert_array_equal(a, b, err_msg=f"{what}: {name}")
