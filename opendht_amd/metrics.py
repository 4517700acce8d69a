"""Algorithmic byte counts for the roofline, computed exactly on the host.

RoutingTable query:  20 (target) + sum over the visited window W(R) of (8 + n_b + 20 g_b)
                     + 4 count (output indices)
                     -- a bucket extent entry, one status byte per node and one 20-byte ID per
                     good node of every visited bucket: what any correct implementation must read.
NodeCache query:     20 + 8 + 21 per walk step + 4 count.
"""
from __future__ import annotations

import numpy as np


def good_counts(status: np.ndarray, off: np.ndarray) -> np.ndarray:
    c = np.concatenate([[0], np.cumsum(status & 1, dtype=np.int64)])
    return (c[off[1:]] - c[off[:-1]]).astype(np.int64)


def window_radii(good: np.ndarray, count: int) -> np.ndarray:
    """R(b) for every bucket b: the least round r whose window [max(0,b-1-r), min(B-1,b+r)]
    holds >= count good nodes or is the whole table (routing_table.cpp:89-104), vectorised."""
    B = good.shape[0]
    c = np.concatenate([[0], np.cumsum(good, dtype=np.int64)])
    b = np.arange(B, dtype=np.int64)
    R = np.full(B, -1, np.int64)
    r = 0
    while (R < 0).any():
        lo = np.maximum(0, b - 1 - r)
        hi = np.minimum(B - 1, b + r)
        done = (R < 0) & (((c[hi + 1] - c[lo]) >= count) | ((lo == 0) & (hi == B - 1)))
        R[done] = r
        r += 1
    return R


def rt_algorithmic_bytes(status: np.ndarray, off: np.ndarray, target_buckets: np.ndarray, count: int):
    """Total algorithmic bytes of a batch of RoutingTable queries whose targets fall in buckets
    `target_buckets` (RoutingTable::findBucket). Returns (bytes, mean buckets, mean nodes, mean good)."""
    off = np.asarray(off, dtype=np.int64)
    B = off.shape[0] - 1
    q = target_buckets.shape[0]
    if B == 0 or count == 0 or q == 0:
        return 20 * q + 4 * count * q, 0.0, 0.0, 0.0
    g = good_counts(status, off)
    n = np.diff(off)
    R = window_radii(g, count)
    b = target_buckets.astype(np.int64)
    lo = np.maximum(0, b - 1 - R[b])
    hi = np.minimum(B - 1, b + R[b])
    w = np.concatenate([[0], np.cumsum(8 + n + 20 * g, dtype=np.int64)])
    cn = np.concatenate([[0], np.cumsum(n, dtype=np.int64)])
    cg = np.concatenate([[0], np.cumsum(g, dtype=np.int64)])
    tot = int((w[hi + 1] - w[lo]).sum()) + (20 + 4 * count) * q
    return tot, float((hi - lo + 1).mean()), float((cn[hi + 1] - cn[lo]).mean()), float((cg[hi + 1] - cg[lo]).mean())
