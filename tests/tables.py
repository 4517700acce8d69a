"""Test tables: the BASELINE configs at test sizes plus the adversarial shapes of SURVEY.md §4
(empty buckets, all-bad tables, targets equal to node IDs, first/last bucket targets, top-64
ties, duplicate IDs, tiny tables)."""
from __future__ import annotations

import numpy as np

from opendht_amd import synth as S


def table(ids, status, first, off, sorted_=False, name=""):
    return dict(ids=np.ascontiguousarray(ids, np.uint8), status=np.ascontiguousarray(status, np.uint8),
                first=None if first is None else np.ascontiguousarray(first, np.uint8),
                off=None if off is None else np.ascontiguousarray(off, np.uint32), sorted=sorted_, name=name)


def split_config(n=10_000, seed=S.SEED_IDS, good=80, expired=10, cap=8):
    """Config 1 shape S: reference split policy over mt19937_64 IDs."""
    ids = S.random_ids(n, seed)
    st = S.random_status(n, S.SEED_STATUS ^ seed, good, expired)
    perm, first, off = S.split_table(ids, cap)
    return table(ids[perm], st[perm], first, off, name=f"S{n}")


def uniform_config(n=10_000, depth=10, seed=S.SEED_IDS, good=80, expired=10):
    """Config 1 shape U(d): uniform depth over sorted IDs (also a valid NodeCache table)."""
    ids, _ = S.sort_ids(S.random_ids(n, seed))
    st = S.random_status(n, S.SEED_STATUS ^ seed, good, expired)
    first, off = S.uniform_buckets(ids, depth)
    return table(ids, st, first, off, sorted_=True, name=f"U{depth}_{n}")


def tiny_tables():
    out = []
    # empty routing table (no buckets, no nodes)
    out.append(table(np.zeros((0, 20), np.uint8), np.zeros(0, np.uint8), np.zeros((0, 20), np.uint8),
                     np.zeros(1, np.uint32), sorted_=True, name="empty"))
    # one bucket, zero nodes (a fresh Dht table: Bucket{af} with first = zeroes)
    out.append(table(np.zeros((0, 20), np.uint8), np.zeros(0, np.uint8), np.zeros((1, 20), np.uint8),
                     np.zeros(2, np.uint32), sorted_=True, name="one_empty_bucket"))
    for n in (1, 3, 50, 257):
        t = split_config(n, seed=0x5EED + n)
        t["name"] = f"S{n}"
        out.append(t)
    return out


def all_bad_table(n=2000):
    t = uniform_config(n, 6, seed=0xBAD)
    rng = np.random.default_rng(1)
    t["status"] = rng.choice(np.array([0, 2], np.uint8), size=n)  # dubious or expired only
    t["name"] = "all_bad"
    return t


def sparse_good_table(n=4000):
    """Mostly-bad table with empty buckets: windows grow over many rounds."""
    t = uniform_config(n, 11, seed=0x5A5E)
    rng = np.random.default_rng(2)
    t["status"] = np.where(rng.random(n) < 0.03, 1, 2).astype(np.uint8)
    t["name"] = "sparse_good"
    return t


def tie_table(groups=64, per=6, seed=7, tag=""):
    """Many nodes share their top 64 bits (exercises the exact 160-bit tie path), plus one
    bucket holding duplicate IDs (RoutingTable order = index order). per > 32 puts more nodes in one
    NodeCache radix slot than the window kernel loads (its binary-search path)."""
    rng = np.random.default_rng(seed)
    heads = rng.integers(0, 256, size=(groups, 8), dtype=np.uint8)
    ids = np.empty((groups * per, 20), np.uint8)
    for g in range(groups):
        ids[g * per:(g + 1) * per, :8] = heads[g]
        ids[g * per:(g + 1) * per, 8:] = rng.integers(0, 256, size=(per, 12), dtype=np.uint8)
        ids[g * per + 1, 8:] = 0  # some tails differ only in the last bytes
        ids[g * per + 2, 8:] = 0
        ids[g * per + 2, 19] = 1
    ids, _ = S.sort_ids(ids)
    first, off = S.uniform_buckets(ids, 4)
    st = np.where(rng.random(ids.shape[0]) < 0.85, 1, 0).astype(np.uint8)
    srt = table(ids, st, first, off, sorted_=True, name="ties" + tag)
    # duplicate IDs inside a bucket (unsorted RoutingTable snapshot)
    dup = ids.copy()
    dup[5] = dup[3]
    dup[6] = dup[3]
    st2 = st.copy()
    st2[3:7] = 1
    return [srt, table(dup, st2, first, off, sorted_=False, name="dups" + tag)]


def offset_first_table(n=3000):
    """First bucket does not start at zeroes (targets below it clamp to bucket 0)."""
    ids, _ = S.sort_ids(S.random_ids(n, 0xF1257))
    lo, hi = 300, 700  # buckets 300..699 of U(10)
    hi_ids = ids[:, :8].copy().view(">u8").reshape(-1)
    keep = (hi_ids >= np.uint64(lo << 54)) & (hi_ids < np.uint64(hi << 54))
    ids = np.ascontiguousarray(ids[keep])
    first, off = S.uniform_buckets(ids, 10, lo, hi)
    st = S.random_status(ids.shape[0], 99)
    return table(ids, st, first, off, sorted_=True, name="offset_first")


def adversarial_targets(t, extra=256, seed=3):
    """Targets equal to node IDs, bucket firsts, first/last bucket, 00..0, FF..F, random."""
    rng = np.random.default_rng(seed)
    parts = [np.zeros((1, 20), np.uint8), np.full((1, 20), 255, np.uint8)]
    ids, first = t["ids"], t["first"]
    if ids.shape[0]:
        parts.append(ids[rng.integers(0, ids.shape[0], size=min(64, ids.shape[0]))])
        parts.append(ids[:1])
        parts.append(ids[-1:])
    if first is not None and first.shape[0]:
        parts.append(first[rng.integers(0, first.shape[0], size=min(32, first.shape[0]))])
        parts.append(first[-1:])
        # one below each sampled bucket first (…FF tail)
        f = first[rng.integers(0, first.shape[0], size=min(16, first.shape[0]))].copy()
        parts.append(_minus_one(f))
    parts.append(rng.integers(0, 256, size=(extra, 20), dtype=np.uint8))
    return np.ascontiguousarray(np.concatenate(parts), np.uint8)


def _minus_one(ids):
    out = ids.copy()
    for r in range(out.shape[0]):
        x = int.from_bytes(out[r].tobytes(), "big")
        x = (x - 1) % (1 << 160)
        out[r] = np.frombuffer(x.to_bytes(20, "big"), np.uint8)
    return out


def all_small_tables():
    ts = tiny_tables()
    ts.append(split_config(10_000))
    ts.append(uniform_config(10_000, 10))
    ts.append(all_bad_table())
    ts.append(sparse_good_table())
    ts.extend(tie_table())
    ts.extend(tie_table(groups=24, per=48, seed=8, tag="48"))
    ts.append(offset_first_table())
    return ts
