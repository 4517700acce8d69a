"""ID-range sharding of a swarm-scale routing table across the GPUs of one node.

Design: "owner routing + halo". Buckets are contiguous ID ranges and a query only reads the
window W(R) of adjacent buckets around its target's bucket (routing_table.cpp:89-104), so the
table shards by the top log2(n_shards) ID bits with no data-path collective:

  * shard s owns buckets [lo_s, hi_s) of the global U(depth) table and every target whose top
    bits are s;
  * it additionally holds H_L / H_R halo buckets from its neighbours, where H is the largest
    window overhang of any owned bucket (computed exactly from the good counts at build time
    for the largest supported count), so each owned query is answered locally and bit-exactly
    as the whole table would answer it;
  * node indices are global (index_base = nodes in buckets below the shard's first bucket).

The bench runs weak scaling (each GPU: one 1/8 shard of the 100M-node table and a fixed batch
of queries targeted into it). A serving front end that receives arbitrary targets needs one
exchange step -- route targets to owners and results back -- see ``route_queries`` (an
all-to-all, the only collective on this path).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import synth as S
from .metrics import good_counts as _good_counts
from .metrics import window_radii

SEED_SWARM = 0x0D470100


@dataclass
class ShardSpec:
    """A global U(depth) table cut into n_shards ID ranges. recipe_n > 0: the table is SURVEY.md §8d's recipe of
    recipe_n nodes (std::mt19937_64 IDs and status, synth.recipe_range: any shard regenerated from the seeds alone,
    in one pass over all recipe_n draws); recipe_n = 0: counter-based Poisson(mean_per_bucket) buckets (any bucket
    range generated on its own; the small multi-shard tests)."""
    n_shards: int = 8
    depth: int = 24
    mean_per_bucket: float = 100e6 / 2**24
    seed: int = SEED_SWARM
    good_pct: int = 80
    expired_pct: int = 10
    k_max: int = 32
    recipe_n: int = 0
    _below: dict = field(default_factory=dict, repr=False, compare=False)  # nodes_below cache (recipe passes)

    @property
    def shard_bits(self) -> int:
        b = self.n_shards.bit_length() - 1
        if 1 << b != self.n_shards:
            raise ValueError("n_shards must be a power of two")
        return b

    @property
    def n_buckets(self) -> int:
        return 1 << self.depth

    def owned(self, s: int) -> tuple[int, int]:
        per = self.n_buckets // self.n_shards
        return s * per, (s + 1) * per

    def targets_for(self, s: int, q: int, seed: int = S.SEED_TARGETS) -> np.ndarray:
        """q uniform random targets owned by shard s (top shard_bits bits = s)."""
        return S.random_targets(q, seed=seed ^ (s * 0x9E37), prefix_bits=self.shard_bits, prefix=s)

    def bucket_range(self, lo: int, hi: int):
        """(ids sorted, status, offsets) of global buckets [lo, hi)."""
        return self.bucket_range_below(lo, hi)[:3]

    def bucket_range_below(self, lo: int, hi: int):
        """(ids sorted, status, offsets, global index of the range's first node) of global buckets [lo, hi)."""
        if self.recipe_n:
            return S.recipe_range(self.recipe_n, self.depth, lo, hi, self.good_pct, self.expired_pct)
        ids, st, off = S.uniform_shard(self.seed, self.depth, lo, hi, self.mean_per_bucket, self.good_pct,
                                       self.expired_pct)
        return ids, st, off, self.nodes_below(lo)

    def nodes_below(self, b: int) -> int:
        """Global index of the first node of bucket b."""
        if b <= 0:
            return 0
        if self.recipe_n:
            if b >= self.n_buckets:
                return self.recipe_n
            if b not in self._below:  # one pass over all recipe_n draws: cached per spec
                import ctypes as C

                from ._lib import check, lib

                n, below = C.c_uint32(), C.c_uint64()
                check(lib().kad_synth_recipe_range(S.SEED_IDS, S.SEED_STATUS, self.recipe_n, self.depth, b,
                                                   self.n_buckets, self.good_pct, self.expired_pct, 0, C.byref(n),
                                                   C.byref(below), None, None, None), "kad_synth_recipe_range")
                self._below[b] = int(below.value)
            return self._below[b]
        import ctypes as C

        from ._lib import check, lib

        n = C.c_uint32()
        check(lib().kad_synth_uniform_shard(self.seed, self.depth, 0, b, self.mean_per_bucket, self.good_pct,
                                            self.expired_pct, C.byref(n), None, None, None),
              "kad_synth_uniform_shard")
        return n.value


def config3_spec(n_shards: int = 8) -> ShardSpec:
    """BASELINE config 3: SURVEY.md §8d's 100M-node U(24) table (mt19937_64 recipe) in n_shards ID-range shards."""
    return ShardSpec(n_shards=n_shards, depth=24, recipe_n=100_000_000)


def halo_widths_from(good: np.ndarray, a: int, lo: int, hi: int, n_buckets: int, count: int):
    """Exact halo (H_L, H_R) for owned buckets [lo, hi), given good counts of global buckets
    [a, a + len(good)). Returns None if some owned window reaches a non-global edge of the probe
    range (the probe must grow)."""
    e = a + good.shape[0]
    R = window_radii(good, count)
    b = np.arange(lo, hi, dtype=np.int64)
    Rb = R[lo - a:hi - a]
    wl = np.maximum(a, b - 1 - Rb)
    wh = np.minimum(e - 1, b + Rb)
    if (a > 0 and (wl <= a).any()) or (e < n_buckets and (wh >= e - 1).any()):
        return None
    return int(max(0, (lo - wl).max())), int(max(0, (wh - (hi - 1)).max()))


@dataclass
class Shard:
    spec: ShardSpec
    s: int
    lo: int          # first owned global bucket
    hi: int          # one past the last owned bucket
    b0: int          # first held bucket (lo - H_L)
    b1: int          # one past the last held bucket (hi + H_R)
    index_base: int  # global index of the shard table's node 0
    ids: np.ndarray = field(repr=False)
    status: np.ndarray = field(repr=False)
    first: np.ndarray = field(repr=False)
    off: np.ndarray = field(repr=False)


def build_shard(spec: ShardSpec, s: int, probe: int = 64) -> Shard:
    """Generate shard s of the global table with the exact halo for counts <= spec.k_max."""
    lo, hi = spec.owned(s)
    B = spec.n_buckets
    while True:
        a, e = max(0, lo - probe), min(B, hi + probe)
        ids, st, off, below_a = spec.bucket_range_below(a, e)
        hw = halo_widths_from(_good_counts(st, off), a, lo, hi, B, spec.k_max)
        if hw is not None:
            break
        probe *= 4
    HL, HR = hw
    b0, b1 = max(0, lo - HL), min(B, hi + HR)
    n0, n1 = off[b0 - a], off[b1 - a]
    ids = np.ascontiguousarray(ids[n0:n1])
    st = np.ascontiguousarray(st[n0:n1])
    off = np.ascontiguousarray(off[b0 - a:b1 - a + 1] - n0).astype(np.uint32)
    first = S.bucket_firsts(spec.depth, b0, b1)
    return Shard(spec, s, lo, hi, b0, b1, below_a + int(n0), ids, st, first, off)


class HaloError(RuntimeError):
    """A status change made some owned window reach past the shard's halo: the shard can no longer answer
    every owned query as the whole table would. Rebuild the shard (build_shard) with the new status."""


def halo_ok(sh: Shard, status) -> bool:
    """Whether the shard's held buckets [b0, b1) still contain every owned window W(R) for counts <= k_max
    under `status` (the shard's node statuses). The held good counts get a sentinel bucket of k_max good
    nodes on each side that is not a global edge: a window stays inside [b0, b1) exactly when its local
    rounds (routing_table.cpp:89-104) never reach a sentinel."""
    g = _good_counts(np.asarray(status), sh.off).astype(np.int64)
    left, right = sh.b0 > 0, sh.b1 < sh.spec.n_buckets
    k = sh.spec.k_max
    ext = np.concatenate([[k] if left else [], g, [k] if right else []]).astype(np.int64)
    R = window_radii(ext, k)
    b = np.arange(sh.lo - sh.b0, sh.hi - sh.b0) + (1 if left else 0)
    wl, wh = b - 1 - R[b], b + R[b]
    return not ((left and (wl <= 0).any()) or (right and (wh >= ext.shape[0] - 1).any()))


class ShardTable:
    """A shard's DeviceTable whose status changes are checked against the halo it was built with: the
    halo width comes from the good counts at build time, so a refresh that turns enough nodes bad next to
    a shard edge would let a window run past the held buckets and the shard would answer with its local
    edge as the table edge. Every status change here re-checks the halo and raises HaloError instead."""

    def __init__(self, sh: Shard, device: int = 0):
        from .table import DeviceTable

        self.shard = sh
        self.table = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=device, index_base=sh.index_base,
                                 sorted=True)

    def _check(self):
        st = self.table.export_status()
        if not halo_ok(self.shard, st):
            raise HaloError(f"shard {self.shard.s}: an owned window now reaches past the halo "
                            f"[{self.shard.b0}, {self.shard.b1}); rebuild the shard")

    def update_status(self, status):
        self.table.update_status(status)
        self._check()

    def patch_status(self, nodes, status):
        self.table.patch_status(nodes, status)
        self._check()

    def refresh_status(self, now_ns: int, stream=None):
        import torch

        self.table.refresh_status(now_ns, stream=stream)
        torch.cuda.synchronize(self.table.device)
        self._check()

    def __getattr__(self, name):  # queries and the rest: the DeviceTable's
        return getattr(self.table, name)

    def close(self):
        self.table.close()


def route_queries(targets, spec: ShardSpec, group=None):
    """Serving-mode exchange: send each target to its owner shard (its top shard_bits bits; one rank
    per shard) with all_to_all_single. `targets` is a (q, 20) uint8 tensor on the backend's device
    (cuda for RCCL, cpu for gloo); everything stays on that device except the split sizes.
    Returns (local_targets, ctx) for ``return_results``."""
    import torch
    import torch.distributed as dist

    if isinstance(targets, np.ndarray):
        targets = torch.from_numpy(np.ascontiguousarray(targets, dtype=np.uint8))
    world = dist.get_world_size(group)
    if spec.shard_bits:
        owner = (targets[:, 0].to(torch.int64) >> (8 - spec.shard_bits)) % world
    else:
        owner = torch.zeros(targets.shape[0], dtype=torch.int64, device=targets.device)
    order = torch.argsort(owner, stable=True)
    send_counts = torch.bincount(owner, minlength=world)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    recv = targets.new_empty((sum(rc), 20))
    dist.all_to_all_single(recv, targets[order].contiguous(), output_split_sizes=rc, input_split_sizes=sc, group=group)
    return recv, (rc, sc, order, targets.shape[0])


def return_results(local_idx, local_cnt, ctx, group=None):
    """Inverse of route_queries for (q_local, k) int32 results and (q_local,) counts (tensors on the
    backend's device, or numpy): each query's answer back at its position on its sender."""
    import torch
    import torch.distributed as dist

    rc, sc, order, q = ctx
    if isinstance(local_idx, np.ndarray):
        local_idx = torch.from_numpy(np.ascontiguousarray(local_idx).view(np.int32))
        local_cnt = torch.from_numpy(np.ascontiguousarray(local_cnt))
    k = local_idx.shape[1]
    back_idx = local_idx.new_empty((sum(sc), k))
    back_cnt = torch.empty((sum(sc),), dtype=torch.int32, device=local_idx.device)
    dist.all_to_all_single(back_idx, local_idx.contiguous(), output_split_sizes=sc, input_split_sizes=rc, group=group)
    dist.all_to_all_single(back_cnt, local_cnt.to(torch.int32).contiguous(), output_split_sizes=sc,
                           input_split_sizes=rc, group=group)
    out_idx = local_idx.new_empty((q, k))
    out_cnt = torch.empty((q,), dtype=torch.uint8, device=local_idx.device)
    out_idx[order] = back_idx
    out_cnt[order] = back_cnt.to(torch.uint8)
    return out_idx, out_cnt
