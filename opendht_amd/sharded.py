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
    n_shards: int = 8
    depth: int = 24
    mean_per_bucket: float = 100e6 / 2**24
    seed: int = SEED_SWARM
    good_pct: int = 80
    expired_pct: int = 10
    k_max: int = 32

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
        return S.uniform_shard(self.seed, self.depth, lo, hi, self.mean_per_bucket, self.good_pct,
                               self.expired_pct)

    def nodes_below(self, b: int) -> int:
        """Global index of the first node of bucket b."""
        if b <= 0:
            return 0
        import ctypes as C

        from ._lib import check, lib

        n = C.c_uint32()
        check(lib().kad_synth_uniform_shard(self.seed, self.depth, 0, b, self.mean_per_bucket, self.good_pct,
                                            self.expired_pct, C.byref(n), None, None, None),
              "kad_synth_uniform_shard")
        return n.value


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
        ids, st, off = spec.bucket_range(a, e)
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
    return Shard(spec, s, lo, hi, b0, b1, spec.nodes_below(b0), ids, st, first, off)


def route_queries(targets, spec: ShardSpec, group=None):
    """Serving-mode exchange: send each target to its owner shard (top bits), one rank per shard,
    via torch.distributed all_to_all; returns (local_targets, recv_splits, send_order) so the
    answers can be sent back with ``return_results``. Works on gloo (CPU) and RCCL."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    tnp = targets.cpu().numpy() if hasattr(targets, "cpu") else targets
    owner = (tnp[:, 0].astype(np.int64) >> (8 - spec.shard_bits)) if spec.shard_bits else np.zeros(len(tnp), int)
    owner = owner % world
    order = np.argsort(owner, kind="stable")
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    sc = torch.tensor(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc, group=group)
    send = torch.from_numpy(np.ascontiguousarray(tnp[order]))
    recv = torch.empty((int(rc.sum()), 20), dtype=torch.uint8)
    dist.all_to_all_single(recv, send, output_split_sizes=rc.tolist(), input_split_sizes=sc.tolist(), group=group)
    return recv, rc.tolist(), sc.tolist(), order


def return_results(local_idx, local_cnt, recv_splits, send_splits, order, group=None):
    """Inverse of route_queries for (q_local, k) uint32 results and (q_local,) counts."""
    import torch
    import torch.distributed as dist

    k = local_idx.shape[1]
    idx = torch.from_numpy(np.ascontiguousarray(local_idx).view(np.int32))
    cnt = torch.from_numpy(np.ascontiguousarray(local_cnt).astype(np.int32))
    back_idx = torch.empty((sum(send_splits), k), dtype=torch.int32)
    back_cnt = torch.empty((sum(send_splits),), dtype=torch.int32)
    dist.all_to_all_single(back_idx, idx, output_split_sizes=send_splits, input_split_sizes=recv_splits, group=group)
    dist.all_to_all_single(back_cnt, cnt, output_split_sizes=send_splits, input_split_sizes=recv_splits, group=group)
    out_idx = np.empty((len(order), k), np.uint32)
    out_cnt = np.empty((len(order),), np.uint8)
    out_idx[order] = back_idx.numpy().view(np.uint32)
    out_cnt[order] = back_cnt.numpy().astype(np.uint8)
    return out_idx, out_cnt
