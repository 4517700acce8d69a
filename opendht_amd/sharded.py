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


class OwnerRoute:
    """Device-only owner routing of one step shape (q targets per rank, count, world ranks): the serving front end's
    exchange without a host read per batch and without sorting.

      pack    kad_route_pack: every target into the fixed-size send block of its owner (rank (byte 0 >> (8 -
              shard_bits)) % world), its place recorded per query
      send    all_to_all_single of the target blocks (equal splits; RCCL over xGMI, gloo through the host)
      answer  the owner's table answers every record of the received blocks (padding records included: their rows
              are never read back)
      return  all_to_all_single of the row and count blocks, back to the senders
      unpack  kad_route_unpack: each query's row to its original position
    packed (the default for counts 4, 8, ..., 32): the rows go back packed (a base index and a byte per entry, 12 bytes
    for count 8 instead of 33; one collective instead of two) — written packed by the query kernel itself at count 8
    on tables with short window lines (kad_rt_closest_batch_packed), by kad_route_compress otherwise — and
    kad_route_unpack_packed expands them; a row spanning more than 254 indices sets a sticky word (escaped()), and the batch's way back
    runs again unpacked.

    cap: records per block, a multiple of KAD_ROUTE_SUBS: a block is 8 sub-blocks, workgroup w (1,024 targets)
    appending to sub-block w % 8; default 8 x (the most targets one sub-block's workgroups hold / world + 6 sigma +
    32) for uniform targets. A sub-block that fills sets a sticky word; overflowed() combines it over the ranks (one
    host read per batch, or per K steps), grown() sizes the blocks from the counts, and the batch runs again.
    collective=True forces the collectives at world 1 (a one-rank RCCL group).

    keys (the default at count 8 with packed rows): the targets travel as 8-byte keys, their top 64 bits
    (kad_route_pack_keys), which is all the owner's short and 128-byte window lines read; the owner answers with
    kad_rt_closest_keys_packed, whose exact path (the ~0.001 % of queries no line answers) is exact from the key alone
    unless two nodes of its window share their top 64 bits — then a sticky tail word (tailed()) asks for the batch
    again from full targets (keys=False), as does an owner table without short lines. 8 + 12 bytes per query on the
    links instead of 20 + 12."""

    def __init__(self, q: int, count: int, world: int, shard_bits: int, device, cap: int | None = None,
                 collective: bool | None = None, packed: bool | None = None, keys: bool | None = None):
        import torch

        from ._lib import KAD_ROUTE_PACKED_MAX_COUNT, KAD_ROUTE_QPW, KAD_ROUTE_SUBS, route_ctr_words, route_packed_words

        self.q, self.count, self.world, self.shard_bits, self.dev = q, count, world, shard_bits, device
        # packed by default for the counts the vector kernels take (multiples of 4 up to 32: count 8 packs in 11.7 us
        # and unpacks in 8.3 us per 1M rows, against 13.1 us for the plain unpack; tools/route_packed_check.py)
        self.packed = (count % 4 == 0 and 1 <= count <= KAD_ROUTE_PACKED_MAX_COUNT) if packed is None else bool(packed)
        self.collective = world > 1 if collective is None else bool(collective)
        self.keys = (count == 8 and self.packed) if keys is None else bool(keys)
        if self.keys and not (count == 8 and self.packed):
            raise ValueError("key-only routing needs count 8 and packed rows")
        # the most targets the workgroups of one sub-block hold (workgroup w -> sub-block w % 8): a sub-block can never
        # receive more, so 8 x that is the capacity that never overflows
        S = KAD_ROUTE_SUBS
        qs = min(max(q, 1), -(-(-(-q // KAD_ROUTE_QPW)) // S) * KAD_ROUTE_QPW)
        self.cap_max = S * max(1, qs)
        nominal = -(-qs // world)
        sub = cap if cap is None else -(-cap // S)
        self.cap = S * max(1, min(qs, sub or nominal + 6 * int(np.sqrt(nominal)) + 32))
        n = world * self.cap
        self.send = torch.empty((n, 20), dtype=torch.uint8, device=device)
        pad_blocks(self.send, world, shard_bits, self.cap)
        self.recv = torch.empty_like(self.send) if self.collective else self.send
        self.send_keys = self.recv_keys = None
        if self.keys:
            self.send_keys = torch.empty((n,), dtype=torch.int64, device=device)
            pad_keys(self.send_keys, world, shard_bits, self.cap)
            self.recv_keys = torch.empty_like(self.send_keys) if self.collective else self.send_keys
        self.slot = torch.empty((max(q, 1),), dtype=torch.int32, device=device)
        self.ctr = torch.zeros((route_ctr_words(world),), dtype=torch.int32, device=device)
        self.rows = torch.empty((n, max(count, 1)), dtype=torch.int32, device=device)
        self.cnt = torch.empty((n,), dtype=torch.uint8, device=device)
        self.back_rows = torch.empty_like(self.rows) if self.collective else self.rows
        self.back_cnt = torch.empty_like(self.cnt) if self.collective else self.cnt
        self.pw = route_packed_words(count) if self.packed else 0
        self.prow = torch.empty((n, self.pw), dtype=torch.int32, device=device) if self.packed else None
        self.back_prow = (torch.empty_like(self.prow) if self.collective else self.prow) if self.packed else None

    @property
    def xgmi_bytes(self) -> dict:
        """Bytes a rank sends to the other ranks per step: targets out, rows + counts back."""
        per = 4 * self.pw if self.packed else 4 * self.count + 1
        return {"targets": self.record_bytes * (self.world - 1) * self.cap, "rows": per * (self.world - 1) * self.cap}

    @property
    def record_bytes(self) -> int:
        """Bytes per target record on the links: an 8-byte key, or the 20-byte target."""
        return 8 if self.keys else 20

    def pack(self, targets, stream, keys: bool | None = None):
        import ctypes as C

        from ._lib import check, lib, ptr

        if self.keys if keys is None else keys:
            check(lib().kad_route_pack_keys(ptr(targets), self.q, self.world, self.shard_bits, self.cap,
                                            ptr(self.send_keys), ptr(self.slot), ptr(self.ctr), self.dev.index or 0,
                                            C.c_void_p(stream)), "kad_route_pack_keys")
            return
        check(lib().kad_route_pack(ptr(targets), self.q, self.world, self.shard_bits, self.cap, ptr(self.send),
                                   ptr(self.slot), ptr(self.ctr), self.dev.index or 0, C.c_void_p(stream)),
              "kad_route_pack")

    def unpack(self, out_idx, out_cnt, stream):
        import ctypes as C

        from ._lib import check, lib, ptr

        check(lib().kad_route_unpack(ptr(self.slot), self.q, self.count, ptr(self.back_rows), ptr(self.back_cnt),
                                     ptr(out_idx), ptr(out_cnt), self.dev.index or 0, C.c_void_p(stream)),
              "kad_route_unpack")

    def compress(self, stream):
        """The answered rows packed for the way back (escape word: ctr[KAD_ROUTE_OVERFLOW_WORD(world) + 1])."""
        import ctypes as C

        from ._lib import check, lib, ptr, route_overflow_word

        n = self.world * self.cap
        check(lib().kad_route_compress(ptr(self.rows), ptr(self.cnt), n, self.count, ptr(self.prow),
                                       C.c_void_p(self.ctr.data_ptr() + 4 * (route_overflow_word(self.world) + 1)),
                                       self.dev.index or 0, C.c_void_p(stream)), "kad_route_compress")

    def unpack_packed(self, out_idx, out_cnt, stream):
        import ctypes as C

        from ._lib import check, lib, ptr

        check(lib().kad_route_unpack_packed(ptr(self.slot), self.q, self.count, ptr(self.back_prow), ptr(out_idx),
                                            ptr(out_cnt), self.dev.index or 0, C.c_void_p(stream)),
              "kad_route_unpack_packed")

    def answer(self, table, stream, packed: bool | None = None, keys: bool | None = None):
        """The owner's rows for every record of the received blocks (table: a DeviceTable). Packed rows at count 8 on
        a table with short window lines come packed out of the query kernel itself (kad_rt_closest_batch_packed:
        `fused`); otherwise full rows, packed by compress() on the way back. keys: from the received 8-byte keys
        (kad_rt_closest_keys_packed; an owner table without short lines sets the tail word)."""
        import ctypes as C

        from ._lib import KAD_ERR_UNSUPPORTED, check, lib, ptr, route_overflow_word

        self.fused = False
        if self.keys if keys is None else keys:
            esc = self.ctr.data_ptr() + 4 * (route_overflow_word(self.world) + 1)
            rc = lib().kad_rt_closest_keys_packed(table._h, ptr(self.recv_keys), self.world * self.cap, self.count,
                                                  ptr(self.prow), C.c_void_p(esc), C.c_void_p(esc + 4),
                                                  C.c_void_p(stream))
            self.fused = True
            if rc == KAD_ERR_UNSUPPORTED:
                import torch

                from .global_shard import _torch_stream

                w = route_overflow_word(self.world) + 2
                with torch.cuda.stream(_torch_stream(stream, self.dev)):
                    self.ctr[w:w + 1].fill_(1)
                return
            check(rc, "kad_rt_closest_keys_packed")
            return
        if (self.packed if packed is None else packed) and self.count == 8:
            rc = lib().kad_rt_closest_batch_packed(
                table._h, ptr(self.recv), self.world * self.cap, self.count, ptr(self.prow),
                C.c_void_p(self.ctr.data_ptr() + 4 * (route_overflow_word(self.world) + 1)), C.c_void_p(stream))
            if rc != KAD_ERR_UNSUPPORTED:
                check(rc, "kad_rt_closest_batch_packed")
                self.fused = True
                return
        table.rt_closest(self.recv, self.count, out_idx=self.rows, out_cnt=self.cnt, stream=stream)

    def step(self, table, targets, out_idx, out_cnt, group=None, stream=None, packed: bool | None = None,
             keys: bool | None = None):
        """pack, send, answer, return, unpack: device-only (check overflowed(), then tailed(), then escaped(), after).
        packed=False: the way back unpacked (the rerun of a batch whose rows escaped packing); keys=False: full
        targets (the rerun of a batch whose key-only answer needed the targets' low bits)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        packed = self.packed if packed is None else packed
        keys = (self.keys if keys is None else keys) and packed
        self.pack(targets, s, keys)
        self.send_targets(group, s, keys)
        self.answer(table, s, packed, keys)
        self.back(out_idx, out_cnt, group, s, packed)

    def back(self, out_idx, out_cnt, group, s, packed: bool):
        """The way back of the answered rows: return + unpack (packed or not)."""
        if packed and not getattr(self, "fused", False):
            self.compress(s)
        self.send_back(group, s, packed)
        self.unpack_rows(out_idx, out_cnt, s, packed)

    def send_targets(self, group, s, keys: bool | None = None):
        """The target blocks to their owners (all_to_all_single on stream s; nothing without a collective)."""
        import torch

        from .global_shard import _torch_stream

        if self.collective:
            with torch.cuda.stream(_torch_stream(s, self.dev)):
                if self.keys if keys is None else keys:
                    _all_to_all(self.recv_keys, self.send_keys, group)
                else:
                    _all_to_all(self.recv, self.send, group)

    def send_back(self, group, s, packed: bool):
        """The answered rows back to their senders (packed: one all_to_all_single of the packed rows, already
        written; else the rows and the counts)."""
        import torch

        from .global_shard import _torch_stream

        if not self.collective:
            return
        with torch.cuda.stream(_torch_stream(s, self.dev)):
            if packed:
                _all_to_all(self.back_prow, self.prow, group)
            else:
                _all_to_all(self.back_rows, self.rows, group)
                _all_to_all(self.back_cnt, self.cnt, group)

    def unpack_rows(self, out_idx, out_cnt, s, packed: bool):
        if packed:
            self.unpack_packed(out_idx, out_cnt, s)
        else:
            self.unpack(out_idx, out_cnt, s)

    def fold_flags(self, acc, s):
        """acc (3 int32, device) |= this batch's overflow, escape and tail words, on stream s: kad_route_pack zeroes
        them with the counters, so a caller running many batches folds them after each one and reads acc once."""
        import torch

        from ._lib import route_overflow_word
        from .global_shard import _torch_stream

        w = route_overflow_word(self.world)
        with torch.cuda.stream(_torch_stream(s, self.dev)):
            torch.maximum(acc, self.ctr[w:w + 3], out=acc)

    def tailed(self, group=None, combine: bool = True) -> bool:
        """Host read of the key-only tail word (a batch answered from keys needs the full targets), combined."""
        if not self.keys:
            return False
        from ._lib import route_overflow_word

        return self._flag(route_overflow_word(self.world) + 2, group, combine)

    def escaped(self, group=None, combine: bool = True) -> bool:
        """Host read of the packing escape word (a row spanning more than 254 indices), combined over the ranks."""
        if not self.packed:
            return False
        from ._lib import route_overflow_word

        return self._flag(route_overflow_word(self.world) + 1, group, combine)

    def overflowed(self, group=None, combine: bool = True) -> bool:
        """Host read of the sticky overflow word, combined over the ranks (every rank decides the same)."""
        from ._lib import route_overflow_word

        return self._flag(route_overflow_word(self.world), group, combine)

    def _flag(self, w: int, group, combine: bool) -> bool:
        return bool(combine_max(self.ctr[w:w + 1], group, combine and self.collective)[0])

    def need(self, group=None, local: int | None = None) -> int:
        """The block capacity the last pack needed (8 x its fullest sub-block; or `local`), combined over the ranks."""
        import torch

        n = need_of(self.ctr, self.world) if local is None else int(local)
        if self.collective:
            import torch.distributed as dist

            nccl = dist.get_backend(group) == "nccl"
            t = torch.tensor([n], dtype=torch.int64, device=self.dev if nccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            n = int(t.item())
        return n

    def grown(self, group=None, need: int | None = None) -> "OwnerRoute":
        n = self.need(group) if need is None else need
        return OwnerRoute(self.q, self.count, self.world, self.shard_bits, self.dev,
                          cap=min(self.cap_max, max(2 * self.cap, n * 5 // 4)), collective=self.collective,
                          packed=self.packed, keys=self.keys)


def combine_max(words, group=None, combine: bool = True) -> list[int]:
    """Host read of a few device int32 words, each the MAX over the ranks when `combine` (RCCL: a device-tensor
    all_reduce on the group; gloo: through a host tensor), so that every rank decides the same."""
    if combine:
        import torch.distributed as dist

        if dist.get_backend(group) == "nccl":
            dist.all_reduce(words, op=dist.ReduceOp.MAX, group=group)
        else:
            h = words.cpu()
            dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
            words.copy_(h)
    return [int(x) for x in words.cpu()]


def pad_blocks(send, world: int, shard_bits: int, cap: int):
    """Fill every record of the `world` send blocks with a padding target owned by the block's rank, in the middle of
    its shard (byte 0 = d << (8 - shard_bits) | half of the rest, the other 19 bytes zero). The owner answers the
    whole of every block it receives, so records past a sub-block's count are answered too: before their first use
    they would otherwise be uninitialised memory whose rows could span more than 254 indices and set the packing
    escape word for the whole batch (then stale targets of the same owner, which pack like any other)."""
    import torch

    send.zero_()
    b = torch.arange(world, dtype=torch.int32, device=send.device)
    v = send.view(world, cap, 20)
    if shard_bits >= 8:
        v[:, :, 0] = b.to(torch.uint8)[:, None]
        v[:, :, 1] = 0x80
    else:
        v[:, :, 0] = ((b << (8 - shard_bits)) | (1 << (7 - shard_bits))).to(torch.uint8)[:, None]


def pad_keys(keys, world: int, shard_bits: int, cap: int):
    """pad_blocks for key-only blocks: every key the padding target's top 64 bits."""
    import torch

    b = torch.arange(world, dtype=torch.int64, device=keys.device)
    if shard_bits >= 8:
        k = (b << 56) | (0x80 << 48)
    else:
        k = ((b << (8 - shard_bits)) | (1 << (7 - shard_bits))) << 56
    keys.view(world, cap)[:] = k[:, None]


def need_of(ctr, world: int) -> int:
    """The block capacity a pack needed: KAD_ROUTE_SUBS x the fullest sub-block's record count."""
    from ._lib import KAD_ROUTE_CSTRIDE, KAD_ROUTE_SUBS

    c = ctr[:world * KAD_ROUTE_SUBS * KAD_ROUTE_CSTRIDE].view(world * KAD_ROUTE_SUBS, KAD_ROUTE_CSTRIDE)[:, 0]
    return KAD_ROUTE_SUBS * int(c.max().item())


def _all_to_all(recv, send, group=None):
    """recv <- block r of every rank's send, equal splits (dim 0): RCCL on device tensors; gloo through the host."""
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        dist.all_to_all_single(recv, send, group=group)
        return
    from .global_shard import exchange_into

    exchange_into(recv.view(-1), send.view(-1), group)


def owner_shard_bits(world: int, spec: ShardSpec | None = None) -> int:
    """The routing bits of owner routing over `world` ranks, one shard per rank: kad_route_pack sends a target to rank
    (byte 0 >> (8 - shard_bits)) % world, which is the rank holding its shard only when the table has exactly `world`
    shards and `world` is a power of two. Anything else raises instead of answering from the wrong shard."""
    if world < 1 or world & (world - 1):
        raise ValueError(f"owner routing needs a power-of-two world size, got {world}")
    if spec is not None and spec.n_shards != world:
        raise ValueError(f"the table has {spec.n_shards} shards but the group {world} ranks: one shard per rank")
    return world.bit_length() - 1


def serve_owner(table, targets, count: int, route: OwnerRoute | None = None, group=None, stream=None,
                spec: ShardSpec | None = None):
    """Answer a batch of arbitrary targets through the owner-routed shards (every rank calls it with its own batch):
    returns (out_idx, out_cnt, route) with each query's row at its position. Grows the blocks and runs again when
    one overflowed (the decision combined over the ranks). spec: the ShardSpec the tables were built from (checked
    against the group: one shard per rank)."""
    import torch
    import torch.distributed as dist

    q = targets.shape[0]
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if route is None:
        route = OwnerRoute(q, count, world, owner_shard_bits(world, spec), targets.device)
    elif route.world != world:
        raise ValueError(f"route built for {route.world} ranks, group has {world}")
    out_idx = torch.empty((q, count), dtype=torch.int32, device=targets.device)
    out_cnt = torch.empty((q,), dtype=torch.uint8, device=targets.device)
    while True:
        route.step(table, targets, out_idx, out_cnt, group, stream)
        if not route.overflowed(group):
            import torch as _t

            s = stream if stream is not None else _t.cuda.current_stream(targets.device).cuda_stream
            route.last_tailed = route.tailed(group)
            if route.last_tailed:  # a key-only answer needed the low bits: the batch again from full targets
                route.step(table, targets, out_idx, out_cnt, group, stream, keys=False)
            route.last_escaped = route.escaped(group)
            if route.last_escaped:  # a row too wide to pack: this batch's rows go back unpacked
                if route.keys:  # (the received keys cannot answer unpacked: the full targets travel)
                    route.pack(targets, s, keys=False)
                    route.send_targets(group, s, keys=False)
                route.answer(table, s, packed=False, keys=False)  # (the received targets are in place)
                route.back(out_idx, out_cnt, group, s, packed=False)
            return out_idx, out_cnt, route
        route = route.grown(group)


class OwnerPipeline:
    """Owner routing of consecutive batches with the exchanges overlapped: three OwnerRoute buffer
    sets, a compute stream (pack, answer, unpack: the kernels) and a comm stream (the all_to_alls), ordered by events.
    The host issues, for batch i,

        compute:  pack(i+1)                answer(i)                 unpack(i-1)
        comm:                 targets(i+1)             rows back(i)

    so batch i+1's pack and batch i's answer run while batch i's and i-1's blocks are on the links. A buffer set is
    reused by batch i+3 only after batch i's unpack (same compute stream, issued before): three sets, never two
    (pack(i+1) would overwrite the slots unpack(i-1) still reads). No host read inside run(): each batch's overflow
    and escape words are folded into one device accumulator; check overflowed() / escaped() after (combined over the
    ranks), and run the batches again grown() / unpacked when set."""

    DEPTH = 3

    def __init__(self, q: int, count: int, world: int, shard_bits: int, device, cap: int | None = None,
                 collective: bool | None = None, packed: bool | None = None, keys: bool | None = None):
        import torch

        self.routes = [OwnerRoute(q, count, world, shard_bits, device, cap=cap, collective=collective, packed=packed,
                                  keys=keys) for _ in range(self.DEPTH)]
        r = self.routes[0]
        self.q, self.count, self.world, self.shard_bits, self.dev = q, count, world, shard_bits, device
        self.cap, self.packed, self.collective = r.cap, r.packed, r.collective
        self.compute = torch.cuda.Stream(device)
        self.comm = torch.cuda.Stream(device)
        self.keys = r.keys
        self.acc = torch.zeros((3,), dtype=torch.int32, device=device)  # [overflow, escape, tail] over the batches

    def run(self, table, batches, outs, group=None, packed: bool | None = None, keys: bool | None = None):
        """Route every batch of `batches` ((q, 20) device targets) and unpack its rows into outs[i] = (out_idx,
        out_cnt). Returns when everything is issued; the caller's current stream waits for the last unpack.
        packed=False / keys=False: the reruns (rows back unpacked / full targets on the links)."""
        import torch

        packed = self.packed if packed is None else bool(packed)
        keys = (self.keys if keys is None else bool(keys)) and packed
        cur = torch.cuda.current_stream(self.dev)
        cs, xs = self.compute, self.comm
        cs.wait_stream(cur)
        xs.wait_stream(cur)
        n = len(batches)
        sent, back = [None] * n, [None] * n
        c, x = cs.cuda_stream, xs.cuda_stream
        R = lambda i: self.routes[i % self.DEPTH]  # noqa: E731

        def pack(i):
            R(i).pack(batches[i], c, keys)
            e = torch.cuda.Event()
            e.record(cs)
            xs.wait_event(e)
            R(i).send_targets(group, x, keys)
            sent[i] = torch.cuda.Event()
            sent[i].record(xs)

        def answer(i):
            r = R(i)
            cs.wait_event(sent[i])
            r.answer(table, c, packed, keys)
            if packed and not r.fused:
                r.compress(c)
            e = torch.cuda.Event()
            e.record(cs)
            xs.wait_event(e)
            r.send_back(group, x, packed)
            back[i] = torch.cuda.Event()
            back[i].record(xs)

        def unpack(i):
            r = R(i)
            cs.wait_event(back[i])
            r.unpack_rows(outs[i][0], outs[i][1], c, packed)
            r.fold_flags(self.acc, c)

        if n:
            pack(0)
        for i in range(n):
            if i + 1 < n:
                pack(i + 1)
            answer(i)
            if i >= 1:
                unpack(i - 1)
        if n:
            unpack(n - 1)
        cur.wait_stream(cs)
        cur.wait_stream(xs)

    def flags(self, group=None, combine: bool = True) -> tuple[bool, bool, bool]:
        """(overflowed, escaped, tailed) over every batch run since the last call, combined over the ranks;
        cleared."""
        ov, esc, tail = combine_max(self.acc, group, combine and self.collective)
        self.acc.zero_()
        return bool(ov), bool(esc) and self.packed, bool(tail) and self.keys

    def grown(self, group=None) -> "OwnerPipeline":
        """Larger blocks, sized from the fullest sub-block of the last batch each buffer set packed (combined)."""
        n = max(need_of(r.ctr, self.world) for r in self.routes)
        n = self.routes[0].need(group, local=n) if self.collective else n
        cap = min(self.routes[0].cap_max, max(2 * self.cap, n * 5 // 4))
        return OwnerPipeline(self.q, self.count, self.world, self.shard_bits, self.dev, cap=cap,
                             collective=self.collective, packed=self.packed, keys=self.keys)


def serve_pipelined(table, batches, count: int, pipe: OwnerPipeline | None = None, group=None, outs=None):
    """serve_owner for a run of batches through the overlapped OwnerPipeline: grows the blocks and runs everything
    again when some batch overflowed, from full targets when some key-only answer needed them, and with the rows back
    unpacked when some row escaped packing (every decision combined over the ranks). Returns (outs, pipe)."""
    import torch
    import torch.distributed as dist

    q = batches[0].shape[0]
    dev = batches[0].device
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if pipe is None:
        pipe = OwnerPipeline(q, count, world, owner_shard_bits(world), dev)
    if outs is None:
        outs = [(torch.empty((q, count), dtype=torch.int32, device=dev), torch.empty((q,), dtype=torch.uint8,
                                                                                     device=dev)) for _ in batches]
    while True:
        pipe.run(table, batches, outs, group)
        over, esc, tail = pipe.flags(group)
        if over:
            pipe = pipe.grown(group)
            continue
        if tail:  # some key-only answer needed the targets' low bits: everything again from full targets
            pipe.run(table, batches, outs, group, keys=False)
            _, esc, _ = pipe.flags(group)
        if esc:
            pipe.run(table, batches, outs, group, packed=False)
            pipe.flags(group)
        return outs, pipe


def route_simulated(tables, batches, count: int, shard_bits: int, cap: int | None = None, packed: bool = False):
    """Every rank of the owner-routed exchange in ONE process (one GPU): rank r packs batches[r]; rank d receives
    block d of every rank's send buffer, concatenated in rank order (what all_to_all_single delivers), answers it
    with tables[d]; rank s receives block s of every rank's rows; rank s unpacks. Grows and reruns on overflow.
    Returns ([(out_idx, out_cnt)] per rank, the last OwnerRoute of rank 0)."""
    import torch

    world = len(tables)
    dev = batches[0].device
    s = torch.cuda.current_stream(dev).cuda_stream
    while True:
        routes = [OwnerRoute(b.shape[0], count, world, shard_bits, dev, cap=cap, collective=False, packed=packed,
                             keys=False) for b in batches]
        if len({r.cap for r in routes}) != 1:
            raise ValueError("every rank's batch must give the same block size")
        c = routes[0].cap
        for r, b in zip(routes, batches):
            r.pack(b, s)
        over = any(r.overflowed(combine=False) for r in routes)
        if over:
            cap = max(2 * c, max(need_of(r.ctr, world) for r in routes) * 5 // 4)
            continue
        answered = []
        for d in range(world):
            recv = torch.cat([r.send[d * c:(d + 1) * c] for r in routes])
            rows = torch.empty((world * c, count), dtype=torch.int32, device=dev)
            cnt = torch.empty((world * c,), dtype=torch.uint8, device=dev)
            tables[d].rt_closest(recv, count, out_idx=rows, out_cnt=cnt)
            answered.append((rows, cnt))
        escaped = False
        if packed:  # owner d packs its rows (its route object's buffers hold them), the escape words combined
            packs = []
            for d in range(world):
                R = routes[d]
                R.rows, R.cnt = answered[d]
                R.compress(s)
                packs.append(R.prow.clone())
            escaped = any(R.escaped(combine=False) for R in routes)
        out = []
        for src, r in enumerate(routes):
            oi = torch.empty((r.q, count), dtype=torch.int32, device=dev)
            oc = torch.empty((r.q,), dtype=torch.uint8, device=dev)
            if packed and not escaped:
                r.back_prow = torch.cat([packs[d][src * c:(src + 1) * c] for d in range(world)])
                r.unpack_packed(oi, oc, s)
            else:
                r.back_rows = torch.cat([answered[d][0][src * c:(src + 1) * c] for d in range(world)])
                r.back_cnt = torch.cat([answered[d][1][src * c:(src + 1) * c] for d in range(world)])
                r.unpack(oi, oc, s)
            out.append((oi, oc))
        routes[0].sim_escaped = escaped
        return out, routes[0]
