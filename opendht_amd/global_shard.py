"""North-star multi-GPU variant: the table is sharded across the GPUs of one node
with NO halo; every GPU answers its part of every query's window, the parts are all-gathered over
RCCL and merged on the device.

Per rank s (one process per GPU):
  * the shard table holds global buckets [lo, hi) of a global U(depth) table, with global node
    indices (index_base = nodes below lo); window lines make its interior queries one line each;
  * the GLOBAL good prefix sums (4 bytes per global bucket) are all-gathered once at setup, so the
    rank can compute any query's global window W(R) (routing_table.cpp:89-104);
  * a step: kad_rt_shard_batch over the replicated batch appends complete rows (W(R) inside the
    shard) and partial rows (W(R) crossing an edge, with XOR distances); the ranks' counters are
    all-gathered (one small collective, one host read), then one payload per rank (its rows, then
    its parts) in one all_gather_into_tensor; kad_rt_scatter_rows writes the rows straight from
    the received buffer, kad_rt_merge_parts merges the parts. Every rank ends with every query's
    result, bit-exact with RoutingTable::findClosestNodes on the whole table.

The owner-routed halo variant (sharded.py) moves only results a client asked for; this variant
is the one the north star describes and config 3 names ("RCCL all-gather + top-k merge").
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import synth as S
from ._lib import check, lib, part_words, ptr, row_words
from .metrics import good_counts
from .table import DeviceTable

REGIONS = 8    # KAD_SHARD_REGIONS
COUNTERS = 10  # KAD_SHARD_COUNTERS
CSTRIDE = 32   # KAD_SHARD_COUNTER_STRIDE


def reach(gpre: np.ndarray, lo: int, hi: int, count_max: int) -> tuple[int, int]:
    """[reach_lo, reach_hi): every global bucket whose window (count <= count_max) can touch
    buckets [lo, hi). A bucket b < lo - X cannot reach lo if buckets [lo - X, lo) hold >= count_max
    good nodes: W(R_b - 1) would already contain them, contradicting the least R (symmetric on the
    right). gpre: global good prefix sums (B + 1)."""
    B = gpre.shape[0] - 1
    x = 1
    while lo - x > 0 and gpre[lo] - gpre[lo - x] < count_max:
        x *= 2
    rlo = max(0, lo - x)
    x = 1
    while hi + x < B and gpre[hi + x] - gpre[hi] < count_max:
        x *= 2
    rhi = min(B, hi + x)
    return rlo, rhi


def allgather_padded(x, n: int, group=None):
    """All-gather the first n rows of x (rows may differ per rank). Returns (stacked (world, maxn, ...),
    counts list). Works on gloo (CPU) and RCCL (device tensors): counts first, then a padded gather."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    cnt = torch.tensor([n], dtype=torch.int64, device=x.device)
    cnts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(cnts, cnt, group=group)
    counts = [int(c.item()) for c in cnts]
    maxn = max(counts)
    send = x[:maxn]
    if send.shape[0] < maxn:
        send = torch.cat([send, send.new_zeros((maxn - send.shape[0],) + tuple(send.shape[1:]))])
    out = [torch.empty_like(send) for _ in range(world)]
    dist.all_gather(out, send.contiguous(), group=group)
    return torch.stack(out), counts


class GlobalShard:
    """Rank s's shard of a global U(depth) table, queried with the replicated-batch protocol."""

    def __init__(self, ids, status, off, lo: int, hi: int, depth: int, index_base: int, gpre_global,
                 device: int = 0, count_max: int = 32, base_hi: int = 0):
        import torch

        self.lo, self.hi, self.depth, self.device = lo, hi, depth, device
        self.dev = torch.device("cuda", device)
        first = S.bucket_firsts(depth, lo, hi)
        self.table = DeviceTable(ids, status, first, off, device=device, index_base=index_base, sorted=True)
        gp = np.ascontiguousarray(gpre_global, dtype=np.int64)
        self.GB = gp.shape[0] - 1
        self.gpre = torch.from_numpy(gp.astype(np.uint32).view(np.int32)).to(self.dev)
        self.reach = reach(gp, lo, hi, count_max)
        self.base_hi = base_hi
        self.ctr = torch.zeros(COUNTERS * CSTRIDE, dtype=torch.int32, device=self.dev)
        self._cap = (0, 0, 0, 0)

    def close(self):
        self.table.close()

    def _buffers(self, q: int, count: int, part_cap: int = 0):
        import torch

        if self._cap[:2] != (q, count) or part_cap > self._cap[3]:
            # rows of query block k go to region k % 8: this capacity can never overflow
            row_cap = -(-(-(-q // 256)) // 8) * 256
            part_cap = max(part_cap, 4096, q // 16)
            self.rows = torch.empty((REGIONS * row_cap, row_words(count)), dtype=torch.int32, device=self.dev)
            self.parts = torch.empty((part_cap, part_words(count)), dtype=torch.int32, device=self.dev)
            self._cap = (q, count, row_cap, part_cap)
        return self._cap[2], self._cap[3]

    def local(self, targets, count: int, stream=None):
        """This rank's rows (REGIONS regions of row_cap) and parts for a replicated (q, 20) device batch;
        async on `stream`. Counters: rows per region, parts, overflow flag."""
        import torch

        q = targets.shape[0]
        row_cap, part_cap = self._buffers(q, count)
        s = C.c_void_p(stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream)
        self.ctr.zero_()
        check(lib().kad_rt_shard_batch(self.table.handle, ptr(self.gpre), self.GB, C.c_uint64(self.base_hi),
                                       self.depth, self.lo, self.reach[0], self.reach[1], ptr(targets), q, count,
                                       ptr(self.rows), row_cap, ptr(self.parts), part_cap, ptr(self.ctr), s),
              "kad_rt_shard_batch")
        return self.rows, self.parts, self.ctr

    def local_compact(self, targets, count: int):
        """local(), a host sync, and the valid rows / parts as contiguous (n, words) tensors. A part
        buffer overflow (windows crossing many shard edges) grows the buffer and runs again."""
        import torch

        while True:
            rows, parts, ctr = self.local(targets, count)
            c = ctr.cpu().numpy()[::CSTRIDE]
            if not c[9]:
                break
            if (c[:REGIONS] > self._cap[2]).any():
                raise RuntimeError("kad_rt_shard_batch: row region overflow")
            self._buffers(targets.shape[0], count, part_cap=2 * int(c[8]))
        cap = self._cap[2]
        valid = torch.cat([rows[r * cap:r * cap + int(c[r])] for r in range(REGIONS)])
        return valid, parts[:int(c[8])]

    def query(self, targets, count: int, group=None, out_idx=None, out_cnt=None, single_rank_shard_kernel=False):
        """Every query's RoutingTable::findClosestNodes result on every rank: local rows and parts,
        all-gather (RCCL / gloo), device scatter and merge. A single rank holds the whole table: the
        exchange is empty and the batch is the plain kad_rt_closest_batch (single_rank_shard_kernel:
        the shard kernel and the scatter instead, what each rank runs at N > 1 minus the exchange)."""
        import torch
        import torch.distributed as dist

        q = targets.shape[0]
        if out_idx is None:
            out_idx = torch.empty((q, count), dtype=torch.int32, device=self.dev)
        if out_cnt is None:
            out_cnt = torch.empty((q,), dtype=torch.uint8, device=self.dev)
        if count == 0:
            out_cnt.zero_()
            return out_idx, out_cnt
        s = C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        if world == 1:
            if (self.lo, self.hi) != (0, self.GB):
                raise ValueError("a single rank must hold the whole table")
            if not single_rank_shard_kernel:
                return self.table.rt_closest(targets, count, out_idx=out_idx, out_cnt=out_cnt)
            # one shard = the whole table: every window is complete, no parts, no host sync
            rows, _, ctr = self.local(targets, count)
            check(lib().kad_rt_scatter_rows(ptr(rows), ptr(ctr), CSTRIDE, REGIONS, self._cap[2], count, ptr(out_idx),
                                            ptr(out_cnt), self.device, s), "kad_rt_scatter_rows")
            return out_idx, out_cnt
        rw, pw = row_words(count), part_words(count)
        while True:  # every rank's counters in one small gather, read once on the host
            rows, parts, ctr = self.local(targets, count)
            c_all = torch.empty((world, COUNTERS), dtype=torch.int32, device=self.dev)
            gather_into(c_all.view(-1), ctr[::CSTRIDE][:COUNTERS].contiguous(), group)
            c = c_all.cpu().numpy()
            if not c[:, 9].any():
                break
            if (c[:, :REGIONS] > self._cap[2]).any():
                raise RuntimeError("kad_rt_shard_batch: row region overflow")
            # a part buffer overflowed somewhere: every rank grows its buffer and runs again
            self._buffers(q, count, part_cap=2 * int(c[:, 8].max()))
        n_r = c[:, :REGIONS].sum(axis=1)
        maxr, maxp = int(n_r.max()), int(c[:, 8].max())
        # one payload per rank: its rows, then its parts, padded to block_cap rows of rw words
        block_cap = maxr + -(-maxp * pw // rw)
        send = torch.empty((block_cap * rw,), dtype=torch.int32, device=self.dev)
        cap, at = self._cap[2], 0
        for r in range(REGIONS):
            n = int(c[rank_of(group), r])
            send[at:at + n * rw] = rows[r * cap:r * cap + n].reshape(-1)
            at += n * rw
        n_p = int(c[rank_of(group), 8])
        send[maxr * rw:maxr * rw + n_p * pw] = parts[:n_p].reshape(-1)
        recv = torch.empty((world * block_cap * rw,), dtype=torch.int32, device=self.dev)
        gather_into(recv, send, group)
        n_rows = torch.from_numpy(n_r.astype(np.int32)).to(self.dev)
        check(lib().kad_rt_scatter_rows(ptr(recv), ptr(n_rows), 1, world, block_cap, count, ptr(out_idx),
                                        ptr(out_cnt), self.device, s), "kad_rt_scatter_rows")
        if maxp:
            g = recv.view(world, block_cap * rw)
            valid = torch.cat([g[r, maxr * rw:maxr * rw + int(c[r, 8]) * pw].view(-1, pw) for r in range(world)
                               if c[r, 8]])
            merge_valid_parts(valid, count, out_idx, out_cnt, self.device)
        return out_idx, out_cnt


def gather_into(recv, send, group=None):
    """recv (world * send.numel(),) <- every rank's send, in rank order: one all_gather_into_tensor on RCCL;
    a list all-gather elsewhere (gloo, which stages device tensors through the host)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(recv, send, group=group)
    else:
        out = list(recv.view(dist.get_world_size(group), -1).unbind(0))
        tmp = [torch.empty_like(send) for _ in out]
        dist.all_gather(tmp, send, group=group)
        for o, t in zip(out, tmp):
            o.copy_(t)


def rank_of(group=None) -> int:
    import torch.distributed as dist

    return dist.get_rank(group)


def merge_parts(g_parts, pcounts, count: int, out_idx, out_cnt, device: int):
    """Valid gathered parts, sorted by qid, through kad_rt_merge_parts."""
    import torch

    if sum(pcounts) == 0:
        return
    merge_valid_parts(torch.cat([g_parts[r, :n] for r, n in enumerate(pcounts) if n]), count, out_idx, out_cnt,
                      device)


def merge_valid_parts(valid, count: int, out_idx, out_cnt, device: int):
    """Parts (n, part_words) of every rank, in any order: sorted by qid, merged by kad_rt_merge_parts."""
    import torch

    order = torch.argsort(valid[:, 0], stable=True)
    valid = valid[order].contiguous()
    s = C.c_void_p(torch.cuda.current_stream(valid.device).cuda_stream)
    check(lib().kad_rt_merge_parts(ptr(valid), valid.shape[0], count, ptr(out_idx), ptr(out_cnt), device, s),
          "kad_rt_merge_parts")


def global_good_prefix(local_good: np.ndarray, group=None, device=None) -> np.ndarray:
    """All-gather every rank's per-bucket good counts (equal bucket counts per rank, rank order =
    bucket order) and return the global good prefix sums (B + 1), host int64."""
    import torch
    import torch.distributed as dist

    x = torch.from_numpy(np.ascontiguousarray(local_good, dtype=np.int32))
    if device is not None:
        x = x.to(device)
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    if world > 1:
        parts = [torch.empty_like(x) for _ in range(world)]
        dist.all_gather(parts, x, group=group)
        x = torch.cat(parts)
    g = x.cpu().numpy().astype(np.int64)
    return np.concatenate([[0], np.cumsum(g)])


def build_plain_shard(spec, s: int):
    """Shard s of spec's global U(depth) table without halo: (ids, status, off, lo, hi, index_base,
    good counts per bucket)."""
    lo, hi = spec.owned(s)
    ids, st, off, below = spec.bucket_range_below(lo, hi)
    return ids, st, off.astype(np.uint32), lo, hi, below, good_counts(st, off)
