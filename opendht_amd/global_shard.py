"""North-star multi-GPU variant: the table is sharded across the GPUs of one node
with NO halo; every GPU answers its part of every query's window, the parts are exchanged over RCCL
and merged on the device.

Per rank s (one process per GPU):
  * the shard table holds global buckets [lo, hi) of a global U(depth) table, with global node
    indices (index_base = nodes below lo); window lines make its interior queries one line each;
  * the GLOBAL good prefix sums (4 bytes per global bucket) are all-gathered once at setup, so the
    rank can compute any query's global window W(R) (routing_table.cpp:89-104);
  * a step is device-only: kad_rt_shard_batch_home over the replicated batch appends complete rows (W(R)
    inside the shard) and partial rows (W(R) crossing an edge, with XOR distances) straight into the
    send block of the query's HOME rank (query block k of 256 queries: rank k * world / nblk); one
    all_to_all_single of the fixed-size blocks (RCCL over xGMI) delivers to every rank only the rows of its
    own home range, ~q / world rows instead of q; kad_rt_home_finish scatters them and merges each query's
    parts, reading every count on the device. Every rank ends with its home range's results, bit-exact with
    RoutingTable::findClosestNodes on the whole table. No host read per step (a full buffer sets a
    sticky overflow word, combined over the ranks once per batch), so steps can be captured in a HIP graph.
  * the all-gather form (kad_rt_shard_batch + kad_rt_gather_finish: every rank ends with every result, q
    rows into every rank) is kept as Exchange(home=False).

The owner-routed halo variant (sharded.py) moves only results a client asked for; this variant
is the one the north star describes and config 3 names ("RCCL all-gather + top-k merge").
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import synth as S
from ._lib import check, lib, part_words, ptr, row_words, shard_block_words
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


def home_range(q: int, world: int, rank: int) -> tuple[int, int]:
    """Rank `rank`'s home queries [lo, hi) of a q-query batch (kad_home_range: query blocks of 256 split evenly)."""
    lo, hi = C.c_uint32(), C.c_uint32()
    lib().kad_home_range(q, world, rank, C.byref(lo), C.byref(hi))
    return lo.value, hi.value


SHARD_QB = (256, 512, 1024, 2048)  # queries per workgroup of rt_shard_kernel (csrc KAD_SHARD_QB; 2,048 in a
# tools-build A/B)


def region_queries(q: int, world: int, qb: int) -> int:
    """The most queries of one home range (kad_home_range's split of 256-query blocks) that fall in one row region:
    workgroup w of the shard kernel (qb queries) appends its rows to region w % REGIONS."""
    nblk = -(-q // 256)
    worst = 0
    for d in range(world):
        lo = -(-(d * nblk) // world) * 256
        hi = min(q, -(-((d + 1) * nblk) // world) * 256)
        per = [0] * REGIONS
        for w in range(lo // qb, -(-hi // qb)):
            per[w % REGIONS] += max(0, min(hi, (w + 1) * qb) - max(lo, w * qb))
        worst = max(worst, max(per))
    return worst


class Exchange:
    """Fixed-size send / receive blocks of one step shape (q queries, count, world ranks).

    home=True (the default step): the send buffer is `world` blocks, block d holding what goes to rank d (the
    rows and parts of rank d's home queries: REGIONS regions of row_cap complete rows, part_cap partial rows, the
    counters); one all_to_all_single, then kad_rt_home_finish on the received blocks. A rank receives ~q / world
    rows per step.
    home=False: the all-gather layout of kad_rt_gather_finish: one block with the rows of every query, one
    all_gather_into_tensor; every rank receives every row.
    The capacities are the same on every rank (they depend on q, count and world only, or on counters combined
    over the ranks), so the collective is always matched. No host read per step: a region or part buffer that
    fills sets the sticky overflow word, which the caller checks (combined over the ranks) once per batch or once
    per K steps and then runs again with grown()."""

    def __init__(self, q: int, count: int, world: int, device, row_cap: int | None = None,
                 part_cap: int | None = None, home: bool = True, collective: bool | None = None):
        import torch

        self.q, self.count, self.world, self.dev, self.home = q, count, world, device, home
        # the step runs the collective (and the overflow combine) at world > 1; collective=True forces it at
        # world 1 too (a one-rank RCCL group: the same calls on the same buffers, tests/rccl_world1_worker.py)
        self.collective = world > 1 if collective is None else bool(collective)
        nblk = -(-q // 256)
        if home:
            # region w % 8 of the workgroups (QB = 256 ... 2,048 queries, the shard kernel's shard_qb) holding a
            # home range's queries, two rows per query at most (a line query its line cannot answer leaves a
            # tombstone row, then its wave-path row): this capacity can never overflow, for any QB of SHARD_QB
            worst = max(region_queries(q, world, qb) for qb in SHARD_QB)
            self.row_cap_max = 2 * worst
            # uniform targets: a source shard answers ~1/world of a region's queries
            exp = -(-worst // world)
            est = exp + 6 * int(np.sqrt(exp)) + 32
            part_def = 256
        else:
            # rows of workgroup w (QB queries) go to region w % 8 (two per query at most: tombstones)
            self.row_cap_max = 2 * max(region_queries(q, 1, qb) for qb in SHARD_QB)
            est = -(-q // (REGIONS * world)) * 5 // 4 + 256  # ~q / world rows per rank
            part_def = 1024
        self.row_cap = max(1, min(self.row_cap_max, row_cap or est))
        self.part_cap = max(1, part_cap or part_def)
        rw, pw = row_words(count), part_words(count)
        self.parts_off = REGIONS * self.row_cap * rw
        self.ctr_off = self.parts_off + self.part_cap * pw
        self.block = shard_block_words(count, self.row_cap, self.part_cap)
        nsend = world if home else 1
        self.send = torch.zeros((nsend * self.block,), dtype=torch.int32, device=device)
        self.recv = self.send if not self.collective else torch.empty((world * self.block,), dtype=torch.int32,
                                                                      device=device)
        qh = max(home_range(q, world, r)[1] - home_range(q, world, r)[0] for r in range(world)) if home else q
        self.scratch = torch.full((qh + world * self.part_cap,), -1, dtype=torch.int32, device=device)
        self.overflow = torch.zeros((1,), dtype=torch.int32, device=device)

    @property
    def gathered_bytes(self) -> int:
        """Bytes every rank receives per step (world fixed-size blocks, its own included)."""
        return 4 * self.world * self.block

    @property
    def xgmi_bytes(self) -> int:
        """Bytes every rank receives from the other ranks per step (over xGMI)."""
        return 4 * (self.world - 1) * self.block

    def counters(self):
        """This rank's counter words (a view of the send block; the all-gather layout)."""
        return self.send[self.ctr_off:self.ctr_off + COUNTERS * CSTRIDE]

    def overflowed(self, group=None, combine: bool = True) -> bool:
        """Host read of the sticky overflow word (synchronises), cleared. The home exchange combines it over the
        ranks first (each rank sees only the blocks sent to it), so every rank decides the same (combine=False:
        one process simulating the ranks)."""
        if combine and self.home and self.collective:
            import torch.distributed as dist

            if dist.get_backend(group) == "nccl":
                dist.all_reduce(self.overflow, op=dist.ReduceOp.MAX, group=group)
            else:  # gloo: through a host tensor (its device-tensor path does not order after the finish kernel)
                h = self.overflow.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.MAX, group=group)
                self.overflow.copy_(h)
        v = bool(int(self.overflow.item()))
        if v:
            self.overflow.zero_()
        return v

    def parts_received(self) -> int:
        """Partial rows in the received blocks of the last step."""
        c = self.recv.view(self.world, self.block)[:, self.ctr_off:self.ctr_off + COUNTERS * CSTRIDE]
        return int(c.cpu().numpy().reshape(self.world, COUNTERS, CSTRIDE)[:, 8, 0].astype(np.int64).sum())

    def needs(self) -> tuple[int, int]:
        """The largest region and part counts in the received blocks of the last step."""
        c = self.recv.view(self.world, self.block)[:, self.ctr_off:self.ctr_off + COUNTERS * CSTRIDE]
        c = c.cpu().numpy().reshape(self.world, COUNTERS, CSTRIDE)[:, :, 0].astype(np.int64)
        return int(c[:, :REGIONS].max()), int(c[:, 8].max())

    def grown(self, group=None, needs: tuple[int, int] | None = None) -> "Exchange":
        """A new layout sized from the counters of the last step, combined over the ranks (the same on every
        rank). needs: the (rows, parts) counts to fit, if known (query_simulated)."""
        need_r, need_p = needs if needs is not None else self.needs()
        if needs is None and self.home and self.collective:
            import torch
            import torch.distributed as dist

            nccl = dist.get_backend(group) == "nccl"
            t = torch.tensor([need_r, need_p], dtype=torch.int64, device=self.dev if nccl else "cpu")
            dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
            need_r, need_p = (int(x) for x in t.cpu())
        row_cap = self.row_cap if need_r <= self.row_cap else max(2 * self.row_cap, need_r * 5 // 4)
        part_cap = self.part_cap if need_p <= self.part_cap else max(2 * self.part_cap, need_p * 5 // 4)
        return Exchange(self.q, self.count, self.world, self.dev, row_cap=min(row_cap, self.row_cap_max),
                        part_cap=part_cap, home=self.home, collective=self.collective)

    def home_finish(self, rank: int, out_idx, out_cnt, stream, reset: bool = False):
        """kad_rt_home_finish over the received blocks: rank `rank`'s rows (device only). reset: also zero the send
        blocks' counters for the next step (kad_rt_home_finish_reset; the send buffer must not be the receive one)."""
        if reset:
            check(lib().kad_rt_home_finish_reset(ptr(self.recv), ptr(self.send), self.world, rank, self.row_cap,
                                                 self.part_cap, self.q, self.count, ptr(self.scratch), ptr(out_idx),
                                                 ptr(out_cnt), ptr(self.overflow), self.dev.index or 0, stream),
                  "kad_rt_home_finish_reset")
            return
        check(lib().kad_rt_home_finish(ptr(self.recv), self.world, rank, self.row_cap, self.part_cap, self.q,
                                       self.count, ptr(self.scratch), ptr(out_idx), ptr(out_cnt), ptr(self.overflow),
                                       self.dev.index or 0, stream), "kad_rt_home_finish")

    def finish(self, out_idx, out_cnt, stream):
        """kad_rt_gather_finish over the received blocks (device only)."""
        check(lib().kad_rt_gather_finish(ptr(self.recv), self.world, self.row_cap, self.part_cap, self.q, self.count,
                                         ptr(self.scratch), ptr(out_idx), ptr(out_cnt), ptr(self.overflow),
                                         self.dev.index or 0, stream), "kad_rt_gather_finish")


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
        self._ex = {}

    def close(self):
        self.table.close()

    def exchange(self, q: int, count: int, world: int, home: bool = True, collective: bool | None = None) -> Exchange:
        """The cached step layout for (q, count, world, home, collective)."""
        coll = world > 1 if collective is None else bool(collective)
        key = (q, count, world, home, coll)
        if key not in self._ex:
            self._ex[key] = Exchange(q, count, world, self.dev, home=home, collective=coll)
        return self._ex[key]

    def home_block(self, targets, ex: Exchange, stream=None, zeroed: bool = False):
        """kad_rt_shard_batch_home over a replicated (q, 20) device batch into ex's `world` send blocks (their
        counters zeroed by the call; zeroed=True: kad_rt_shard_step_home, the counters already zero, as the
        previous step's finish with reset leaves them); async on `stream` (a raw hipStream_t; default: the current
        torch stream)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        fn = lib().kad_rt_shard_step_home if zeroed else lib().kad_rt_shard_batch_home
        check(fn(self.table.handle, ptr(self.gpre), self.GB, C.c_uint64(self.base_hi), self.depth, self.lo,
                 self.reach[0], self.reach[1], ptr(targets), ex.q, ex.count, ex.world, ptr(ex.send), ex.row_cap,
                 ex.part_cap, C.c_void_p(s)), "kad_rt_shard_batch_home")

    def local_block(self, targets, ex: Exchange, stream=None):
        """kad_rt_shard_batch over a replicated (q, 20) device batch into ex's send block (counters zeroed
        first); async on `stream` (a raw hipStream_t; default: the current torch stream)."""
        import torch

        ctr = ex.counters()
        if stream is None:
            s = torch.cuda.current_stream(self.dev).cuda_stream
            ctr.zero_()
        else:
            s = stream
            with torch.cuda.stream(_torch_stream(s, self.dev)):
                ctr.zero_()
        base = ex.send.data_ptr()
        check(lib().kad_rt_shard_batch(self.table.handle, ptr(self.gpre), self.GB, C.c_uint64(self.base_hi),
                                       self.depth, self.lo, self.reach[0], self.reach[1], ptr(targets), ex.q,
                                       ex.count, C.c_void_p(base), ex.row_cap, C.c_void_p(base + 4 * ex.parts_off),
                                       ex.part_cap, ptr(ctr), C.c_void_p(s)), "kad_rt_shard_batch")

    def step(self, targets, ex: Exchange, out_idx, out_cnt, group=None, stream=None, rank: int | None = None):
        """One device-only step: the send blocks, the collective (home: all_to_all_single of the world blocks;
        else all_gather_into_tensor; RCCL, gloo through the host in the CPU-rank tests; nothing at world 1), the
        scatter + merge. home: out_idx / out_cnt get this rank's home range (home_range) only. No host read:
        check ex.overflowed(group) after. `stream`: a raw hipStream_t, default the current torch stream (what
        graph capture uses)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        if ex.home:
            if rank is None:
                rank = rank_of(group) if ex.world > 1 else 0
            # with a collective the send blocks are a buffer of their own: their counters start zero (a new layout
            # is zero-filled) and each finish zeroes them for the next step, so the step has no zeroing launch
            self.home_block(targets, ex, s, zeroed=ex.collective)
            if ex.collective:
                with torch.cuda.stream(_torch_stream(s, self.dev)):
                    exchange_into(ex.recv, ex.send, group)
            ex.home_finish(rank, out_idx, out_cnt, C.c_void_p(s), reset=ex.collective)
            return
        self.local_block(targets, ex, stream)
        if ex.collective:
            if stream is None:
                gather_into(ex.recv, ex.send, group)
            else:
                with torch.cuda.stream(_torch_stream(s, self.dev)):
                    gather_into(ex.recv, ex.send, group)
        ex.finish(out_idx, out_cnt, C.c_void_p(s))

    def pipeline(self, q: int, count: int, world: int, like: Exchange | None = None) -> list:
        """Three home-exchange buffer sets (collective) for run_pipelined, with the capacities of `like` (a grown
        exchange of the same shape) or the defaults."""
        rc, pc = (like.row_cap, like.part_cap) if like is not None else (None, None)
        return [Exchange(q, count, world, self.dev, row_cap=rc, part_cap=pc, collective=True) for _ in range(3)]

    def run_pipelined(self, batches, exs, outs, group=None, rank: int = 0):
        """The north-star step over consecutive batches with the exchange overlapped: three Exchange
        buffer sets, a compute stream (kad_rt_shard_step_home, kad_rt_home_finish_reset) and a comm stream (the
        all_to_all_single), ordered by events. For batch i the host issues

            compute:  shard kernel(i+1)                    finish(i)
            comm:                      all_to_all(i+1)

        so the all_to_all of batch i+1 runs under batch i's finish and batch i+2's shard kernel. A set is reused by
        batch i+3 only after batch i's finish (which zeroed its send counters, on the same compute stream); batch i+1's
        all_to_all writes its receive blocks only after batch i-2's finish read them. outs[i] = (out_idx, out_cnt):
        this rank's home rows of batch i. No host read: check overflowed() on every set after (any(...))."""
        import torch

        if not all(ex.collective and ex.home for ex in exs) or len(exs) != 3:
            raise ValueError("run_pipelined takes three collective home exchanges (GlobalShard.pipeline)")
        cur = torch.cuda.current_stream(self.dev)
        if not hasattr(self, "_streams"):
            self._streams = (torch.cuda.Stream(self.dev), torch.cuda.Stream(self.dev))
        cs, xs = self._streams
        cs.wait_stream(cur)
        xs.wait_stream(cur)
        n = len(batches)
        sent = [None] * n

        def shard(i):
            ex = exs[i % 3]
            self.home_block(batches[i], ex, cs.cuda_stream, zeroed=True)
            e = torch.cuda.Event()
            e.record(cs)
            xs.wait_event(e)
            with torch.cuda.stream(xs):
                exchange_into(ex.recv, ex.send, group)
            sent[i] = torch.cuda.Event()
            sent[i].record(xs)

        if n:
            shard(0)
        for i in range(n):
            if i + 1 < n:
                shard(i + 1)
            cs.wait_event(sent[i])
            exs[i % 3].home_finish(rank, outs[i][0], outs[i][1], C.c_void_p(cs.cuda_stream), reset=True)
        cur.wait_stream(cs)
        cur.wait_stream(xs)

    def query(self, targets, count: int, group=None, out_idx=None, out_cnt=None, single_rank_shard_kernel=False,
              home: bool = True, force_collective: bool = False):
        """RoutingTable::findClosestNodes over a replicated batch: local rows and parts, the exchange (RCCL /
        gloo), device scatter and merge; one combined host read of the overflow word per call (a full buffer
        grows the layout and runs the batch again on every rank). home (default): returns (lo, out_idx, out_cnt)
        with this rank's home queries [lo, lo + len(out_idx)); home=False: (0, every query's rows) on every rank
        (the all-gather). A single rank holds the whole table: the plain kad_rt_closest_batch
        (single_rank_shard_kernel: the shard kernel and the finish instead, what each rank runs at N > 1 minus
        the collective; force_collective: and the collective too, through the one-rank process group)."""
        import torch
        import torch.distributed as dist

        q = targets.shape[0]
        world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        rank = rank_of(group) if world > 1 else 0
        lo, hi = home_range(q, world, rank) if home else (0, q)
        if out_idx is None:
            out_idx = torch.empty((hi - lo, count), dtype=torch.int32, device=self.dev)
        if out_cnt is None:
            out_cnt = torch.empty((hi - lo,), dtype=torch.uint8, device=self.dev)
        if count == 0 or q == 0:
            out_cnt.zero_()
            return lo, out_idx, out_cnt
        if world == 1:
            if (self.lo, self.hi) != (0, self.GB):
                raise ValueError("a single rank must hold the whole table")
            if not (single_rank_shard_kernel or force_collective):
                return 0, *self.table.rt_closest(targets, count, out_idx=out_idx, out_cnt=out_cnt)
        coll = world > 1 or force_collective
        self.tries = []  # (row_cap, part_cap) of every step of the last call
        while True:
            ex = self.exchange(q, count, world, home, coll)
            self.tries.append((ex.row_cap, ex.part_cap))
            self.step(targets, ex, out_idx, out_cnt, group, rank=rank)
            if not ex.overflowed(group):
                return lo, out_idx, out_cnt
            self._ex[(q, count, world, home, coll)] = ex.grown(group)


def query_simulated(shards, targets, count: int, out_idx=None, out_cnt=None, row_cap=None, part_cap=None,
                    home: bool = True):
    """Every shard of a global table in ONE process (one GPU, no collective), the N ranks' step:
    home (default): each shard's `world` send blocks; for every rank r the blocks the shards address to r,
    concatenated in source order (exactly what all_to_all_single delivers to rank r), then kad_rt_home_finish
    for r into r's home range of the output; home=False: each shard's block, the blocks concatenated (what
    all_gather_into_tensor delivers to every rank), kad_rt_gather_finish. How the tests drive the exchange of N
    ranks on one GPU. Returns (out_idx, out_cnt, the last Exchange) with every query's row."""
    import torch

    q, world = targets.shape[0], len(shards)
    dev = shards[0].dev
    if out_idx is None:
        out_idx = torch.empty((q, count), dtype=torch.int32, device=dev)
    if out_cnt is None:
        out_cnt = torch.empty((q,), dtype=torch.uint8, device=dev)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    while home:
        exs = [Exchange(q, count, world, dev, row_cap=row_cap, part_cap=part_cap) for _ in shards]
        for sh, ex in zip(shards, exs):
            sh.home_block(targets, ex)
        ex0 = exs[0]
        ovf, need_r, need_p, ptot = False, 0, 0, 0
        for r in range(world):
            if world > 1:
                torch.cat([e.send[r * e.block:(r + 1) * e.block] for e in exs], out=ex0.recv)
            lo, hi = home_range(q, world, r)
            ex0.home_finish(r, out_idx[lo:hi], out_cnt[lo:hi], s)
            nr, npt = ex0.needs()
            need_r, need_p = max(need_r, nr), max(need_p, npt)
            ptot += ex0.parts_received()
            ovf = ex0.overflowed(combine=False) or ovf
        if not ovf:
            ex0.parts_total = ptot
            return out_idx, out_cnt, ex0
        g = ex0.grown(needs=(need_r, need_p))
        row_cap, part_cap = g.row_cap, g.part_cap
    while True:
        exs = [Exchange(q, count, world, dev, row_cap=row_cap, part_cap=part_cap, home=False) for _ in shards]
        for sh, ex in zip(shards, exs):
            sh.local_block(targets, ex)
        ex0 = exs[0]
        if world > 1:
            torch.cat([e.send for e in exs], out=ex0.recv)
        ex0.finish(out_idx, out_cnt, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
        if not ex0.overflowed():
            ex0.parts_total = ex0.parts_received()
            return out_idx, out_cnt, ex0
        g = ex0.grown()
        row_cap, part_cap = g.row_cap, g.part_cap


def exchange_into(recv, send, group=None):
    """recv (world blocks) <- block r of every rank's send, in rank order: one all_to_all_single with equal
    splits on RCCL; elsewhere (gloo) through host tensors (gloo's all_to_all on CPU, else an all-gather of the
    whole send buffers)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "nccl":
        dist.all_to_all_single(recv, send, group=group)
        return
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    cs = send.cpu()
    cr = torch.empty_like(cs)
    try:
        dist.all_to_all_single(cr, cs, group=group)  # a real failure (timeout, dead peer) raises
    except (RuntimeError, NotImplementedError) as e:
        # a backend without all_to_all refuses it locally, before any communication, and the same way on every
        # rank (same backend), so every rank takes the all-gather together; nothing is cached per group
        if "not supported" not in str(e).lower() and "not implemented" not in str(e).lower():
            raise
        full = [torch.empty_like(cs) for _ in range(world)]
        dist.all_gather(full, cs, group=group)
        cr = torch.cat([f.view(world, -1)[rank] for f in full])
    recv.copy_(cr.to(recv.device))


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


def _torch_stream(s, dev):
    """The torch stream object for a raw hipStream_t handle. 0 is the null (legacy default) stream, which is torch's
    default stream: that stream itself, never ExternalStream(0), which does not name the null stream (work on it
    would not be ordered after the kernels the library launched on the null stream)."""
    import torch

    if not s:
        return torch.cuda.default_stream(dev)
    return torch.cuda.ExternalStream(s, device=dev)


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
