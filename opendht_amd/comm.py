"""The native multi-GPU executor (csrc/kad_comm.hip): an RCCL communicator of the engine's own and the
owner-routed and north-star steps issued from C++ (kad_route_run, kad_shard_run), one call per run of batches.

Driving the same steps from Python costs ~100-160 us of host issue per batch (c10d collectives, events, ctypes
launches: profiles/r06/pipeline_issue.json), more than the device work of a 1M-query step; here the host issues a
batch in a few microseconds and the pipelined form (three buffer sets, the engine's compute and comm streams) keeps
the links busy under the kernels.

    comm = Comm(device, world, rank)          # every rank at once; rank 0's id reaches the others over a gloo group
    route = NativeRoute(q, 8, world, shard_bits, dev, comm=comm)
    route.run(table, batches, outs)           # outs[i] = (out_idx, out_cnt) of batches[i]
    over, esc = route.flags(group)            # combined over the ranks; grown() / run(packed=False) when set
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import KAD_COMM_ID_BYTES, check, lib, ptr, route_set


def _ptrs(xs):
    return (C.c_void_p * max(1, len(xs)))(*[x.data_ptr() for x in xs])


class Comm:
    """kad_comm: one rank's communicator on `device`. world > 1: rank 0 makes the id (kad_comm_unique_id) and
    broadcasts it over `group` (a torch.distributed group; gloo host tensors are fine), then every rank joins."""

    def __init__(self, device: int, world: int = 1, rank: int = 0, group=None):
        import torch

        self.device, self.world, self.rank = int(device), int(world), int(rank)
        uid = np.zeros(KAD_COMM_ID_BYTES, np.uint8)
        if rank == 0:
            check(lib().kad_comm_unique_id(ptr(uid)), "kad_comm_unique_id")
        if world > 1:
            import torch.distributed as dist

            t = torch.from_numpy(uid)
            if dist.get_backend(group) == "nccl":
                t = t.to(torch.device("cuda", self.device))
            dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
            uid = t.cpu().numpy().copy()
        h = C.c_void_p()
        check(lib().kad_comm_create(C.byref(h), self.device, self.world, self.rank, ptr(uid)), "kad_comm_create")
        self._h = h

    @property
    def handle(self):
        return self._h

    def all_to_all(self, recv, send, stream=None):
        """recv <- block r of every rank's send (equal blocks, dim 0), ncclAllToAll on `stream` (raw; default the
        current torch stream)."""
        import torch

        s = stream if stream is not None else torch.cuda.current_stream(send.device).cuda_stream
        nbytes = send.numel() * send.element_size()
        check(lib().kad_comm_all_to_all(self._h, ptr(send), ptr(recv), nbytes // self.world, C.c_void_p(s)),
              "kad_comm_all_to_all")

    def close(self):
        if getattr(self, "_h", None):
            lib().kad_comm_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class NativeRoute:
    """Buffers of kad_route_run: n_sets sets shaped like sharded.OwnerRoute (n_sets = 1: serial on the caller's
    stream; >= 3: pipelined on the communicator's streams). comm None: world 1 without a collective."""

    def __init__(self, q: int, count: int, world: int, shard_bits: int, device, cap: int | None = None,
                 n_sets: int = 3, packed: bool | None = None, comm: Comm | None = None, keys: bool | None = None):
        import torch

        from .sharded import OwnerRoute

        if comm is None and n_sets != 1:
            raise ValueError("the pipelined form needs a communicator")
        if comm is not None and comm.world != world:
            raise ValueError("world differs from the communicator's")
        self.sets = [OwnerRoute(q, count, world, shard_bits, device, cap=cap, collective=comm is not None,
                                packed=packed, keys=keys) for _ in range(n_sets)]
        r = self.sets[0]
        self.q, self.count, self.world, self.shard_bits, self.dev = q, count, world, shard_bits, device
        self.cap, self.packed, self.keys, self.comm, self.n_sets = r.cap, r.packed, r.keys, comm, n_sets

        def sets(keys):
            return (route_set * n_sets)(*[route_set(*[C.c_void_p(t.data_ptr()) if t is not None else None for t in (
                R.send_keys if keys else R.send, R.recv_keys if keys else R.recv, R.slot, R.ctr, R.rows, R.cnt,
                R.back_rows, R.back_cnt, R.prow, R.back_prow)]) for R in self.sets])

        self._sets = sets(False)
        self._sets_keys = sets(True) if self.keys else None
        # [overflow, escape, tail, capacity needed], folded by every batch's unpack (kad_route_unpack_packed_fold)
        self.acc = torch.zeros((4,), dtype=torch.int32, device=device)

    def run(self, table, batches, outs, stream=None, packed: bool | None = None, keys: bool | None = None):
        """Route batches[i] ((q, 20) device targets) and unpack its rows into outs[i] = (out_idx, out_cnt); the
        overflow / escape / tail words folded into the accumulator (flags()). packed=False / keys=False: the reruns."""
        import torch

        from ._lib import KAD_ROUTE_KEYS, KAD_ROUTE_PACKED

        packed = self.packed if packed is None else bool(packed)
        keys = (self.keys if keys is None else bool(keys)) and packed
        s = stream if stream is not None else torch.cuda.current_stream(self.dev).cuda_stream
        n = len(batches)
        mode = (KAD_ROUTE_PACKED if packed else 0) | (KAD_ROUTE_KEYS if keys else 0)
        check(lib().kad_route_run(self.comm.handle if self.comm else None, table.handle, n, _ptrs(batches), self.q,
                                  self.count, self.world, self.shard_bits, self.cap, mode, self.n_sets,
                                  self._sets_keys if keys else self._sets, _ptrs([o[0] for o in outs]),
                                  _ptrs([o[1] for o in outs]), ptr(self.acc), C.c_void_p(s)), "kad_route_run")

    def flags(self, group=None) -> tuple[bool, bool, bool]:
        """(overflowed, escaped, tailed) over every batch run since the last call, combined over the ranks (torch
        group); cleared."""
        from .sharded import combine_max

        ov, esc, tail, need = combine_max(self.acc, group, self.world > 1)
        self.acc.zero_()
        self.need = need
        return bool(ov), bool(esc) and self.packed, bool(tail) and self.keys

    def grown(self, group=None) -> "NativeRoute":
        """Larger blocks: from the largest capacity a batch of the last run needed (flags(), combined over the ranks
        already; the counters themselves are zeroed by every unpack)."""
        n = getattr(self, "need", 0)
        cap = min(self.sets[0].cap_max, max(2 * self.cap, n * 5 // 4))
        return NativeRoute(self.q, self.count, self.world, self.shard_bits, self.dev, cap=cap, n_sets=self.n_sets,
                           packed=self.packed, comm=self.comm, keys=self.keys)


def serve_native(table, batches, count: int, route: NativeRoute, group=None, outs=None):
    """serve_owner over a run of batches through kad_route_run: grows and runs everything again when a block
    overflowed, again from full targets when a key-only answer needed them, again unpacked when a row escaped packing
    (every decision combined over the ranks). Returns (outs, route)."""
    import torch

    q, dev = batches[0].shape[0], batches[0].device
    if outs is None:
        outs = [(torch.empty((q, count), dtype=torch.int32, device=dev), torch.empty((q,), dtype=torch.uint8,
                                                                                     device=dev)) for _ in batches]
    while True:
        route.run(table, batches, outs)
        over, esc, tail = route.flags(group)
        if over:
            route = route.grown(group)
            continue
        if tail:  # a key-only answer needed the targets' low bits: everything again from full targets
            route.run(table, batches, outs, keys=False)
            _, esc, _ = route.flags(group)
        if esc:
            route.run(table, batches, outs, packed=False)
            route.flags(group)
        return outs, route


def shard_run(G, comm: Comm, batches, exs, outs, stream=None):
    """kad_shard_run: the north-star step of GlobalShard G over batches (replicated (q, 20) device targets) with the
    exchange sets `exs` (1: serial; 3: pipelined; collective home Exchanges of one shape, e.g. G.pipeline()), rows of
    this rank's home range into outs[i]. The sticky overflow word is exs[0].overflow (check exs[0].overflowed())."""
    import torch

    ex = exs[0]
    s = stream if stream is not None else torch.cuda.current_stream(G.dev).cuda_stream
    check(lib().kad_shard_run(comm.handle, G.table.handle, ptr(G.gpre), G.GB, C.c_uint64(G.base_hi), G.depth, G.lo,
                              G.reach[0], G.reach[1], len(batches), _ptrs(batches), ex.q, ex.count, ex.row_cap,
                              ex.part_cap, len(exs), _ptrs([e.send for e in exs]), _ptrs([e.recv for e in exs]),
                              _ptrs([e.scratch for e in exs]), ptr(ex.overflow), _ptrs([o[0] for o in outs]),
                              _ptrs([o[1] for o in outs]), C.c_void_p(s)), "kad_shard_run")
