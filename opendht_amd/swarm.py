"""Config 5: a simulated swarm whose per-peer shape-K routing tables live
in HBM, and batched synchronous iterative lookups over it (libkadgpu: kad_swarm_* / kad_search_*;
model in opendht_amd/csrc/kad_swarm.hip). Thin plumbing for tests and tools/bench_swarm.py."""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import check, lib, ptr

LEVELS = 28
SEARCH_NODES = 14
SEARCH_LIST = 32  # KAD_SEARCH_LIST


class Swarm:
    def __init__(self, sorted_ids, device: int = 0):
        ids = np.ascontiguousarray(sorted_ids, dtype=np.uint8).reshape(-1, 20)
        self.n = ids.shape[0]
        self.device = device
        h = C.c_void_p()
        check(lib().kad_swarm_create(C.byref(h), device, self.n, ptr(ids)), "kad_swarm_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().kad_swarm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def device_bytes(self) -> int:
        b = C.c_uint64()
        check(lib().kad_swarm_info(self._h, None, C.byref(b)), "kad_swarm_info")
        return b.value

    def table(self, p: int):
        d = C.c_uint32()
        cnt = np.zeros(LEVELS, np.uint8)
        ent = np.zeros((LEVELS, 8), np.uint32)
        check(lib().kad_swarm_get_table(self._h, p, C.byref(d), ptr(cnt), ptr(ent)), "kad_swarm_get_table")
        return d.value, cnt, ent

    def closest(self, peers, targets, count: int):
        """Device tensors: peers (q,) int32, targets (q, 20) uint8 -> (idx (q, count), cnt (q,))."""
        import torch

        q = peers.shape[0]
        idx = torch.empty((q, count), dtype=torch.int32, device=peers.device)
        cnt = torch.empty((q,), dtype=torch.uint8, device=peers.device)
        s = C.c_void_p(torch.cuda.current_stream(peers.device).cuda_stream)
        check(lib().kad_swarm_closest_batch(self._h, ptr(peers), ptr(targets), q, count, ptr(idx), ptr(cnt), s),
              "kad_swarm_closest_batch")
        return idx, cnt

    def search(self, src, targets, offline_per_10k: int = 0) -> "Search":
        return Search(self, src, targets, offline_per_10k)


class Search:
    def __init__(self, swarm: Swarm, src, targets, offline_per_10k: int = 0):
        import torch

        self.S = src.shape[0]
        self.swarm = swarm
        h = C.c_void_p()
        s = C.c_void_p(torch.cuda.current_stream(swarm.device).cuda_stream)
        check(lib().kad_search_create(C.byref(h), swarm._h, self.S, ptr(src), ptr(targets), offline_per_10k, s),
              "kad_search_create")
        self._h = h

    def hop(self) -> int:
        a = C.c_uint32()
        check(lib().kad_search_hop(self._h, C.byref(a)), "kad_search_hop")
        return a.value

    def run(self, max_hops: int = 64) -> int:
        """Hops until every lookup is done (or max_hops); returns the rounds run."""
        for h in range(max_hops):
            if self.hop() == 0:
                return h + 1
        return max_hops

    def get(self, full: bool = False):
        """(list, queried, n, hops, done) with lists cut to SEARCH_NODES entries (n clamped to them); full=True:
        (list, queried, bad, n, hops, done, overflow) with the KAD_SEARCH_LIST-wide lists."""
        S = self.S
        lst = np.empty((S, SEARCH_LIST), np.uint32)
        q = np.empty((S, SEARCH_LIST), np.uint8)
        bad = np.empty((S, SEARCH_LIST), np.uint8)
        n = np.empty((S,), np.uint8)
        hops = np.empty((S,), np.uint32)
        done = np.empty((S,), np.uint8)
        ovf = C.c_uint32()
        check(lib().kad_search_get(self._h, ptr(lst), ptr(q), ptr(bad), ptr(n), ptr(hops), ptr(done), C.byref(ovf)),
              "kad_search_get")
        if full:
            return lst, q, bad, n, hops, done, ovf.value
        # the truncated view: n clamped to the columns returned (with offline peers a list also holds bad nodes and
        # can be longer than SEARCH_NODES; full=True returns it whole)
        return lst[:, :SEARCH_NODES].copy(), q[:, :SEARCH_NODES].copy(), np.minimum(n, SEARCH_NODES), hops, done

    def close(self):
        if getattr(self, "_h", None):
            lib().kad_search_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
