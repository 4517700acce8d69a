"""DeviceTable: a routing-table / NodeCache snapshot resident in HBM, queried in batches.

Thin Python plumbing over the C ABI (include/kadgpu.h) for tests and bench.py. The drop-in
host interface for OpenDHT's C++ code is include/kadgpu.hpp (RoutingTable::findClosestNodes,
NodeCache::getCachedNodes, Dht-style findClosestNodes(id, af, count)).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import KAD_TABLE_EAGER, KAD_TABLE_NO_SLOT_LINES, KAD_TABLE_SORTED, check, lib, ptr


def _as_ids(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint8)
    if a.ndim == 1:
        a = a.reshape(-1, 20)
    if a.ndim != 2 or a.shape[1] != 20:
        raise ValueError(f"ids must be (n, 20) uint8, got {a.shape}")
    return a


def _stream_of(t, stream):
    if stream is not None:  # a raw hipStream_t handle or a torch.cuda.Stream
        return C.c_void_p(getattr(stream, "cuda_stream", stream))
    import torch

    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


class DeviceTable:
    """One address family's RoutingTable and/or NodeCache map, snapshotted at `now`.

    ids            (n, 20) uint8, InfoHash bytes; grouped by bucket in list order
    status         (n,) uint8, bit0 Node::isGood(now), bit1 Node::isExpired()
    bucket_first   (B, 20) uint8 ascending, or None for a NodeCache-only table
    bucket_offset  (B+1,) uint32
    sorted         ids strictly ascending (enables NodeCache queries)
    eager          build every line set now (default: the count <= 8 lines; the others on first use)
    slot_lines     general-line tables: build slot lines (KAD_TABLE_NO_SLOT_LINES when False)
    """

    def __init__(self, ids, status, bucket_first=None, bucket_offset=None, *, device: int = 0,
                 index_base: int = 0, sorted: bool = False, eager: bool = False,
                 slot_lines: bool = True):
        L = lib()
        ids = _as_ids(ids)
        status = np.ascontiguousarray(status, dtype=np.uint8)
        n = ids.shape[0]
        if status.shape != (n,):
            raise ValueError("status must have one byte per node")
        if bucket_first is not None:
            bucket_first = _as_ids(bucket_first)
            bucket_offset = np.ascontiguousarray(bucket_offset, dtype=np.uint32)
            B = bucket_first.shape[0]
            if bucket_offset.shape != (B + 1,):
                raise ValueError("bucket_offset must have B+1 entries")
        else:
            B = 0
        h = C.c_void_p()
        rc = L.kad_table_create(C.byref(h), device, n, ptr(ids), ptr(status), B,
                                ptr(bucket_first) if B else None, ptr(bucket_offset) if B else None,
                                index_base, (KAD_TABLE_SORTED if sorted else 0) | (KAD_TABLE_EAGER if eager else 0)
                                | (0 if slot_lines else KAD_TABLE_NO_SLOT_LINES))
        check(rc, "kad_table_create")
        self._h = h
        self.device = device
        self.n = n
        self.B = B

    # -- lifetime ------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None):
            lib().kad_table_destroy(self._h)
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

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self) -> dict:
        inf = _lib.table_info()
        check(lib().kad_table_get_info(self._h, C.byref(inf)), "kad_table_get_info")
        out = {f: getattr(inf, f) for f, _ in inf._fields_}
        built = C.c_uint32()
        nb = (C.c_uint64 * 4)()
        ms = (C.c_float * 4)()
        check(lib().kad_table_line_sets(self._h, C.byref(built), nb, ms), "kad_table_line_sets")
        out["line_sets"] = {name: {"built": bool(built.value & (1 << k)), "bytes": int(nb[k]), "build_ms": float(ms[k])}
                            for k, name in enumerate(("rt16", "rt32", "nc16", "nc32"))}
        return out

    def serve(self, idle_us: int = 2000) -> None:
        """Resident query service (kad_table_serve): host batches of up to 64 queries with count <= 64 are answered
        by a workgroup that stays on the GPU, without a launch per call. idle_us = 0 turns it off."""
        check(lib().kad_table_serve(self._h, idle_us), "kad_table_serve")

    def serve_stats(self) -> dict:
        """kad_table_serve_stats: launches, requests, and the last request's header reads and device time."""
        st = _lib.serve_stats()
        check(lib().kad_table_serve_stats(self._h, C.byref(st)), "kad_table_serve_stats")
        return {f: getattr(st, f) for f, _ in st._fields_}

    def prepare(self, sets: int = _lib.KAD_LINES_ALL) -> None:
        """Build the line sets `sets` (KAD_LINES_*) now instead of on first use (e.g. before a graph capture)."""
        check(lib().kad_table_prepare(self._h, sets), "kad_table_prepare")

    # -- status --------------------------------------------------------------------------
    def update_status(self, status) -> None:
        status = np.ascontiguousarray(status, dtype=np.uint8)
        check(lib().kad_table_update_status(self._h, ptr(status)), "kad_table_update_status")

    def set_times(self, time_ns, reply_time_ns, expired) -> None:
        a = np.ascontiguousarray(time_ns, dtype=np.int64)
        b = np.ascontiguousarray(reply_time_ns, dtype=np.int64)
        e = np.ascontiguousarray(expired, dtype=np.uint8)
        check(lib().kad_table_set_times(self._h, ptr(a), ptr(b), ptr(e)), "kad_table_set_times")

    def patch_status(self, nodes, status) -> None:
        """Incremental status update of the listed nodes (kad_table_patch_status)."""
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        status = np.ascontiguousarray(status, dtype=np.uint8)
        if nodes.shape != status.shape:
            raise ValueError("nodes and status must have the same length")
        check(lib().kad_table_patch_status(self._h, nodes.shape[0], ptr(nodes), ptr(status)), "kad_table_patch_status")

    def patch_times(self, nodes, time_ns, reply_time_ns, expired) -> None:
        """New liveness of the listed nodes (kad_table_patch_times); applied at the next refresh_status."""
        nodes = np.ascontiguousarray(nodes, dtype=np.uint32)
        a = np.ascontiguousarray(time_ns, dtype=np.int64)
        b = np.ascontiguousarray(reply_time_ns, dtype=np.int64)
        e = np.ascontiguousarray(expired, dtype=np.uint8)
        if not (nodes.shape == a.shape == b.shape == e.shape):
            raise ValueError("patch arrays must have the same length")
        check(lib().kad_table_patch_times(self._h, nodes.shape[0], ptr(nodes), ptr(a), ptr(b), ptr(e)),
              "kad_table_patch_times")

    def refresh_status(self, now_ns: int, stream=None) -> None:
        check(lib().kad_table_refresh_status(self._h, C.c_int64(now_ns), _stream_of(self, stream)),
              "kad_table_refresh_status")

    def refresh_diag(self) -> dict:
        """kad_table_refresh_diag: the small refresh's spin timeouts, lines its last block built, guard errors."""
        d = _lib.refresh_diag()
        check(lib().kad_table_refresh_diag(self._h, C.byref(d)), "kad_table_refresh_diag")
        return {f: getattr(d, f) for f, _ in d._fields_}

    def apply(self, ops, new_ids=None, new_status=None, remap=None):
        """Incremental mirror (kad_table_apply): ops (m, 3) uint32 rows (kind, a, b). Returns the new
        nodes' indices (host uint32); `remap` (device int32 tensor, old n) receives every old node's
        new index."""
        ops = np.ascontiguousarray(ops, dtype=np.uint32).reshape(-1, 3)
        nid = _as_ids(new_ids) if new_ids is not None and len(new_ids) else np.zeros((0, 20), np.uint8)
        nst = np.ascontiguousarray(new_status if new_status is not None else np.zeros(0), dtype=np.uint8)
        out = np.zeros(max(nid.shape[0], 1), np.uint32)
        check(lib().kad_table_apply(self._h, ptr(ops), ops.shape[0], ptr(nid), ptr(nst), nid.shape[0], ptr(remap),
                                    ptr(out)), "kad_table_apply")
        inf = self.info()
        self.n, self.B = inf["n_nodes"], inf["n_buckets"]
        return out[:nid.shape[0]]

    def nc_apply(self, erase=None, ins_ids=None, ins_status=None):
        """NodeCache map mutations (kad_nc_apply) on a NodeCache-only table: erase the listed node indices,
        insert new IDs. Returns (remap (old n,) uint32, new_index (n_ins,) uint32), both host arrays."""
        er = np.ascontiguousarray(erase if erase is not None else np.zeros(0), dtype=np.uint32)
        nid = _as_ids(ins_ids) if ins_ids is not None and len(ins_ids) else np.zeros((0, 20), np.uint8)
        nst = np.ascontiguousarray(ins_status if ins_status is not None else np.zeros(0), dtype=np.uint8)
        if nst.shape[0] != nid.shape[0]:
            raise ValueError("one status byte per inserted ID")
        remap = np.zeros(max(self.n, 1), np.uint32)
        new_index = np.zeros(max(nid.shape[0], 1), np.uint32)
        check(lib().kad_nc_apply(self._h, ptr(er), er.shape[0], ptr(nid), ptr(nst), nid.shape[0], ptr(remap),
                                 ptr(new_index)), "kad_nc_apply")
        old_n = self.n
        self.n = self.info()["n_nodes"]
        return remap[:old_n], new_index[:nid.shape[0]]

    def export(self):
        """(ids, status, bucket_first, bucket_offset) host arrays of the device table."""
        inf = self.info()
        n, B = inf["n_nodes"], inf["n_buckets"]
        ids = np.zeros((max(n, 1), 20), np.uint8)
        st = np.zeros(max(n, 1), np.uint8)
        first = np.zeros((max(B, 1), 20), np.uint8)
        off = np.zeros(B + 1, np.uint32)
        check(lib().kad_table_export(self._h, ptr(ids), ptr(st), ptr(first), ptr(off)), "kad_table_export")
        return ids[:n], st[:n], first[:B], off

    def export_lines(self, which: int):
        """A derived array (KAD_LINESET_*) as host bytes (kad_table_export_lines), or None if absent."""
        nb = C.c_uint64(0)
        check(lib().kad_table_export_lines(self._h, which, None, C.byref(nb)), "kad_table_export_lines")
        if nb.value == 0:
            return None
        out = np.empty(nb.value, np.uint8)
        check(lib().kad_table_export_lines(self._h, which, ptr(out), C.byref(nb)), "kad_table_export_lines")
        return out

    def export_status(self):
        """The device's status bytes (n,), e.g. after refresh_status."""
        st = np.zeros(max(self.n, 1), np.uint8)
        check(lib().kad_table_export(self._h, None, ptr(st), None, None), "kad_table_export")
        return st[:self.n]

    def set_addrs(self, addrs) -> None:
        """Node address records (n, 6) for IPv4 (in_addr + port bytes) or (n, 18) for IPv6."""
        addrs = np.ascontiguousarray(addrs, dtype=np.uint8)
        if addrs.ndim != 2 or addrs.shape[0] != self.n or addrs.shape[1] not in (6, 18):
            raise ValueError(f"addrs must be (n, 6) or (n, 18) uint8, got {addrs.shape}")
        check(lib().kad_table_set_addrs(self._h, addrs.shape[1], ptr(addrs)), "kad_table_set_addrs")
        self.addr_len = addrs.shape[1]

    def buffer_nodes(self, targets, idx, cnt=None, stream=None):
        """NetworkEngine::bufferNodes per query (network_engine.cpp:942-974) over device tensors: the
        candidates of row i of idx (cnt[i] of them, or up to the first KAD_NO_NODE) sorted by XOR
        distance, the first 8 packed as 26- / 38-byte records. Returns (out (q, 8 * rec) uint8, n (q,))."""
        import torch

        q, k = idx.shape
        rec = 20 + self.addr_len
        out = torch.zeros((q, 8 * rec), dtype=torch.uint8, device=targets.device)
        n = torch.empty((q,), dtype=torch.uint8, device=targets.device)
        check(lib().kad_buffer_nodes_batch(self._h, ptr(targets), q, ptr(idx), ptr(cnt), k, ptr(out), ptr(n),
                                           _stream_of(self, stream)), "kad_buffer_nodes_batch")
        return out, n

    # -- device-pointer batch queries (torch tensors on this table's device) ---------------
    def rt_closest(self, targets, count: int, out_idx=None, out_cnt=None, stream=None):
        """RoutingTable::findClosestNodes over a (q, 20) uint8 device tensor of targets.
        Returns (idx int32 view of uint32 (q, count), cnt uint8 (q,))."""
        import torch

        q = targets.shape[0]
        if out_idx is None:
            out_idx = torch.empty((q, count), dtype=torch.int32, device=targets.device)
        if out_cnt is None:
            out_cnt = torch.empty((q,), dtype=torch.uint8, device=targets.device)
        check(lib().kad_rt_closest_batch(self._h, ptr(targets), q, count, ptr(out_idx), ptr(out_cnt),
                                         _stream_of(self, stream)), "kad_rt_closest_batch")
        return out_idx, out_cnt

    def nc_closest(self, targets, count: int, out_idx=None, out_cnt=None, stream=None):
        """NodeCache::getCachedNodes over a (q, 20) uint8 device tensor of targets."""
        import torch

        q = targets.shape[0]
        if out_idx is None:
            out_idx = torch.empty((q, count), dtype=torch.int32, device=targets.device)
        if out_cnt is None:
            out_cnt = torch.empty((q,), dtype=torch.uint8, device=targets.device)
        check(lib().kad_nc_closest_batch(self._h, ptr(targets), q, count, ptr(out_idx), ptr(out_cnt),
                                         _stream_of(self, stream)), "kad_nc_closest_batch")
        return out_idx, out_cnt

    def find_bucket(self, targets, out=None, stream=None):
        import torch

        q = targets.shape[0]
        if out is None:
            out = torch.empty((q,), dtype=torch.int32, device=targets.device)
        check(lib().kad_rt_find_bucket_batch(self._h, ptr(targets), q, ptr(out), _stream_of(self, stream)),
              "kad_rt_find_bucket_batch")
        return out

    # -- host-pointer synchronous queries ---------------------------------------------------
    def rt_closest_host(self, targets, count: int):
        t = _as_ids(targets)
        q = t.shape[0]
        idx = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty((q,), dtype=np.uint8)
        check(lib().kad_rt_closest_batch_host(self._h, ptr(t), q, count, ptr(idx), ptr(cnt)),
              "kad_rt_closest_batch_host")
        return idx, cnt

    def nc_closest_host(self, targets, count: int):
        t = _as_ids(targets)
        q = t.shape[0]
        idx = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty((q,), dtype=np.uint8)
        check(lib().kad_nc_closest_batch_host(self._h, ptr(t), q, count, ptr(idx), ptr(cnt)),
              "kad_nc_closest_batch_host")
        return idx, cnt


def rt_closest_dual(table4: DeviceTable | None, table6: DeviceTable | None, targets, af, count: int,
                    stream=None):
    """Per-query family select (af 0 -> v4, 1 -> v6), as Dht::onGetValues asks both tables."""
    import torch

    q = targets.shape[0]
    out_idx = torch.empty((q, count), dtype=torch.int32, device=targets.device)
    out_cnt = torch.empty((q,), dtype=torch.uint8, device=targets.device)
    s = C.c_void_p(stream) if stream is not None else C.c_void_p(
        torch.cuda.current_stream(targets.device).cuda_stream)
    check(lib().kad_rt_closest_batch_dual(table4.handle if table4 else None, table6.handle if table6 else None,
                                          ptr(targets), ptr(af), q, count, ptr(out_idx), ptr(out_cnt), s),
          "kad_rt_closest_batch_dual")
    return out_idx, out_cnt


def nc_closest_dual(table4: DeviceTable | None, table6: DeviceTable | None, targets, af, count: int, stream=None):
    """NodeCache::getCachedNodes with a per-query family (af 0 -> cache_4, 1 -> cache_6; node_cache.cpp:36-66)."""
    import torch

    q = targets.shape[0]
    out_idx = torch.empty((q, count), dtype=torch.int32, device=targets.device)
    out_cnt = torch.empty((q,), dtype=torch.uint8, device=targets.device)
    s = C.c_void_p(stream) if stream is not None else C.c_void_p(
        torch.cuda.current_stream(targets.device).cuda_stream)
    check(lib().kad_nc_closest_batch_dual(table4.handle if table4 else None, table6.handle if table6 else None,
                                          ptr(targets), ptr(af), q, count, ptr(out_idx), ptr(out_cnt), s),
          "kad_nc_closest_batch_dual")
    return out_idx, out_cnt
