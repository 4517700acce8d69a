"""ctypes binding of the CPU ORACLE (oracle/liboracle.so). TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module,
as the checker or as the timed CPU baseline -- never as the product path.
Parity status: "parity unpinned" (see kad_oracle.cpp header and DESIGN.md "Oracle").
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
NO_NODE = 0xFFFFFFFF

_P = C.c_void_p
_SIG = {
    "orc_cmp": (C.c_int, [_P, _P]),
    "orc_xor_cmp": (C.c_int, [_P, _P, _P]),
    "orc_common_bits": (C.c_uint, [_P, _P]),
    "orc_lowbit": (C.c_uint, [_P]),
    "orc_get_bit": (C.c_int, [_P, C.c_uint]),
    "orc_set_bit": (None, [_P, C.c_uint, C.c_int]),
    "orc_synth_ids": (C.c_int, [C.c_uint64, C.c_uint32, _P]),
    "orc_synth_status": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "orc_table_build": (_P, [C.c_uint32, _P, _P, C.c_uint32, _P, _P, C.c_int]),
    "orc_table_free": (None, [_P]),
    "orc_table_rt_closest": (C.c_int, [_P, C.c_uint32, _P, C.c_uint32, _P, _P, C.c_int]),
    "orc_table_nc_closest": (C.c_int, [_P, C.c_uint32, _P, C.c_uint32, _P, _P, C.c_int]),
    "orc_table_find_bucket": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "orc_flat_rt_closest": (C.c_int, [C.c_uint32, _P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, C.c_uint32,
                                      _P, _P, C.c_int]),
    "orc_flat_nc_closest": (C.c_int, [C.c_uint32, _P, _P, C.c_uint32, _P, C.c_uint32, _P, _P, C.c_int]),
    "orc_flat_rt_bytes": (C.c_uint64, [C.c_uint32, _P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, C.c_uint32,
                                       C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "orc_split_table": (C.c_int, [C.c_uint32, _P, C.c_uint32, _P, _P, _P, _P]),
    "orc_buffer_nodes": (C.c_uint32, [C.c_uint32, _P, _P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, _P]),
    "orc_is_martian": (C.c_int, [_P, C.c_uint32]),
    "orc_parse_nodes": (C.c_int, [C.c_uint32, _P, C.c_uint32, _P, _P]),
    "orc_infohash_get": (C.c_int, [C.c_uint32, _P, _P, _P]),
    "orc_table_apply": (C.c_int, [_P, C.c_uint32, _P, C.c_uint32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "orc_swarm_build": (_P, [C.c_uint32, _P, C.c_int]),
    "orc_swarm_build_lazy": (_P, [C.c_uint32, _P]),
    "orc_swarm_free": (None, [_P]),
    "orc_swarm_table": (None, [_P, C.c_uint32, _P, _P, _P]),
    "orc_swarm_closest": (C.c_int, [_P, C.c_uint32, _P, _P, C.c_uint32, _P, _P, C.c_int]),
    "orc_swarm_search": (C.c_int, [_P, C.c_uint32, _P, _P, C.c_uint32, _P, _P, _P, _P, _P, C.c_int]),
    "orc_swarm_search_ex": (C.c_int, [_P, C.c_uint32, _P, _P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P, _P, C.c_int]),
}
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        for k, (r, a) in _SIG.items():
            f = getattr(L, k)
            f.restype = r
            f.argtypes = a
        _lib = L
    return _lib


def _p(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def _ids(a):
    a = np.ascontiguousarray(a, dtype=np.uint8)
    return a.reshape(-1, 20)


# ---- primitives (bytes in, int out) ----
def xor_cmp(t: bytes, a: bytes, b: bytes) -> int:
    return lib().orc_xor_cmp(t, a, b)


def common_bits(a: bytes, b: bytes) -> int:
    return lib().orc_common_bits(a, b)


def lowbit(a: bytes) -> int:
    return lib().orc_lowbit(a)


def cmp(a: bytes, b: bytes) -> int:
    return lib().orc_cmp(a, b)


def synth_ids(n: int, seed: int) -> np.ndarray:
    out = np.empty((n, 20), dtype=np.uint8)
    lib().orc_synth_ids(seed, n, _p(out))
    return out


def synth_status(n: int, seed: int, good_pct=80, expired_pct=10) -> np.ndarray:
    out = np.empty((n,), dtype=np.uint8)
    lib().orc_synth_status(seed, n, good_pct, expired_pct, _p(out))
    return out


def split_table(ids: np.ndarray, cap: int = 8):
    ids = _ids(ids)
    n = ids.shape[0]
    perm = np.empty((n,), dtype=np.uint32)
    first = np.empty((n + 1, 20), dtype=np.uint8)
    off = np.empty((n + 2,), dtype=np.uint32)
    nb = C.c_uint32()
    lib().orc_split_table(n, _p(ids), cap, _p(perm), _p(first), _p(off), C.byref(nb))
    B = nb.value
    return perm[: off[B]].copy(), first[:B].copy(), off[: B + 1].copy()


class FaithfulTable:
    """Structure-faithful restatement: std::list<Bucket> of std::list<shared_ptr<Node>>,
    linear findBucket, find_if insertion sort, std::map NodeCache (the "port" CPU baseline)."""

    def __init__(self, ids, status, bucket_first=None, bucket_offset=None, with_nc=False):
        self.ids = _ids(ids)
        self.status = np.ascontiguousarray(status, dtype=np.uint8)
        B = 0 if bucket_first is None else bucket_first.shape[0]
        self._first = None if bucket_first is None else _ids(bucket_first)
        self._off = None if bucket_offset is None else np.ascontiguousarray(bucket_offset, dtype=np.uint32)
        self._h = lib().orc_table_build(self.ids.shape[0], _p(self.ids), _p(self.status), B, _p(self._first),
                                        _p(self._off), 1 if with_nc else 0)

    def close(self):
        if self._h:
            lib().orc_table_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rt_closest(self, targets, count, nthreads=1):
        t = _ids(targets)
        q = t.shape[0]
        idx = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty((q,), dtype=np.uint8)
        lib().orc_table_rt_closest(self._h, q, _p(t), count, _p(idx), _p(cnt), nthreads)
        return idx, cnt

    def nc_closest(self, targets, count, nthreads=1):
        t = _ids(targets)
        q = t.shape[0]
        idx = np.empty((q, count), dtype=np.uint32)
        cnt = np.empty((q,), dtype=np.uint8)
        lib().orc_table_nc_closest(self._h, q, _p(t), count, _p(idx), _p(cnt), nthreads)
        return idx, cnt

    def apply(self, ops, new_ids, new_status):
        """Mirror ops (kad_oracle.cpp "Incremental mirror ops"): ops (m, 3) uint32 rows (kind, a, b),
        kinds 1 REMOVE, 2 REPLACE, 3 INSERT, 4 SPLIT. Returns the table written out:
        (ids, status, firsts, offsets, remap of old nodes, indices of new nodes)."""
        ops = np.ascontiguousarray(ops, dtype=np.uint32).reshape(-1, 3)
        new_ids = _ids(new_ids) if len(new_ids) else np.zeros((0, 20), np.uint8)
        new_status = np.ascontiguousarray(new_status, dtype=np.uint8)
        n_old = self.ids.shape[0]
        cap = n_old + new_ids.shape[0]
        ids = np.zeros((max(cap, 1), 20), np.uint8)
        st = np.zeros(max(cap, 1), np.uint8)
        first = np.zeros((cap + ops.shape[0] + 2, 20), np.uint8)
        off = np.zeros(cap + ops.shape[0] + 3, np.uint32)
        remap = np.zeros(max(n_old, 1), np.uint32)
        nidx = np.zeros(max(new_ids.shape[0], 1), np.uint32)
        n, B = C.c_uint32(), C.c_uint32()
        lib().orc_table_apply(self._h, ops.shape[0], _p(ops), new_ids.shape[0], _p(new_ids), _p(new_status),
                              C.byref(n), C.byref(B), _p(ids), _p(st), _p(first), _p(off), _p(remap), _p(nidx))
        n, B = n.value, B.value
        return (ids[:n].copy(), st[:n].copy(), first[:B].copy(), off[:B + 1].copy(), remap[:n_old].copy(),
                nidx[:new_ids.shape[0]].copy())

    def find_bucket(self, targets):
        t = _ids(targets)
        out = np.empty((t.shape[0],), dtype=np.uint32)
        lib().orc_table_find_bucket(self._h, t.shape[0], _p(t), _p(out))
        return out


def flat_rt_closest(ids, status, bucket_first, bucket_offset, targets, count, nthreads=1):
    ids, t, f = _ids(ids), _ids(targets), _ids(bucket_first)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    off = np.ascontiguousarray(bucket_offset, dtype=np.uint32)
    q = t.shape[0]
    idx = np.empty((q, count), dtype=np.uint32)
    cnt = np.empty((q,), dtype=np.uint8)
    lib().orc_flat_rt_closest(ids.shape[0], _p(ids), _p(st), f.shape[0], _p(f), _p(off), q, _p(t), count,
                              _p(idx), _p(cnt), nthreads)
    return idx, cnt


def flat_nc_closest(sorted_ids, status, targets, count, nthreads=1):
    ids, t = _ids(sorted_ids), _ids(targets)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    q = t.shape[0]
    idx = np.empty((q, count), dtype=np.uint32)
    cnt = np.empty((q,), dtype=np.uint8)
    lib().orc_flat_nc_closest(ids.shape[0], _p(ids), _p(st), q, _p(t), count, _p(idx), _p(cnt), nthreads)
    return idx, cnt


def rt_algorithmic_bytes(ids, status, bucket_first, bucket_offset, targets, count):
    """SURVEY.md §8d algorithmic bytes: 20 + sum_{b in W(R)} (8 + n_b + 20 g_b) + 4 count, summed
    over the batch. Returns (total_bytes, visited_buckets, visited_nodes, visited_good)."""
    ids, t, f = _ids(ids), _ids(targets), _ids(bucket_first)
    st = np.ascontiguousarray(status, dtype=np.uint8)
    off = np.ascontiguousarray(bucket_offset, dtype=np.uint32)
    sb, sn, sg = C.c_uint64(), C.c_uint64(), C.c_uint64()
    tot = lib().orc_flat_rt_bytes(ids.shape[0], _p(ids), _p(st), f.shape[0], _p(f), _p(off), t.shape[0],
                                  _p(t), count, C.byref(sb), C.byref(sn), C.byref(sg))
    return int(tot), sb.value, sn.value, sg.value


def buffer_nodes(targets, ids, addrs, idx, cnt):
    """NetworkEngine::bufferNodes per query (network_engine.cpp:942-974): (q, 8*rec) bytes, (q,) counts."""
    t, ids = _ids(targets), _ids(ids)
    addrs = np.ascontiguousarray(addrs, dtype=np.uint8)
    idx = np.ascontiguousarray(idx, dtype=np.uint32)
    cnt = np.ascontiguousarray(cnt, dtype=np.uint8)
    q, k = idx.shape
    al = addrs.shape[1]
    out = np.zeros((q, 8 * (20 + al)), dtype=np.uint8)
    n = np.zeros((q,), dtype=np.uint8)
    lib().orc_buffer_nodes(q, _p(t), _p(ids), _p(addrs), al, _p(idx), _p(cnt), k, _p(out), _p(n))
    return out, n


def parse_nodes(records, rec_len, myid):
    """deserializeNodes' filter (network_engine.cpp:788-828): keep flags per record."""
    rec = np.ascontiguousarray(records, dtype=np.uint8).reshape(-1, rec_len)
    my = np.ascontiguousarray(myid, dtype=np.uint8)
    keep = np.zeros((rec.shape[0],), dtype=np.uint8)
    lib().orc_parse_nodes(rec.shape[0], _p(rec), rec_len, _p(my), _p(keep))
    return keep


SW_LEVELS, SW_BUCKET, SW_SEARCH, SW_LIST = 28, 8, 14, 32


class SwarmModel:
    """Config 5 swarm model (kad_oracle.cpp "Config 5 swarm model"): shape-K peer tables over sorted
    IDs, per-peer findClosestNodes, synchronous iterative lookups."""

    def __init__(self, sorted_ids, nthreads=8, lazy=False):
        """lazy: each peer's table is built when a query first reaches it (10M-peer swarms)."""
        self.ids = _ids(sorted_ids)
        self.n = self.ids.shape[0]
        self._h = (lib().orc_swarm_build_lazy(self.n, _p(self.ids)) if lazy
                   else lib().orc_swarm_build(self.n, _p(self.ids), nthreads))

    def close(self):
        if self._h:
            lib().orc_swarm_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def table(self, p):
        d = C.c_uint32()
        cnt = np.zeros(SW_LEVELS, np.uint8)
        ent = np.zeros((SW_LEVELS, SW_BUCKET), np.uint32)
        lib().orc_swarm_table(self._h, p, C.byref(d), _p(cnt), _p(ent))
        return d.value, cnt, ent

    def closest(self, peers, targets, count, nthreads=8):
        peers = np.ascontiguousarray(peers, np.uint32)
        t = _ids(targets)
        q = peers.shape[0]
        idx = np.empty((q, count), np.uint32)
        cnt = np.empty((q,), np.uint8)
        lib().orc_swarm_closest(self._h, q, _p(peers), _p(t), count, _p(idx), _p(cnt), nthreads)
        return idx, cnt

    def search(self, src, targets, max_hops=64, nthreads=8):
        src = np.ascontiguousarray(src, np.uint32)
        t = _ids(targets)
        S = src.shape[0]
        lst = np.empty((S, SW_SEARCH), np.uint32)
        qf = np.empty((S, SW_SEARCH), np.uint8)
        n = np.empty((S,), np.uint8)
        hops = np.empty((S,), np.uint32)
        done = np.empty((S,), np.uint8)
        lib().orc_swarm_search(self._h, S, _p(src), _p(t), max_hops, _p(lst), _p(qf), _p(n), _p(hops), _p(done),
                               nthreads)
        return lst, qf, n, hops, done

    def search_ex(self, src, targets, offline_per_10k, max_hops=64, nthreads=8):
        """Lookups with offline peers and Search::insertNode's bad-node accounting: (list, queried, bad, n,
        hops, done), lists SW_LIST (32) wide."""
        src = np.ascontiguousarray(src, np.uint32)
        t = _ids(targets)
        S = src.shape[0]
        lst = np.empty((S, SW_LIST), np.uint32)
        qf = np.empty((S, SW_LIST), np.uint8)
        bad = np.empty((S, SW_LIST), np.uint8)
        n = np.empty((S,), np.uint8)
        hops = np.empty((S,), np.uint32)
        done = np.empty((S,), np.uint8)
        lib().orc_swarm_search_ex(self._h, S, _p(src), _p(t), max_hops, offline_per_10k, _p(lst), _p(qf), _p(bad),
                                  _p(n), _p(hops), _p(done), nthreads)
        return lst, qf, bad, n, hops, done


def infohash_get(keys):
    """InfoHash::get (infohash.cpp:46-61) = SHA-1 of each byte string: (n, 20) uint8."""
    data = np.frombuffer(b"".join(keys), dtype=np.uint8) if keys else np.zeros(0, np.uint8)
    data = np.ascontiguousarray(data) if data.size else np.zeros(1, np.uint8)
    off = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.uint64)
    out = np.zeros((len(keys), 20), np.uint8)
    lib().orc_infohash_get(len(keys), _p(data), _p(off), _p(out))
    return out
