"""ctypes binding of libkadgpu.so (the C ABI in include/kadgpu.h).

The library is built in-tree by ``__graft_entry__.build()`` (opendht_amd/csrc/Makefile).
There is no fallback: if the HIP library is missing, importing the query API raises.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libkadgpu.so")

KAD_HASH_LEN = 20
KAD_TARGET_NODES = 8
KAD_SEARCH_NODES = 14
KAD_MAX_COUNT = 32
KAD_NO_NODE = 0xFFFFFFFF
KAD_STATUS_GOOD = 0x01
KAD_STATUS_EXPIRED = 0x02
KAD_TABLE_SORTED = 0x01
KAD_TABLE_EAGER = 0x02
KAD_TABLE_NO_SLOT_LINES = 0x04
KAD_LINES_RT16, KAD_LINES_RT32, KAD_LINES_NC16, KAD_LINES_NC32, KAD_LINES_ALL = 0x01, 0x02, 0x04, 0x08, 0x0F
# kad_table_export_lines sets
(KAD_LINESET_WL, KAD_LINESET_WS, KAD_LINESET_WL16, KAD_LINESET_WL32, KAD_LINESET_GL, KAD_LINESET_GL16, KAD_LINESET_GL32,
 KAD_LINESET_SL, KAD_LINESET_SL16, KAD_LINESET_NCL, KAD_LINESET_NCL32, KAD_LINESET_GCNT, KAD_LINESET_DIR) = range(13)
KAD_INFO_WINDOW_LINES = 0x100
KAD_INFO_GENERAL_LINES = 0x200
KAD_INFO_GENERAL_LINES32 = 0x400
KAD_INFO_GENERAL_LINES16 = 0x4000
KAD_INFO_SLOT_LINES16 = 0x8000
KAD_INFO_SHORT_LINES = 0x800
KAD_INFO_NODECACHE_LINES32 = 0x1000
KAD_INFO_SLOT_LINES = 0x2000
KAD_SERVE_MAX_Q, KAD_SERVE_MAX_COUNT, KAD_SERVE_MAX_IDLE_US = 64, 64, 1000000
KAD_OP_REMOVE, KAD_OP_REPLACE, KAD_OP_INSERT, KAD_OP_SPLIT = 1, 2, 3, 4


def row_words(count: int) -> int:
    """KAD_ROW_WORDS: uint32 words of one complete row of kad_rt_shard_batch."""
    return 4 + ((count + 3) & ~3)


def part_words(count: int) -> int:
    """KAD_PART_WORDS: a row plus the entries' 160-bit XOR distances (5 words each)."""
    return row_words(count) + 5 * count


KAD_SHARD_REGIONS = 8
KAD_SHARD_COUNTERS = 10
KAD_SHARD_COUNTER_STRIDE = 32
KAD_SHARD_MAX_WORLD = 16
KAD_ROUTE_CSTRIDE = 32
KAD_ROUTE_MAX_WORLD = 16
KAD_ROUTE_PACKED_MAX_COUNT = 32
KAD_ROUTE_SUBS = 8
KAD_ROUTE_QPW = 1024


def route_ctr_words(world: int) -> int:
    """KAD_ROUTE_CTR_WORDS(world)"""
    return (world * KAD_ROUTE_SUBS + 1) * KAD_ROUTE_CSTRIDE


def route_overflow_word(world: int) -> int:
    """KAD_ROUTE_OVERFLOW_WORD(world)"""
    return world * KAD_ROUTE_SUBS * KAD_ROUTE_CSTRIDE


def route_packed_words(count: int) -> int:
    """KAD_ROUTE_PACKED_WORDS(count)"""
    return 1 + (count + 3) // 4


def shard_block_words(count: int, row_cap: int, part_cap: int) -> int:
    """KAD_SHARD_BLOCK_WORDS: one rank's send block (regions of rows, parts, counters)."""
    return (KAD_SHARD_REGIONS * row_cap * row_words(count) + part_cap * part_words(count)
            + KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE)


KAD_ERR_NOMEM = -3
KAD_ERR_UNSUPPORTED = -4

ERRORS = {
    -1: "KAD_ERR_INVALID",
    -2: "KAD_ERR_HIP",
    -3: "KAD_ERR_NOMEM",
    -4: "KAD_ERR_UNSUPPORTED",
    -5: "KAD_ERR_NOT_SORTED",
    -6: "KAD_ERR_NO_DEVICE",
}

# Every symbol include/kadgpu.h declares, with its ctypes signature.
_P = C.c_void_p
_u8p = C.POINTER(C.c_uint8)
_u32p = C.POINTER(C.c_uint32)
_i64p = C.POINTER(C.c_int64)
SIGNATURES = {
    "kad_last_error": (C.c_char_p, []),
    "kad_version": (C.c_int, []),
    "kad_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "kad_table_create": (C.c_int, [C.POINTER(_P), C.c_int, C.c_uint32, _P, _P, C.c_uint32, _P, _P,
                                   C.c_uint32, C.c_uint32]),
    "kad_table_destroy": (C.c_int, [_P]),
    "kad_table_get_info": (C.c_int, [_P, _P]),
    "kad_table_prepare": (C.c_int, [_P, C.c_uint32]),
    "kad_table_line_sets": (C.c_int, [_P, _P, _P, _P]),
    "kad_table_update_status": (C.c_int, [_P, _P]),
    "kad_table_apply": (C.c_int, [_P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, _P]),
    "kad_table_export": (C.c_int, [_P, _P, _P, _P, _P]),
    "kad_table_export_lines": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "kad_nc_apply": (C.c_int, [_P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, _P]),
    "kad_table_set_times": (C.c_int, [_P, _P, _P, _P]),
    "kad_table_refresh_status": (C.c_int, [_P, C.c_int64, _P]),
    "kad_table_refresh_diag": (C.c_int, [_P, _P]),
    "kad_table_patch_status": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "kad_table_patch_times": (C.c_int, [_P, C.c_uint32, _P, _P, _P, _P]),
    "kad_rt_closest_batch": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_rt_closest_batch_host": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P]),
    "kad_table_serve": (C.c_int, [_P, C.c_uint32]),
    "kad_table_serve_stats": (C.c_int, [_P, _P]),
    "kad_rt_find_bucket_batch": (C.c_int, [_P, _P, C.c_uint32, _P, _P]),
    "kad_nc_closest_batch": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_nc_closest_batch_host": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P]),
    "kad_rt_closest_batch_dual": (C.c_int, [_P, _P, _P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_nc_closest_batch_dual": (C.c_int, [_P, _P, _P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_rt_shard_batch": (C.c_int, [_P, _P, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                     C.c_uint32, _P, C.c_uint32, C.c_uint32, _P, C.c_uint32, _P, C.c_uint32,
                                     _P, _P]),
    "kad_rt_scatter_rows": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, C.c_int,
                                      _P]),
    "kad_rt_merge_parts": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, C.c_int, _P]),
    "kad_rt_gather_finish": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P,
                                       _P, C.c_int, _P]),
    "kad_home_range": (None, [C.c_uint32, C.c_uint32, C.c_uint32, _P, _P]),
    "kad_rt_shard_batch_home": (C.c_int, [_P, _P, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                          _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, C.c_uint32, C.c_uint32, _P]),
    "kad_rt_home_finish": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P,
                                     _P, _P, _P, C.c_int, _P]),
    "kad_rt_shard_step_home": (C.c_int, [_P, _P, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                         _P, C.c_uint32, C.c_uint32, C.c_uint32, _P, C.c_uint32, C.c_uint32, _P]),
    "kad_rt_home_finish_reset": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                           C.c_uint32, _P, _P, _P, _P, C.c_int, _P]),
    "kad_route_pack": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_int, _P]),
    "kad_route_unpack": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, C.c_int, _P]),
    "kad_route_compress": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P, C.c_int, _P]),
    "kad_rt_closest_batch_packed": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_route_unpack_packed": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_int, _P]),
    "kad_route_fold_flags": (C.c_int, [_P, C.c_uint32, _P, C.c_int, _P]),
    "kad_route_pack_keys": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_int, _P]),
    "kad_rt_closest_keys_packed": (C.c_int, [_P, _P, C.c_uint32, C.c_uint32, _P, _P, _P, _P]),
    "kad_route_pack_ex": (C.c_int, [_P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P, C.c_uint32, C.c_int,
                                    _P]),
    "kad_route_unpack_packed_fold": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, _P, _P, C.c_uint32, _P, C.c_int,
                                               _P]),
    "kad_comm_unique_id": (C.c_int, [_P]),
    "kad_comm_create": (C.c_int, [C.POINTER(_P), C.c_int, C.c_uint32, C.c_uint32, _P]),
    "kad_comm_destroy": (C.c_int, [_P]),
    "kad_comm_info": (C.c_int, [_P, _P, _P, _P]),
    "kad_comm_all_to_all": (C.c_int, [_P, _P, _P, C.c_uint64, _P]),
    "kad_route_run": (C.c_int, [_P, _P, C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_uint32, C.c_uint32, _P, _P, _P, _P, _P]),
    "kad_shard_run": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                C.c_uint32, _P, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32, _P, _P, _P,
                                _P, _P, _P, _P]),
    "kad_table_set_addrs": (C.c_int, [_P, C.c_uint32, _P]),
    "kad_buffer_nodes_batch": (C.c_int, [_P, _P, C.c_uint32, _P, _P, C.c_uint32, _P, _P, _P]),
    "kad_parse_nodes_batch": (C.c_int, [_P, C.c_uint32, C.c_uint32, _P, _P, C.c_int, _P]),
    "kad_swarm_create": (C.c_int, [C.POINTER(_P), C.c_int, C.c_uint32, _P]),
    "kad_swarm_destroy": (C.c_int, [_P]),
    "kad_swarm_info": (C.c_int, [_P, _P, _P]),
    "kad_swarm_get_table": (C.c_int, [_P, C.c_uint32, _P, _P, _P]),
    "kad_swarm_closest_batch": (C.c_int, [_P, _P, _P, C.c_uint32, C.c_uint32, _P, _P, _P]),
    "kad_search_create": (C.c_int, [C.POINTER(_P), _P, C.c_uint32, _P, _P, C.c_uint32, _P]),
    "kad_search_hop": (C.c_int, [_P, _P]),
    "kad_search_get": (C.c_int, [_P, _P, _P, _P, _P, _P, _P, _P]),
    "kad_search_destroy": (C.c_int, [_P]),
    "kad_xor_cmp_batch": (C.c_int, [_P, _P, _P, C.c_uint32, _P, _P]),
    "kad_common_bits_batch": (C.c_int, [_P, _P, C.c_uint32, _P, _P]),
    "kad_lowbit_batch": (C.c_int, [_P, C.c_uint32, _P, _P]),
    "kad_infohash_get_batch": (C.c_int, [_P, _P, C.c_uint32, _P, C.c_int, _P]),
    "kad_synth_ids": (C.c_int, [C.c_uint64, C.c_uint32, _P]),
    "kad_synth_status": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, _P]),
    "kad_sort_ids": (C.c_int, [C.c_uint32, _P, _P]),
    "kad_uniform_buckets": (C.c_int, [C.c_uint32, _P, C.c_uint32, C.c_uint64, C.c_uint64, _P, _P]),
    "kad_split_table": (C.c_int, [C.c_uint32, _P, C.c_uint32, _P, _P, _P, _P]),
    "kad_synth_uniform_shard": (C.c_int, [C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64, C.c_double,
                                          C.c_uint32, C.c_uint32, _P, _P, _P, _P]),
    "kad_synth_recipe_range": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, C.c_uint64, C.c_uint64,
                                         C.c_uint32, C.c_uint32, C.c_uint64, _P, _P, _P, _P, _P]),
}


class KadError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


class table_info(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint32), ("n_buckets", C.c_uint32), ("index_base", C.c_uint32),
        ("flags", C.c_uint32), ("device", C.c_int32), ("rt_radix_bits", C.c_uint32),
        ("nc_radix_bits", C.c_uint32), ("n_good", C.c_uint32), ("device_bytes", C.c_uint64),
    ]


KAD_COMM_ID_BYTES = 128
KAD_ROUTE_PACKED, KAD_ROUTE_KEYS, KAD_ROUTE_ZEROED = 1, 2, 4


class route_set(C.Structure):
    """kad_route_set: one buffer set of kad_route_run (device pointers)."""
    _fields_ = [(n, C.c_void_p) for n in ("send", "recv", "slot", "ctr", "rows", "cnt", "back_rows", "back_cnt", "prow",
                                          "back_prow")]


class serve_stats(C.Structure):
    _fields_ = [
        ("idle_us", C.c_uint32), ("last_polls", C.c_uint32), ("launches", C.c_uint64), ("requests", C.c_uint64),
        ("last_busy_ns", C.c_uint64),
    ]


class refresh_diag(C.Structure):
    _fields_ = [("spin_timeouts", C.c_uint32), ("last_block_lines", C.c_uint32), ("guard_errors", C.c_uint32)]


_lib = None


def use_ablation_build() -> None:
    """Tools only (tools/bench_paths.py, tools/ab_bench.py): load libkadgpu_abl.so, the build with the
    timing-ablation kernels (make -C opendht_amd/csrc ablations), instead of the product library.
    Must run before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libkadgpu.so is already loaded")
    LIB_PATH = os.path.join(_HERE, "libkadgpu_abl.so")


def use_library(path: str) -> None:
    """Tools only (tools/nc32_ab.py): load a variant build of the engine (an A/B against the product library).
    Must run before the first lib() call."""
    global LIB_PATH
    if _lib is not None:
        raise RuntimeError("libkadgpu.so is already loaded")
    LIB_PATH = os.path.abspath(path)


def lib() -> C.CDLL:
    """Load libkadgpu.so, raising loudly (no fallback) if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build the HIP engine first (python -c "
                f"'import __graft_entry__ as g; g.build()'). There is no CPU fallback.")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, where: str) -> None:
    if rc != 0:
        raise KadError(rc, where, lib().kad_last_error().decode(errors="replace"))


def ptr(a) -> C.c_void_p | None:
    """Raw pointer of a numpy array or a torch tensor (host or device); None for None."""
    if a is None:
        return None
    if hasattr(a, "data_ptr"):
        return C.c_void_p(a.data_ptr())
    return C.c_void_p(a.ctypes.data)
