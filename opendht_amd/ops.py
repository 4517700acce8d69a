"""Batched InfoHash primitives on the GPU (infohash.h:84-146): device tensors in, device out."""
from __future__ import annotations

import ctypes as C

from ._lib import check, lib, ptr


def _stream(t):
    import torch

    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def xor_cmp(targets, a, b):
    """out[i] = targets[i].xorCmp(a[i], b[i]) in {-1, 0, 1} (int8)."""
    import torch

    n = targets.shape[0]
    out = torch.empty((n,), dtype=torch.int8, device=targets.device)
    check(lib().kad_xor_cmp_batch(ptr(targets), ptr(a), ptr(b), n, ptr(out), _stream(targets)), "kad_xor_cmp_batch")
    return out


def common_bits(a, b):
    """out[i] = InfoHash::commonBits(a[i], b[i]) (int32 view of uint32)."""
    import torch

    n = a.shape[0]
    out = torch.empty((n,), dtype=torch.int32, device=a.device)
    check(lib().kad_common_bits_batch(ptr(a), ptr(b), n, ptr(out), _stream(a)), "kad_common_bits_batch")
    return out


def lowbit(a):
    """out[i] = a[i].lowbit(); 0xFFFFFFFF for the zero ID (int32 view of uint32)."""
    import torch

    n = a.shape[0]
    out = torch.empty((n,), dtype=torch.int32, device=a.device)
    check(lib().kad_lowbit_batch(ptr(a), n, ptr(out), _stream(a)), "kad_lowbit_batch")
    return out


def parse_nodes(records, rec_len: int, myid: bytes):
    """NetworkEngine::deserializeNodes' filter (network_engine.cpp:788-828) over a device tensor of
    packed 26- or 38-byte node records: keep flags (uint8), 0 for our own ID or a martian address."""
    import numpy as np
    import torch

    n = records.numel() // rec_len
    keep = torch.empty((n,), dtype=torch.uint8, device=records.device)
    me = np.frombuffer(bytes(myid), dtype=np.uint8).copy()
    check(lib().kad_parse_nodes_batch(ptr(records), n, rec_len, ptr(me), ptr(keep), records.device.index or 0,
                                      _stream(records)), "kad_parse_nodes_batch")
    return keep


def infohash_get(data, offsets):
    """InfoHash::get (infohash.cpp:46-61) of every key: SHA-1 of data[offsets[i]:offsets[i+1]].
    data: device uint8 tensor (keys back to back), offsets: device int64 tensor (n + 1). -> (n, 20) uint8."""
    import torch

    n = offsets.shape[0] - 1
    out = torch.empty((max(n, 0), 20), dtype=torch.uint8, device=offsets.device)
    check(lib().kad_infohash_get_batch(ptr(data), ptr(offsets), n, ptr(out), offsets.device.index or 0,
                                       _stream(offsets)), "kad_infohash_get_batch")
    return out
