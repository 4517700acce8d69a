"""opendht_amd — MI355X-native batched Kademlia closest-node engine for OpenDHT's lookup path.

The hot path (RoutingTable::findClosestNodes / findBucket, NodeCache::getCachedNodes and the
InfoHash XOR primitives) runs as hand-written HIP kernels for gfx950 in libkadgpu.so, behind
the C ABI of include/kadgpu.h. This package is thin Python plumbing for tests and the bench;
the drop-in host interface for OpenDHT's C++ code is include/kadgpu.hpp.
"""
from ._lib import (KAD_MAX_COUNT, KAD_NO_NODE, KAD_SEARCH_NODES, KAD_STATUS_EXPIRED, KAD_STATUS_GOOD,
                   KAD_TARGET_NODES, KadError, lib)
from .infohash import InfoHash, zeroes
from .table import DeviceTable, nc_closest_dual, rt_closest_dual

__all__ = [
    "DeviceTable", "InfoHash", "KadError", "KAD_MAX_COUNT", "KAD_NO_NODE", "KAD_SEARCH_NODES",
    "KAD_STATUS_EXPIRED", "KAD_STATUS_GOOD", "KAD_TARGET_NODES", "lib", "nc_closest_dual", "rt_closest_dual", "zeroes",
]
