"""Timing of the paths besides the headline on the bench shard (1/8 of the 100M-node U(24) table,
1M owned queries): RoutingTable k = 8/14/16/32, NodeCache k = 14, dual-family k = 8/16 (both families
= the shard and a copy), bufferNodes packing of the k = 8 results. HIP events, median of rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable, rt_closest_dual  # noqa: E402
from opendht_amd.sharded import ShardSpec, build_shard  # noqa: E402


def timeit(fn, reps=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / reps * 1e3)
    return float(np.median(ts))


dev = torch.device("cuda:0")
spec = ShardSpec()
sh = build_shard(spec, 0)
q = 1 << 20
tg = torch.from_numpy(spec.targets_for(0, q, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
res = {}
for k in (8, 14, 16, 32):
    us = timeit(lambda: T.rt_closest(tg, k))
    res[f"rt_k{k}_us"] = round(us, 1)
    res[f"rt_k{k}_Gq_s"] = round(q / us / 1e3, 2)
us = timeit(lambda: T.nc_closest(tg, 14))
res["nc_k14_us"], res["nc_k14_Gq_s"] = round(us, 1), round(q / us / 1e3, 2)
af = (torch.arange(q, device=dev) % 2).to(torch.uint8)
for k in (8, 16):
    us = timeit(lambda: rt_closest_dual(T, T, tg, af, k))
    res[f"dual_k{k}_us"] = round(us, 1)
rng = np.random.default_rng(1)
T.set_addrs(rng.integers(0, 256, (sh.ids.shape[0], 6), dtype=np.uint8))
idx, cnt = T.rt_closest(tg, 8)
us = timeit(lambda: T.buffer_nodes(tg, idx, cnt))
res["buffer_nodes_v4_us"] = round(us, 1)
print(json.dumps(res, indent=1))
os.environ["KAD_NC_KERNEL"] = "serial"
us = timeit(lambda: T.nc_closest(tg, 14))
os.environ.pop("KAD_NC_KERNEL")
res["nc_k14_serial_us"] = round(us, 1)
a = T.nc_closest(tg, 14)
os.environ["KAD_NC_KERNEL"] = "serial"
b = T.nc_closest(tg, 14)
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_group_equals_serial"] = bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]))
print(json.dumps(res, indent=1))
