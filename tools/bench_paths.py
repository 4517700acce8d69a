"""Timing of the paths besides the headline on the bench shard (1/8 of the 100M-node U(24) table,
1M owned queries): RoutingTable k = 8/14/16/32, NodeCache k = 14, dual-family k = 8/16 (both families
= the shard and a copy), bufferNodes packing of the k = 8 results. HIP events, median of rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import opendht_amd._lib as _kl  # noqa: E402

_kl.use_ablation_build()  # the wl_abl* / *_abl1 timing ablations live only in the tools build
from opendht_amd import DeviceTable, rt_closest_dual  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


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
spec = config3_spec()
sh = build_shard(spec, 0)
q = 1 << 20
tg = torch.from_numpy(spec.targets_for(0, q, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
res = {}
for k in (8, 14, 16, 32):
    us = timeit(lambda: T.rt_closest(tg, k))
    res[f"rt_k{k}_us"] = round(us, 1)
    res[f"rt_k{k}_Gq_s"] = round(q / us / 1e3, 2)
for k in (14, 16):  # ablation: the count 9..16 line kernel without its exact path
    a = T.rt_closest(tg, k)
    os.environ["KAD_RT_KERNEL"] = "wl16_abl1"
    res[f"rt_k{k}_no_exact_us"] = round(timeit(lambda: T.rt_closest(tg, k)), 1)
    c = T.rt_closest(tg, k, out_idx=torch.full((q, k), -1, dtype=torch.int32, device=dev))
    os.environ.pop("KAD_RT_KERNEL")
    torch.cuda.synchronize()
    res[f"rt_k{k}_exact_rows"] = int((c[0] != a[0]).any(dim=1).sum().item())
os.environ["KAD_RT_KERNEL"] = "lane"
for k in (16, 32):
    us = timeit(lambda: T.rt_closest(tg, k))
    res[f"rt_k{k}_lane_us"] = round(us, 1)
a = T.rt_closest(tg, 32)
os.environ.pop("KAD_RT_KERNEL")
b = T.rt_closest(tg, 32)
res["rt_k32_wl_equals_lane"] = bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]))
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
os.environ["KAD_NC_KERNEL"] = "group1"  # the binary-search + LDS-mask version, for A/B
us = timeit(lambda: T.nc_closest(tg, 14))
c = T.nc_closest(tg, 14)
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_k14_group1_us"] = round(us, 1)
res["nc_group1_equals"] = bool(torch.equal(a[0], c[0]) and torch.equal(a[1], c[1]))
os.environ["KAD_NC_KERNEL"] = "group2"  # window load, one query per wave, not pipelined
us = timeit(lambda: T.nc_closest(tg, 14))
c = T.nc_closest(tg, 14)
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_k14_group2_us"] = round(us, 1)
res["nc_group2_equals"] = bool(torch.equal(a[0], c[0]) and torch.equal(a[1], c[1]))
os.environ["KAD_NC_KERNEL"] = "multi2"  # wave per query, two queries' loads interleaved
us = timeit(lambda: T.nc_closest(tg, 14))
c = T.nc_closest(tg, 14)
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_k14_multi2_us"] = round(us, 1)
res["nc_multi2_equals"] = bool(torch.equal(a[0], c[0]) and torch.equal(a[1], c[1]))
for k in (1, 8, 16, 32):
    us = timeit(lambda: T.nc_closest(tg, k))
    res[f"nc_k{k}_us"] = round(us, 1)
a32 = T.nc_closest(tg, 32)
for kern in ("multi2", "wave64", "w64_abl1"):  # counts > 16: 32-node runs only; 64-node runs only; without the serial fallback
    os.environ["KAD_NC_KERNEL"] = kern
    res[f"nc_k32_{kern}_us"] = round(timeit(lambda: T.nc_closest(tg, 32)), 1)
    c = T.nc_closest(tg, 32, out_idx=torch.full((q, 32), -1, dtype=torch.int32, device=dev))
    os.environ.pop("KAD_NC_KERNEL")
    torch.cuda.synchronize()
    res[f"nc_k32_{kern}_rows_differ"] = int((c[0] != a32[0]).any(dim=1).sum().item())
os.environ["KAD_NC_KERNEL"] = "lines_abl1"  # ablation: the line kernel without its exact path
for k in (1, 14):
    us = timeit(lambda: T.nc_closest(tg, k))
    res[f"nc_k{k}_lines_no_exact_us"] = round(us, 1)
c = T.nc_closest(tg, 14, out_idx=torch.full((q, 14), -1, dtype=torch.int32, device=dev))
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_k14_lines_exact_rows"] = int((c[0] != a[0]).any(dim=1).sum().item())  # rows the exact path fixes
a1 = T.nc_closest(tg, 1)
os.environ["KAD_NC_KERNEL"] = "lines_abl1"
c1 = T.nc_closest(tg, 1, out_idx=torch.full((q, 1), -1, dtype=torch.int32, device=dev))
os.environ.pop("KAD_NC_KERNEL")
torch.cuda.synchronize()
res["nc_k1_lines_exact_rows"] = int((c1[0] != a1[0]).any(dim=1).sum().item())
print(json.dumps(res, indent=1))

# InfoHash primitives and the wire / hash rows: throughput and effective HBM bandwidth (bytes each
# kernel must read + write, divided by the launch time).
from opendht_amd import ops  # noqa: E402

n = 1 << 24
g = torch.Generator(device=dev).manual_seed(7)
A = torch.randint(0, 256, (n, 20), dtype=torch.uint8, device=dev, generator=g)
B = torch.randint(0, 256, (n, 20), dtype=torch.uint8, device=dev, generator=g)
Tg = torch.randint(0, 256, (n, 20), dtype=torch.uint8, device=dev, generator=g)
for name, fn, nbytes in (("xor_cmp", lambda: ops.xor_cmp(Tg, A, B), 61),
                         ("common_bits", lambda: ops.common_bits(A, B), 44),
                         ("lowbit", lambda: ops.lowbit(A), 24)):
    us = timeit(fn)
    res[f"{name}_16M_us"] = round(us, 1)
    res[f"{name}_GB_s"] = round(n * nbytes / us / 1e3, 1)
del A, B, Tg
nrec = 1 << 22
recs = torch.randint(0, 256, (nrec * 26,), dtype=torch.uint8, device=dev, generator=g)
us = timeit(lambda: ops.parse_nodes(recs, 26, b"\x01" * 20))
res["parse_nodes4_4M_us"] = round(us, 1)
res["parse_nodes4_GB_s"] = round(nrec * 27 / us / 1e3, 1)
for klen in (8, 20, 32, 55, 64, 100, 200):
    nk = 1 << 22
    data = torch.randint(0, 256, (nk * klen,), dtype=torch.uint8, device=dev, generator=g)
    offs = torch.arange(0, nk + 1, dtype=torch.int64, device=dev) * klen
    us = timeit(lambda: ops.infohash_get(data, offs))
    res[f"sha1_{klen}B_4M_us"] = round(us, 1)
    res[f"sha1_{klen}B_Ghash_s"] = round(nk / us / 1e3, 2)
print(json.dumps(res, indent=1))
