"""A/B of two engine builds on NodeCache count 32 and RoutingTable count 32 (bench shard; a 4M-node split-policy
table): run once per
library, alternately (A B A B), under rocprofv3 --kernel-trace for the kernel durations; each run prints the HIP-event
median of 16 launches of 1M queries (bench shard, 8 rotated batches) and a checksum of the rows, which must agree
between the builds.

    python tools/nc32_ab.py opendht_amd/libkadgpu_prev.so
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

if len(sys.argv) > 1:
    _kl.use_library(sys.argv[1])
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS, NB, Q = 16, 8, 1 << 20
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470100 + j)).to(dev) for j in range(NB)]
res = {"lib": _kl.LIB_PATH}
for k in (32, 24, 20, 14, 16):
    outs = [T.nc_closest(tgs[j], k) for j in range(NB)]
    torch.cuda.synchronize()
    ts = []
    for r in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        T.nc_closest(tgs[r % NB], k)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    h = 0
    for idx, cnt in outs:
        h = (h * 1000003 + int(idx.to(torch.int64).sum().item()) * 31 + int(cnt.to(torch.int64).sum().item())) % (1 << 61)
    res[f"nc_k{k}_us"] = round(float(np.median(ts)), 2)
    res[f"nc_k{k}_sum"] = h
for name, tab in (("rt", T), ("split_rt", None)):
    if tab is None:  # a 4M-node split-policy table (tools/paths_pmc_r05.py lines mode): rt_gl32q_kernel
        from opendht_amd import synth as S
        ids = S.random_ids(4_000_000, 0xB5)
        st = S.random_status(4_000_000, 0xB6)
        perm, first, off = S.split_table(ids)
        tab = DeviceTable(ids[perm], st[perm], first, off, device=0, eager=True)
    outs = [tab.rt_closest(tgs[j], 32) for j in range(NB)]
    torch.cuda.synchronize()
    ts = []
    for r in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        tab.rt_closest(tgs[r % NB], 32)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    h = 0
    for idx, cnt in outs:
        h = (h * 1000003 + int(idx.to(torch.int64).sum().item()) * 31 + int(cnt.to(torch.int64).sum().item())) % (1 << 61)
    res[f"{name}_k32_us"] = round(float(np.median(ts)), 2)
    res[f"{name}_k32_sum"] = h
    if tab is not T:
        tab.close()
T.close()
print(json.dumps(res), flush=True)
