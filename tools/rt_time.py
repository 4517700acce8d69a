"""RoutingTable::findClosestNodes timings on the bench shard (1/8 of the 100M-node U(24) table), 1M queries per
launch over 8 rotated target batches, HIP events around 16 launches: counts 8, 14, 16, 17, 24, 32 (the 64-byte,
128-byte and 256-byte window lines). RT_SPLIT=1 adds a 4M-node split-policy table (the general lines): counts 8, 14, 32."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("RT_ABL"):  # A/B against another build placed as libkadgpu_abl.so
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

NB, Q, REPS = 8, 1 << 20, 16
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470200 + j)).to(dev) for j in range(NB)]
res = {}
for k in (8, 14, 16, 17, 24, 32):
    outs = [T.rt_closest(tgs[j], k) for j in range(NB)]
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(REPS):
        T.rt_closest(tgs[j % NB], k, outs[j % NB][0], outs[j % NB][1])
    b.record()
    torch.cuda.synchronize()
    res[f"rt_k{k}_us"] = round(a.elapsed_time(b) / REPS * 1e3, 1)
if os.environ.get("RT_SPLIT"):
    from opendht_amd import synth as S  # noqa: E402

    T.close()
    del sh
    n = 4_000_000
    ids, st = S.random_ids(n, 0xB5), S.random_status(n, 0xB6)
    perm, first, off = S.split_table(ids)
    T = DeviceTable(ids[perm], st[perm], first, off, device=0)
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
    for k in (8, 14, 32):
        outs = [T.rt_closest(tgs[j], k) for j in range(NB)]
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for j in range(REPS):
            T.rt_closest(tgs[j % NB], k, outs[j % NB][0], outs[j % NB][1])
        b.record()
        torch.cuda.synchronize()
        res[f"split4M_k{k}_us"] = round(a.elapsed_time(b) / REPS * 1e3, 1)
print(json.dumps(res), flush=True)
