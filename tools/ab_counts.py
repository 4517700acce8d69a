"""Per-count timing of RoutingTable::findClosestNodes on the bench shard (1M queries), window-line
kernels against the lane kernel (KAD_RT_KERNEL=lane), results checked identical."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
tg = torch.from_numpy(spec.targets_for(0, 1 << 20, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
res = {}
for k in (8, 9, 12, 14, 16):
    row = {}
    outs = {}
    for v in ("wl", "lane"):
        os.environ["KAD_RT_KERNEL"] = v
        T.rt_closest(tg, k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            idx, cnt = T.rt_closest(tg, k)
        b.record()
        torch.cuda.synchronize()
        row[v + "_us"] = round(a.elapsed_time(b) / 10 * 1e3, 1)
        outs[v] = (idx.cpu().numpy(), cnt.cpu().numpy())
    row["identical"] = bool(np.array_equal(outs["wl"][0], outs["lane"][0]) and np.array_equal(outs["wl"][1], outs["lane"][1]))
    res[f"k{k}"] = row
print(json.dumps(res, indent=1))
