"""The share of count-16 / count-14 queries the 128-byte count-16 window lines cannot answer (bench shard, 1M queries,
tools build wl16_stats), with the good-node totals of the queries' windows W(1), W(2) (from the line headers' view:
the oracle's window sizes) for those queries."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

_kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

Q = 1 << 20
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tg = torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470200)).to(dev)
res = {}
os.environ["KAD_RT_KERNEL"] = "wl16_stats"
for k in (9, 12, 14, 16):
    idx, cnt = T.rt_closest(tg, k)
    res[f"k{k}_line_miss_share"] = float((cnt == 250).sum().item()) / Q
os.environ.pop("KAD_RT_KERNEL", None)
print(json.dumps(res), flush=True)
T.close()
