"""Which path answers each query of the bench workload (rotated batches of the 1/8 shard, count 8): the
64-byte short line, its 128-byte fallback line, or the exact path (KAD_RT_KERNEL=ws_stats, tools build).
Prints per-query and per-wave fractions."""
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

spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
res = {}
for count in (8, 4, 1):
    fb = ex = 0
    wfb = wex = 0
    n = 0
    for j in range(4):
        tg = torch.from_numpy(spec.targets_for(0, 1 << 20, seed=0x0D470002 + j)).to("cuda:0")
        os.environ["KAD_RT_KERNEL"] = "ws_stats"
        _, cnt = T.rt_closest(tg, count)
        c = cnt.cpu().numpy()
        f, e = (c >= 100) & (c < 250), c == 250
        fb += int(f.sum()); ex += int(e.sum()); n += c.shape[0]
        wfb += int(f.reshape(-1, 64).any(1).sum()); wex += int(e.reshape(-1, 64).any(1).sum())
    res[f"k{count}"] = {"queries": n, "fallback_q": fb / n, "exact_q": ex / n, "waves_with_fallback": wfb / (n / 64),
                        "waves_with_exact": wex / (n / 64)}
print(json.dumps(res, indent=1))
