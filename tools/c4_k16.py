"""Config 4's count-16 cost: single-family k = 14 / 16 on its v4 table (1M nodes, U(17)) against the dual batch, and
(RT_ABL=1 with KAD_RT_KERNEL=wl16_abl1) the single-family kernel without its wave / exact fallbacks."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("RT_ABL"):
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.table import rt_closest_dual  # noqa: E402

dev = torch.device("cuda:0")


def uniform(n, depth, seed):  # bench.py's config-4 tables
    ids, _ = S.sort_ids(S.random_ids(n, seed))
    st = S.random_status(n, S.SEED_STATUS ^ seed)
    first, off = S.uniform_buckets(ids, depth)
    return ids, st, first, off


fam = [uniform(1_000_000, 17, seed) for seed in (0xC4F4, 0xC4F6)]
Q = 1 << 20
db = [torch.from_numpy(S.random_targets(Q, seed=0x0D4704C4 + j)).to(dev) for j in range(4)]
da = torch.from_numpy((np.arange(Q) % 2).astype(np.uint8)).to(dev)
T4 = DeviceTable(*fam[0], device=0, sorted=True)
T6 = DeviceTable(*fam[1], device=0, sorted=True)


def med(fn, reps=12):
    ts = []
    for r in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(r)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(float(np.median(ts)), 1)


res = {}
for k in (8, 14, 16):
    outs = [T4.rt_closest(db[j], k) for j in range(4)]
    res[f"v4_k{k}_us"] = med(lambda r: T4.rt_closest(db[r % 4], k, outs[r % 4][0], outs[r % 4][1]))
    if not os.environ.get("RT_ABL"):
        res[f"dual_k{k}_us"] = med(lambda r: rt_closest_dual(T4, T6, db[r % 4], da, k))
print(json.dumps(res), flush=True)
