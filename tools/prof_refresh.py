"""Incremental status refresh on the bench shard (1/8 of the 100M-node U(24) table), for a rocprofv3
kernel trace: refresh_status(now) with `now` below the next deadline (no GPU work), ticks of 1 ms .. 10 s
over a live table's deadlines (good nodes heard over the last 10 minutes), patch_times-driven ageing
(0.001 % / 0.1 % / 1 % of the good nodes), then patch_status lists of the same sizes.

    rocprofv3 --kernel-trace --stats -d gpurun_out/x -o run -- python3 tools/prof_refresh.py
"""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import node_times  # noqa: E402
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

sh = build_shard(config3_spec(), 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
now = 10**15
t, rt, ex = node_times(sh.status, now)
T.set_times(t, rt, ex)
T.refresh_status(now)
torch.cuda.synchronize()
rng = np.random.default_rng(1)
res = {}


def wall(fn):
    torch.cuda.synchronize()
    a = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    return round((time.perf_counter() - a) * 1e3, 4)


for j in range(3):
    res.setdefault("no_flip_ms", []).append(wall(lambda: T.refresh_status(now + 1 + j)))
now += 10
for dt_ms in (1, 10, 100, 1000, 10000):
    for rep in range(2):
        now += dt_ms * 10**6
        res.setdefault(f"tick_{dt_ms}ms", []).append(wall(lambda: T.refresh_status(now)))
good = np.flatnonzero(T.export_status() & 1).astype(np.uint32)
for frac in (0.00001, 0.001, 0.01):
    for rep in range(2):
        sel = rng.choice(good, size=max(1, int(good.shape[0] * frac)), replace=False).astype(np.uint32)
        now += 10**6
        T.patch_times(sel, np.full(sel.shape[0], now - 10 * 60 * 10**9 - 1, np.int64),
                      np.full(sel.shape[0], now, np.int64), np.zeros(sel.shape[0], np.uint8))
        res.setdefault(f"ageing_{frac:g}_ms", []).append(wall(lambda: T.refresh_status(now)))
        T.patch_times(sel, np.full(sel.shape[0], now, np.int64), np.full(sel.shape[0], now, np.int64),
                      np.zeros(sel.shape[0], np.uint8))
        T.refresh_status(now)
        torch.cuda.synchronize()
n = sh.ids.shape[0]
st = T.export_status()
for frac in (0.00001, 0.001, 0.01, 0.1):
    nodes = rng.choice(n, size=max(1, int(n * frac)), replace=False).astype(np.uint32)
    res[f"patch_{frac:g}_ms"] = wall(lambda: T.patch_status(nodes, st[nodes] ^ np.uint8(1)))
    T.patch_status(nodes, st[nodes])
print(res)
