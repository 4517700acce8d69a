"""Diagnostics: per-wave timing of the exact-list kernel on the bench batch (KAD_EXACT_STAMPS=1)."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["KAD_EXACT_STAMPS"] = "1"
import opendht_amd  # noqa: E402
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import ShardSpec, build_shard  # noqa: E402

spec = ShardSpec()
sh = build_shard(spec, 0)
dev = torch.device("cuda:0")
tg = torch.from_numpy(spec.targets_for(0, 1 << 20, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
for _ in range(3):
    T.rt_closest(tg, 8)
torch.cuda.synchronize()
L = opendht_amd.lib()
buf = (C.c_uint64 * (4096 * 12))()
L.kad_debug_exact_stamps(buf, 4096 * 12)
all_ = np.frombuffer(buf, dtype=np.uint64)
a = all_[:4096 * 4].reshape(-1, 4).copy()
ph = all_[4096 * 4:].reshape(-1, 8)[:, :5].astype(np.int64)
busy = (a[:, 1] >> np.uint64(63)).astype(bool)
a[:, 1] &= np.uint64((1 << 63) - 1)
t0 = a[:, 0].min()
rel = (a - t0).astype(np.float64) / 100.0  # us (100 MHz)
res = {"waves_with_item": int(busy.sum()),
       "entry_us": [float(np.percentile(rel[:, 0], p)) for p in (0, 50, 99, 100)],
       "ctr_read_us": float(np.median(rel[:, 1] - rel[:, 0])),
       "item_us": [float(np.percentile((rel[busy, 2] - rel[busy, 1]), p)) for p in (0, 50, 90, 100)],
       "exit_us": [float(np.percentile(rel[:, 3], p)) for p in (50, 99, 100)]}
pb = ph[busy]
d = np.diff(pb, axis=1) / 100.0
res["phase_us_median"] = {n: float(np.median(d[:, k])) for k, n in enumerate(["R_probe", "dir", "nodes", "sort"])}
res["phase_us_p90"] = {n: float(np.percentile(d[:, k], 90)) for k, n in enumerate(["R_probe", "dir", "nodes", "sort"])}
res["target_us_median"] = float(np.median((pb[:, 0] - a[busy, 1].astype(np.int64)) / 100.0))
print(json.dumps(res))
