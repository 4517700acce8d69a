"""A/B of engine builds on the count <= 16 NodeCache line kernel (bench shard, 1M queries, 8 rotated batches): per
library (A B A B order comes from the caller), the HIP-event median of REPS launches per count and a checksum of all
rows, which must agree between the builds. With --abl, the ablation build's 128-byte-line-only kernel (lines_abl3,
results wrong) and round 5's 256-byte-line forms (lines_abl1 / lines_abl2) as well.

    python tools/ncl_ab.py [lib.so | --abl]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

ABL = len(sys.argv) > 1 and sys.argv[1] == "--abl"
if ABL:
    _kl.use_ablation_build()
elif len(sys.argv) > 1:
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


def timed(k):
    ts = []
    for r in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        T.nc_closest(tgs[r % NB], k)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(float(np.median(ts)), 2)


for k in (14, 8, 16, 1):
    os.environ.pop("KAD_NC_KERNEL", None)
    outs = [T.nc_closest(tgs[j], k) for j in range(NB)]
    torch.cuda.synchronize()
    res[f"nc_k{k}_us"] = timed(k)
    h = 0
    for idx, cnt in outs:
        h = (h * 1000003 + int(idx.to(torch.int64).sum().item()) * 31 + int(cnt.to(torch.int64).sum().item())) % (1 << 61)
    res[f"nc_k{k}_sum"] = h
    if ABL and k in (14, 8, 16):
        for env in ("lines_abl3", "lines_abl1", "lines_abl2") if k != 16 else ():
            os.environ["KAD_NC_KERNEL"] = env
            T.nc_closest(tgs[0], k)
            res[f"nc_k{k}_{env}_us"] = timed(k)
        os.environ["KAD_NC_KERNEL"] = "lines_stats"
        _, st = T.nc_closest(tgs[0], k)
        res[f"nc_k{k}_steps"] = np.bincount(st.cpu().numpy(), minlength=4).tolist()
        os.environ.pop("KAD_NC_KERNEL", None)
print(json.dumps(res), flush=True)
