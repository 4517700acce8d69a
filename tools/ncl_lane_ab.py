"""A/B of the count <= 14 NodeCache kernel forms on the bench shard (1M queries, 8 rotated batches): the per-lane
128-byte-line kernel in one-wave workgroups (default), aimed at six waves per SIMD (KAD_NCL2_WPE = 6) and in blocks of
four waves (KAD_NCL2_WPE = 256), and with --abl (the tools build) its
line-only ablation (lane_abl1, no wave path, results wrong), round 6's wave-loaded kernel (lines_wave) and the
number of queries each step answers (lane_stats: the line, the wave path, its serial fallback). Per form the
HIP-event median of REPS launches and a checksum of all rows; the product forms must agree with each other and with
the baseline library's checksum (tools/ncl_ab.py prints the same checksum).

    python tools/ncl_lane_ab.py [--abl]
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


def checksum(k):
    outs = [T.nc_closest(tgs[j], k) for j in range(NB)]
    torch.cuda.synchronize()
    h = 0
    for idx, cnt in outs:
        h = (h * 1000003 + int(idx.to(torch.int64).sum().item()) * 31 + int(cnt.to(torch.int64).sum().item())) % (1 << 61)
    return h


forms = [("wave1", {"KAD_NCL2_WPE": "5"}), ("wpe6", {"KAD_NCL2_WPE": "6"}), ("block4", {"KAD_NCL2_WPE": "256"})]
if ABL:
    forms += [("lane_abl1", {"KAD_NC_KERNEL": "lane_abl1"}), ("lane_abl9", {"KAD_NC_KERNEL": "lane_abl9"}),
              ("lane_abl11", {"KAD_NC_KERNEL": "lane_abl11"}),
              ("lane_abl12", {"KAD_NC_KERNEL": "lane_abl12"}), ("lines_wave", {"KAD_NC_KERNEL": "lines_wave"})]
ROUNDS = int(os.environ.get("NCL_ROUNDS", "1"))  # >1: every form again in a second pass (order effects), _r<i>
for k in (14, 8, 1):
    for rnd, (name, env) in [(r, f) for r in range(ROUNDS) for f in forms]:
        if rnd:
            name = f"{name}_r{rnd + 1}"
        for v in ("KAD_NCL2_WPE", "KAD_NC_KERNEL"):
            os.environ.pop(v, None)
        os.environ.update(env)
        T.nc_closest(tgs[0], k)
        res[f"nc_k{k}_{name}_us"] = timed(k)
        if not name.startswith("lane_abl") or name == "lane_abl12":
            res[f"nc_k{k}_{name}_sum"] = checksum(k)
    if ABL:
        os.environ.pop("KAD_NCL2_WPE", None)
        os.environ["KAD_NC_KERNEL"] = "lane_stats"
        _, st = T.nc_closest(tgs[0], k)
        res[f"nc_k{k}_steps"] = np.bincount(st.cpu().numpy(), minlength=4).tolist()
for v in ("KAD_NCL2_WPE", "KAD_NC_KERNEL"):
    os.environ.pop(v, None)
print(json.dumps(res), flush=True)
