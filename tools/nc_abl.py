"""Where the NodeCache line kernels' time goes (counts 8, 14 and 32, bench shard, 1M queries over 8 rotated batches, median of
REPS launches): the kernel, without its exact path (lines_abl1), and the line load + row store alone (lines_abl2,
the memory floor). Needs the tools build (make -C opendht_amd/csrc ablations); ablation results are wrong on purpose."""
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

REPS, NB, Q = 8, 8, 1 << 20
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470100 + j)).to(dev) for j in range(NB)]
res = {}
CASES = [(8, (None, "lines_abl1", "lines_abl2")), (14, (None, "lines_abl1", "lines_abl2")),
         (32, (None, "l32_abl1", "l32_abl2"))]
if len(sys.argv) > 1:  # e.g. "32": that count only
    CASES = [c for c in CASES if str(c[0]) in sys.argv[1].split(",")]
for k, envs in CASES:
    for env in envs:
        if env:
            os.environ["KAD_NC_KERNEL"] = env
        idx, cnt = T.nc_closest(tgs[0], k)
        ts = []
        for j in range(REPS):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            T.nc_closest(tgs[j % NB], k, idx, cnt)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        os.environ.pop("KAD_NC_KERNEL", None)
        res[f"nc_k{k}_{env or 'default'}_us"] = round(float(np.median(ts)), 1)
if any(k == 32 for k, _ in CASES):  # the share of count-32 queries the 512-byte lines hand to the wave path
    os.environ["KAD_NC_KERNEL"] = "l32_stats"
    idx, cnt = T.nc_closest(tgs[0], 32)
    os.environ.pop("KAD_NC_KERNEL", None)
    res["nc_k32_wave_path_share"] = float((cnt == 250).sum().item()) / Q
print(json.dumps(res, indent=1))
