"""NodeCache::getCachedNodes timings on the bench shard (1/8 of the 100M-node U(24) table, 12.5M sorted nodes),
1M queries per launch, 8 rotated target batches, median of REPS launches (HIP events): the default kernels
(256-byte lines for counts <= 16, 512-byte lines for 17..32, the two-pass wave path above) and the two-pass
wave path for 17..32 (KAD_NC_KERNEL=two_pass), results checked identical."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("NC_ABL"):
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS, NB, Q = 8, 8, 1 << 20
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470100 + j)).to(dev) for j in range(NB)]
res = {"device_bytes": T.info()["device_bytes"], "flags": T.info()["flags"]}


def timed(count, env=None):
    if env:
        os.environ["KAD_NC_KERNEL"] = env
    idx, cnt = T.nc_closest(tgs[0], count)
    torch.cuda.synchronize()
    first = (idx.cpu().numpy(), cnt.cpu().numpy())
    ts = []
    for j in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        T.nc_closest(tgs[j % NB], count, idx, cnt)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    os.environ.pop("KAD_NC_KERNEL", None)
    return float(np.median(ts)), first


for k in (14, 17, 24, 32, 40, 64):
    us, r = timed(k)
    res[f"nc_k{k}_us"] = round(us, 1)
    if 17 <= k <= 32:
        us2, r2 = timed(k, "two_pass")
        res[f"nc_k{k}_two_pass_us"] = round(us2, 1)
        res[f"nc_k{k}_identical"] = bool(np.array_equal(r[0], r2[0]) and np.array_equal(r[1], r2[1]))
    if k == 32 and os.environ.get("NC_ABL"):
        for v in ("l32_abl1", "l32_abl2"):
            res[f"nc_k32_{v}_us"] = round(timed(32, v)[0], 1)
        for kk in (17, 32):
            c = timed(kk, "l32_stats")[1][1]
            res[f"nc_k{kk}_wave_path_frac"] = float((c == 250).mean())
    print(json.dumps(res), flush=True)
