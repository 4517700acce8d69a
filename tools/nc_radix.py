"""NodeCache line tables at coarser node radixes (KAD_NC_RADIX_BITS = 21 / 22 / 23 caps the radix slots): the
line table shrinks 2x per bit (fewer TLB misses and Infinity-Cache misses per random line) while slots hold
more nodes (a target's lb shifts further into the window). getCachedNodes timings on the bench shard, 1M queries
per launch over 8 rotated batches, results compared with the 23-bit table's."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS, NB, Q = 8, 8, 1 << 20
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470100 + j)).to(dev) for j in range(NB)]
res = {}
ref = {}
for bits in (23, 22, 21, 20):
    os.environ["KAD_NC_RADIX_BITS"] = str(bits)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    os.environ.pop("KAD_NC_RADIX_BITS")
    res[f"b{bits}_radix_bits"] = T.info()["nc_radix_bits"]
    res[f"b{bits}_device_GB"] = round(T.info()["device_bytes"] / 1e9, 2)
    for k in (8, 14, 16, 24, 32):
        idx, cnt = T.nc_closest(tgs[0], k)
        torch.cuda.synchronize()
        got = (idx.cpu().numpy(), cnt.cpu().numpy())
        if bits == 23:
            ref[k] = got
        else:
            res[f"b{bits}_k{k}_identical"] = bool(np.array_equal(got[0], ref[k][0]) and np.array_equal(got[1], ref[k][1]))
        ts = []
        for j in range(REPS):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            T.nc_closest(tgs[j % NB], k, idx, cnt)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[f"b{bits}_k{k}_us"] = round(float(np.median(ts)), 1)
    T.close()
    print(json.dumps(res), flush=True)
print(json.dumps(res, indent=1))
