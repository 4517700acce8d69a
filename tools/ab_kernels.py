"""A/B of RoutingTable kernel variants on the bench shard (1/8 of the 100M-node U(24) table): for each count,
every variant named by KAD_RT_KERNEL (read per call by the engine; "" = the default dispatch) is timed over 16
launches of 1M queries on 8 rotated target batches (HIP events), interleaved twice, and its rows must equal the
default's (except the ablations, *_abl*, whose results are wrong on purpose; RT_ABL=1 loads their build).

    python tools/ab_kernels.py 17,24,32 ,wl32lane
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("RT_ABL"):  # the timing-ablation build (make -C opendht_amd/csrc ablations): *_abl variants
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

counts = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "17,24,32").split(",")]
variants = (sys.argv[2] if len(sys.argv) > 2 else ",wl32lane").split(",")
NB, Q, REPS = 8, 1 << 20, 16
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
tgs = [torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470200 + j)).to(dev) for j in range(NB)]


def run(v, k):
    if v:
        os.environ["KAD_RT_KERNEL"] = v
    else:
        os.environ.pop("KAD_RT_KERNEL", None)
    outs = [T.rt_closest(tgs[j], k) for j in range(NB)]
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(REPS):
        T.rt_closest(tgs[j % NB], k, outs[j % NB][0], outs[j % NB][1])
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / REPS * 1e3, outs[0]


res = {}
for k in counts:
    ref = None
    for rep in range(2):
        for v in variants:
            us, (idx, cnt) = run(v, k)
            res.setdefault(f"k{k}_{v or 'default'}_us", []).append(round(us, 1))
            if ref is None:
                ref = (idx.cpu().numpy(), cnt.cpu().numpy())
            elif "_abl" not in v:
                assert np.array_equal(idx.cpu().numpy(), ref[0]) and np.array_equal(cnt.cpu().numpy(), ref[1]), (k, v)
print(json.dumps(res), flush=True)
