"""A/B timing of the owner-routing kernels of an engine build (tools/gpu_nc32_ab.sh-style: run once per library,
alternately): kad_route_pack of 1M targets into N = 2, 4, 8 blocks, kad_route_compress and kad_route_unpack_packed
(k = 8), HIP-event medians of 20 launches over 8 rotated batches.

    python tools/route_ab.py [lib.so]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

if len(sys.argv) > 1:
    _kl.use_library(sys.argv[1])
from opendht_amd.sharded import OwnerRoute  # noqa: E402

Q, NB, REPS = 1 << 20, 8, 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(3)
tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
s = torch.cuda.current_stream(dev).cuda_stream
res = {"lib": _kl.LIB_PATH}


def med(fn):
    fn(0)
    torch.cuda.synchronize()
    ts = []
    for r in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(r)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return round(float(np.median(ts)), 2)


for n in (2, 4, 8):
    RK = OwnerRoute(Q, 8, n, 3, dev, collective=False, keys=True)
    res[f"pack_keys_n{n}_us"] = med(lambda r: RK.pack(tgs[r % NB], s))
    assert not RK.overflowed(combine=False)
    del RK
    R = OwnerRoute(Q, 8, n, 3, dev, collective=False, keys=False)
    res[f"pack_n{n}_us"] = med(lambda r: R.pack(tgs[r % NB], s))
    assert not R.overflowed(combine=False)
R.rows.random_(0, 1 << 20)
R.cnt.fill_(8)
R.rows[:, 1:] = R.rows[:, :1] + torch.arange(1, 8, device=dev, dtype=torch.int32)
res["compress_k8_us"] = med(lambda r: R.compress(s))
oi = torch.empty((Q, 8), dtype=torch.int32, device=dev)
oc = torch.empty((Q,), dtype=torch.uint8, device=dev)
res["unpack_packed_k8_us"] = med(lambda r: R.unpack_packed(oi, oc, s))
res["unpack_k8_us"] = med(lambda r: R.unpack(oi, oc, s))
print(json.dumps(res), flush=True)
