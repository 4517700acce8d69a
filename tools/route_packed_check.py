"""Owner-routed step at N = 1 on the bench shard, rows back packed and unpacked, against the direct batch: counts of
differing rows and a few examples (a diagnostic for the packed way back)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import OwnerRoute, build_shard, config3_spec  # noqa: E402

dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
Q = 1 << 20
g = torch.Generator(device=dev)
g.manual_seed(5)
t = torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g)
t[:, 0] &= 0x1F
s = torch.cuda.current_stream(dev).cuda_stream
res = {}
for k in (1, 4, 8, 14, 16, 32):
    want, wc = T.rt_closest(t, k)
    for packed in (False, True):
        R = OwnerRoute(Q, k, 1, 3, dev, packed=packed)
        oi = torch.empty((Q, k), dtype=torch.int32, device=dev)
        oc = torch.empty((Q,), dtype=torch.uint8, device=dev)
        R.step(T, t, oi, oc, None, s)
        torch.cuda.synchronize()
        bad = ((oi != want).any(1) | (oc != wc)).nonzero().flatten()
        e = {"bad_rows": int(bad.numel()), "escaped": R.escaped(combine=False), "overflow": R.overflowed(combine=False)}
        if packed:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                R.compress(s)
            b.record()
            torch.cuda.synchronize()
            e["compress_us"] = round(a.elapsed_time(b) * 100, 2)
            a.record()
            for _ in range(10):
                R.unpack_packed(oi, oc, s)
            b.record()
            torch.cuda.synchronize()
            e["unpack_packed_us"] = round(a.elapsed_time(b) * 100, 2)
        else:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(10):
                R.unpack(oi, oc, s)
            b.record()
            torch.cuda.synchronize()
            e["unpack_us"] = round(a.elapsed_time(b) * 100, 2)
        res[f"k{k} packed={packed}"] = e
print(json.dumps(res), flush=True)
T.close()
