"""Path workload for timings and per-kernel PMC passes (tools/pmc.sh with PMC_PROG=tools/paths_pmc.py; round 3:
tools/gpu_pmc_paths.sh): every launch reads a different batch of 1M targets (8 rotated batches).
  bench shard (1/8 of the 100M-node U(24) table): rt_ws_kernel<0, true, true> (k=8), rt_wl16_kernel<0> (k=16),
  rt_wl32q_kernel<0, true> (k=32), nc_line_kernel (NodeCache k=14), nc32_line_kernel (NodeCache k=32);
  split-policy table of 4M nodes: rt_sl_kernel<0> (k=8), rt_gl16_kernel (k=14), rt_gl32q_kernel (k=32).
Without a profiler it prints the per-launch times (HIP events, median of REPS) as JSON."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS, NB, Q = 6, 8, 1 << 20
dev = torch.device("cuda:0")
g = torch.Generator(device=dev)
g.manual_seed(9)
tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
for t in tgs:
    t[:, 0] = t[:, 0] & 0x1F  # shard 0 of the U(24) table owns the top 3 bits 000
res = {}


def run(name, fn):
    ts = []
    for j in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(tgs[j % NB])
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    res[name] = round(float(np.median(ts)), 2)


sh = build_shard(config3_spec(), 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
run("U24shard_rt_k8_us", lambda t: T.rt_closest(t, 8))
run("U24shard_rt_k16_us", lambda t: T.rt_closest(t, 16))
run("U24shard_rt_k32_us", lambda t: T.rt_closest(t, 32))
run("U24shard_nc_k14_us", lambda t: T.nc_closest(t, 14))
run("U24shard_nc_k32_us", lambda t: T.nc_closest(t, 32))
T.close()
del sh
n = 4_000_000
ids = S.random_ids(n, 0xB5)
st = S.random_status(n, 0xB6)
perm, first, off = S.split_table(ids)
T = DeviceTable(ids[perm], st[perm], first, off, device=0)
for t in tgs:
    t[:, 0] = torch.randint(0, 256, (Q,), dtype=torch.uint8, device=dev, generator=g)
run("S4M_rt_k8_us", lambda t: T.rt_closest(t, 8))
run("S4M_rt_k14_us", lambda t: T.rt_closest(t, 14))
run("S4M_rt_k32_us", lambda t: T.rt_closest(t, 32))
T.close()
print(json.dumps(res), flush=True)
