"""Workload for per-kernel PMC passes over the non-headline paths (tools/pmc.sh with
PMC_PROG=tools/paths_pmc.py): on the bench shard (1/8 of the 100M-node U(24) table, 1M owned
queries) each path runs REPS launches, one kernel name per path, so tools/paths_roofline.py can
split the counters per kernel:
  rt_wl_kernel<0> (k=8), rt_wl16_kernel (k=16), rt_wl32_kernel (k=32), rt_closest_kernel<32> (k=32,
  KAD_RT_KERNEL=lane), nc_line_kernel (NodeCache k=14), nc_multi_kernel<2> (k=14, KAD_NC_KERNEL=multi2),
  rt_dual_wl_kernel (dual family k=8), buffer_nodes_kernel (wire records of the k=8 rows)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable, rt_closest_dual  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS = 5
dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
q = 1 << 20
tg = torch.from_numpy(spec.targets_for(0, q, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)


def run(fn, env=None):
    if env:
        os.environ[env[0]] = env[1]
    for _ in range(REPS):
        fn()
    torch.cuda.synchronize()
    if env:
        os.environ.pop(env[0])


for k in (8, 16, 32):
    run(lambda: T.rt_closest(tg, k))
run(lambda: T.rt_closest(tg, 32), ("KAD_RT_KERNEL", "lane"))
run(lambda: T.nc_closest(tg, 14))
run(lambda: T.nc_closest(tg, 14), ("KAD_NC_KERNEL", "multi2"))
af = (torch.arange(q, device=dev) % 2).to(torch.uint8)
run(lambda: rt_closest_dual(T, T, tg, af, 8))
T.set_addrs(np.random.default_rng(1).integers(0, 256, (sh.ids.shape[0], 6), dtype=np.uint8))
idx, cnt = T.rt_closest(tg, 8)
run(lambda: T.buffer_nodes(tg, idx, cnt))
T.close()
print("ok")
