"""A/B on the FULL 100M-node U(24) table on one GPU: the window-line kernel (kad_rt_closest_batch)
against the north-star shard kernel (kad_rt_shard_batch, one shard = whole table), same 1M queries.
Separates table-size effects (2.1 GB of lines) from the shard kernel's append/scatter costs."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.global_shard import GlobalShard, build_plain_shard  # noqa: E402
from opendht_amd.sharded import config3_spec  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


dev = torch.device("cuda:0")
n_shards = int(os.environ.get("NSH", "1"))
spec = config3_spec(n_shards)
ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
gp = np.concatenate([[0], np.cumsum(good)])
if n_shards > 1:  # pretend the other shards' good counts equal this one's (timing only)
    gp = np.concatenate([[0], np.cumsum(np.tile(good, n_shards))])
G = GlobalShard(ids, st, off, lo, hi, spec.depth, base, gp, device=0)
q = 1 << 20
tg = torch.from_numpy(S.random_targets(q, seed=5) if n_shards == 1 else spec.targets_for(0, q, seed=5)).to(dev)
res = {}
res["wl_kernel_us"] = timeit(lambda: G.table.rt_closest(tg, 8))
res["shard_kernel_us"] = timeit(lambda: G.local(tg, 8))
print(json.dumps(res, indent=1))
