"""The north-star shard kernel's "nothing in reach" case beside the bare batch load (tools/mb_stream.hip), on one
box in one call: rank 0 of 8 of the 100M-node table, a replicated 1M batch none of whose targets rank 0 can reach,
200 launches back to back (kad_rt_shard_step_home: no counter zeroing between them, nothing is appended), on the
tools build with KAD_SHARD_ABL = 0 (the product kernel) and 8 (the target load alone). Run under
rocprofv3 --kernel-trace; the kernel durations are read from the trace (tools/shard_floor_table.py)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opendht_amd import _lib  # noqa: E402

_lib.use_ablation_build()
from opendht_amd.global_shard import GlobalShard, build_plain_shard  # noqa: E402
from opendht_amd.sharded import config3_spec  # noqa: E402

Q, NB, R = 1 << 20, 8, 200
dev = torch.device("cuda:0")
spec = config3_spec(1)
ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
gp = np.concatenate([[0], np.cumsum(good.astype(np.int64))])
h8 = (off.shape[0] - 1) // 8
n0 = int(off[h8])
G0 = GlobalShard(ids[:n0], st[:n0], off[:h8 + 1], 0, h8, spec.depth, 0, gp, device=0)
del ids, st
g = torch.Generator(device=dev)
g.manual_seed(13)
far = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
for t in far:
    t[:, 0] |= 0x80  # beyond rank 0's reach
ex = G0.exchange(Q, 8, 8)
ctr = ex.send.view(8, ex.block)[:, ex.ctr_off:ex.ctr_off + 10 * 32]
ctr.zero_()
res = {}
for abl in ("0", "8"):
    os.environ["KAD_SHARD_ABL"] = abl
    for j in range(20):
        G0.home_block(far[j % NB], ex, zeroed=True)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(R):
        G0.home_block(far[j % NB], ex, zeroed=True)
    b.record()
    torch.cuda.synchronize()
    res[f"reach0_abl{abl}_us_per_launch_events"] = round(a.elapsed_time(b) * 1e3 / R, 2)
os.environ.pop("KAD_SHARD_ABL")
res["appended_or_overflow"] = int(ctr.sum())
G0.close()
print(json.dumps(res), flush=True)
