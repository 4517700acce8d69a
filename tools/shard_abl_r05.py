"""Where the north-star shard kernel's time goes (round 5): rank 0 of 8 of the 100M-node table, the replicated 1M
batch, k = 8, 16 and 32, run on the tools build (libkadgpu_abl.so) with KAD_SHARD_ABL = 0 (the product kernel), 16
(2,048 queries per workgroup instead of 1,024; 18 = 2 + 16), 1 (no
wave path: the edge queries dropped), 2 (no line work either: the target load and the reach compaction alone), 6 (2
with plain target loads), 8 (the target load alone), 12 (8 with plain loads).
Results are wrong on purpose for 1 and 2. Run under rocprofv3 --kernel-trace for the kernel durations; prints the
event times as JSON."""
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

Q, NB, REPS = 1 << 20, 8, 6
dev = torch.device("cuda:0")
spec = config3_spec(1)
ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
gp = np.concatenate([[0], np.cumsum(good.astype(np.int64))])
h8 = (off.shape[0] - 1) // 8
n0 = int(off[h8])
G0 = GlobalShard(ids[:n0], st[:n0], off[:h8 + 1], 0, h8, spec.depth, 0, gp, device=0)
del ids, st
g = torch.Generator(device=dev)
g.manual_seed(11)
tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
res = {}
for k in (8, 16, 32):
    ex = G0.exchange(Q, k, 8)
    ctr = ex.send.view(8, ex.block)[:, ex.ctr_off:ex.ctr_off + 10 * 32]
    for abl in (("0", "16", "1", "2", "18", "6", "8", "12") if k == 8 else ("0", "16", "1", "2")):
        os.environ["KAD_SHARD_ABL"] = abl
        ts = []
        for j in range(REPS):
            ctr.zero_()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            G0.home_block(tgs[j % NB], ex, zeroed=True)
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        res[f"k{k}_abl{abl}_event_us"] = round(float(np.median(ts)), 2)
        if abl in ("0", "16"):
            res[f"k{k}_abl{abl}_overflow"] = int(ctr[:, 9 * 32].max())
os.environ.pop("KAD_SHARD_ABL")
G0.close()
print(json.dumps(res), flush=True)
