"""A/B timing of the north-star shard kernel between engine builds (run once per library, alternately, under
rocprofv3 --kernel-trace --stats; tools/gpu_shard_ab.sh): rank 0 of 8 of the 100M-node table, the replicated 1M
batch, 60 launches each of
  reach0 : a batch none of whose targets rank 0 can reach, back to back (kad_rt_shard_step_home, nothing appended)
  k8, k16, k32: 8 rotated uniform batches into the 8 home blocks (kad_rt_shard_batch_home: counters zeroed by the call)
and the first launch's rows checked equal between builds through a digest of the sorted rows.

    python tools/shard_ab.py [lib.so]
"""
import hashlib
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
from opendht_amd.global_shard import GlobalShard, build_plain_shard  # noqa: E402
from opendht_amd.sharded import config3_spec  # noqa: E402

Q, NB, R = 1 << 20, 8, 60
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
far = [t.clone() for t in tgs]
for t in far:
    t[:, 0] |= 0x80  # beyond rank 0's reach
res = {"lib": _kl.LIB_PATH}


def events(fn):
    fn(0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(R):
        fn(j)
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1e3 / R, 2)


ex = G0.exchange(Q, 8, 8)
ctr = ex.send.view(8, ex.block)[:, ex.ctr_off:ex.ctr_off + 10 * 32]
ctr.zero_()
res["reach0_events_us"] = events(lambda j: G0.home_block(far[j % NB], ex, zeroed=True))
res["reach0_appended"] = int(ctr.sum())
for k in (8, 16, 32):
    ex = G0.exchange(Q, k, 8)
    ctr = ex.send.view(8, ex.block)[:, ex.ctr_off:ex.ctr_off + 10 * 32]
    G0.home_block(tgs[0], ex)
    torch.cuda.synchronize()
    # the digest of every home block's appended rows and parts, in a canonical order (rows carry their qid)
    h = hashlib.sha1()
    rw = 4 + (k + 3) // 4 * 4
    for d in range(8):
        blk = ex.send.view(8, ex.block)[d]
        c = ctr[d].view(10, 32)[:, 0].cpu().numpy().view(np.uint32)
        rows = []
        for r in range(8):
            n = int(min(c[r], ex.row_cap))
            seg = blk[(r * ex.row_cap) * rw:(r * ex.row_cap + n) * rw].view(n, rw).cpu().numpy().view(np.uint32)
            rows.append(seg[seg[:, 0] != 0xFFFFFFFF])
        rows = np.concatenate(rows)
        h.update(rows[np.lexsort(rows.T[::-1])].tobytes())
        h.update(c[8:10].tobytes())
    res[f"k{k}_digest"] = h.hexdigest()[:16]
    res[f"k{k}_overflow"] = int(ctr[:, 9 * 32].max())
    res[f"k{k}_events_us"] = events(lambda j: G0.home_block(tgs[j % NB], ex))
G0.close()
print(json.dumps(res), flush=True)
