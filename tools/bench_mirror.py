"""Incremental mirror cost on the bench shard (1/8 of the 100M-node U(24) table, 12.5M nodes):
kad_table_apply with a batch of removals + in-bucket replacements + insertions (and a variant with
splits), against re-creating the table from host arrays (the snapshot it replaces)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd._lib import KAD_OP_INSERT, KAD_OP_REMOVE, KAD_OP_REPLACE, KAD_OP_SPLIT  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

sh = build_shard(config3_spec(), 0)
t0 = time.perf_counter()
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
torch.cuda.synchronize()
create_s = time.perf_counter() - t0
rng = np.random.default_rng(1)
n = sh.ids.shape[0]
res = {"nodes": n, "buckets": int(sh.first.shape[0]), "create_s": round(create_s, 3)}
for label, n_ops, splits in (("ops_10k", 10_000, 0), ("ops_100k", 100_000, 0), ("ops_10k_100splits", 10_000, 100)):
    pick = rng.choice(T.n, n_ops, replace=False)
    ops, nid = [], []
    for j, a in enumerate(pick):
        r = j % 3
        if r == 0:
            ops.append((KAD_OP_REMOVE, int(a), 0))
        else:
            x = rng.integers(0, 256, 20, dtype=np.uint8)
            x[0] &= 0x1F  # inside shard 0's ID range (top 3 bits 000): the node joins an owned bucket
            if r == 1:
                exp = T.export() if False else None  # noqa: F841
                ops.append((KAD_OP_INSERT, len(nid), 0))
            else:
                ops.append((KAD_OP_REMOVE, int(a), 0))
                ops.append((KAD_OP_INSERT, len(nid), 0))
            nid.append(x)
    for _ in range(splits):
        ops.append((KAD_OP_SPLIT, int(rng.integers(0, T.B)), 0))
    ops = np.array(ops, np.uint32)
    nid = np.array(nid, np.uint8)
    nst = np.ones(nid.shape[0], np.uint8)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    T.apply(ops, nid, nst)
    torch.cuda.synchronize()
    res[label + "_s"] = round(time.perf_counter() - t0, 4)
q = 1 << 20
tg = torch.from_numpy(config3_spec().targets_for(0, q, seed=5)).to(torch.device("cuda:0"))
T.rt_closest(tg, 8)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    T.rt_closest(tg, 8)
b.record()
torch.cuda.synchronize()
res["rt_k8_after_mutation_us"] = round(a.elapsed_time(b) / 10 * 1e3, 1)
res["window_lines_after"] = bool(T.info()["flags"] & 0x100)
print(json.dumps(res, indent=1))
