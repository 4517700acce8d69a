"""kad_rt_closest_batch_host on the bench shard, 1M pageable targets, k = 8: wall time per call with the output
arrays reused (pre-touched) and with fresh np.empty outputs (first-touch page faults in the timed call); median of
5. RT_ABL=1 times libkadgpu_abl.so instead (A/B against another build)."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("RT_ABL"):
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd._lib import check, lib, ptr  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

spec = config3_spec()
sh = build_shard(spec, 0)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
Q, K = 1 << 20, 8
tg = np.ascontiguousarray(spec.targets_for(0, Q, seed=0x0D470002))
res = {}
for mode in ("reused", "fresh"):
    idx = np.zeros((Q, K), np.uint32)
    cnt = np.zeros((Q,), np.uint8)
    ts = []
    for r in range(6):
        if mode == "fresh":
            idx = np.empty((Q, K), np.uint32)
            cnt = np.empty((Q,), np.uint8)
        t0 = time.perf_counter()
        check(lib().kad_rt_closest_batch_host(T.handle, ptr(tg), Q, K, ptr(idx), ptr(cnt)), "host")
        ts.append(time.perf_counter() - t0)
    res[f"{mode}_ms"] = round(float(np.median(ts[1:])) * 1e3, 2)
    res[f"{mode}_Gq_s"] = round(Q / float(np.median(ts[1:])) / 1e9, 3)
t0 = time.perf_counter()
a = tg.copy()
res["memcpy_targets_ms"] = round((time.perf_counter() - t0) * 1e3, 2)
print(json.dumps(res), flush=True)
