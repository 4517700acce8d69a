"""Where the split-policy count-32 kernel's time goes (rt_gl32q_kernel, a 4M-node split-policy table as in
tools/paths_pmc_r05.py lines mode, 1M queries over 8 rotated batches, HIP-event medians): the kernel, without its
exact path (gl32q_abl1), and the share of queries the exact path answers (gl32q_stats). Tools build."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import opendht_amd._lib as _kl  # noqa: E402

_kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd import synth as S  # noqa: E402

REPS, NB, Q = 8, 8, 1 << 20
dev = torch.device("cuda:0")
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
ids = S.random_ids(n, 0xB5)
st = S.random_status(n, 0xB6)
perm, first, off = S.split_table(ids)
T = DeviceTable(ids[perm], st[perm], first, off, device=0, eager=True)
g = torch.Generator(device=dev)
g.manual_seed(10)
tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
res = {"nodes": n, "buckets": int(first.shape[0])}
for env in (None, "gl32q_abl1"):
    if env:
        os.environ["KAD_RT_KERNEL"] = env
    idx, cnt = T.rt_closest(tgs[0], 32)
    ts = []
    for j in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        T.rt_closest(tgs[j % NB], 32, idx, cnt)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    os.environ.pop("KAD_RT_KERNEL", None)
    res[f"k32_{env or 'default'}_us"] = round(float(np.median(ts)), 1)
os.environ["KAD_RT_KERNEL"] = "gl32q_stats"
idx, cnt = T.rt_closest(tgs[0], 32)
os.environ.pop("KAD_RT_KERNEL", None)
res["k32_exact_path_share"] = float((cnt == 250).sum().item()) / Q
print(json.dumps(res), flush=True)
T.close()
