"""RoutingTable::findClosestNodes on split-policy (S) tables against uniform-depth (U) tables of the same
size: general window lines (rt_gl_kernel / rt_gl32_kernel) vs the lane kernel (KAD_RT_KERNEL=lane), and
the U table's uniform lines, 1M queries per launch over 8 rotated target batches (results of the two S
paths must be identical).

    python tools/bench_shapes.py [n_nodes ...]   -> JSON, us per 1M queries
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import opendht_amd._lib as _kl  # noqa: E402

if os.environ.get("SHAPES_ABL"):
    _kl.use_ablation_build()
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd import synth as S  # noqa: E402

dev = torch.device("cuda:0")
Q, NB = 1 << 20, 8
g = torch.Generator(device=dev)
g.manual_seed(5)
tgs = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
outs = {k: [torch.empty((Q, k), dtype=torch.int32, device=dev) for _ in range(NB)] for k in (8, 14, 16, 32)}


def timeit(T, k, reps=24):
    for j in range(NB):
        T.rt_closest(tgs[j], k, outs[k][j])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(reps):
        T.rt_closest(tgs[j % NB], k, outs[k][j % NB])
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


res = {}
for n in [int(x) for x in sys.argv[1:]] or [1_000_000, 12_500_000]:
    t0 = time.perf_counter()
    ids = S.random_ids(n, 0xB5)
    st = S.random_status(n, 0xB6)
    perm, first, off = S.split_table(ids)
    res[f"S{n}_build_s"] = round(time.perf_counter() - t0, 1)
    T = DeviceTable(ids[perm], st[perm], first, off, device=0)
    inf = T.info()
    res[f"S{n}_buckets"] = inf["n_buckets"]
    res[f"S{n}_flags"] = hex(inf["flags"])
    if os.environ.get("SHAPES_ABL"):  # k = 8: slot lines alone (results wrong), the 128-byte general lines alone
        for v in ("sl_abl1", "gl"):
            os.environ["KAD_RT_KERNEL"] = v
            res[f"S{n}_k8_only_{v}_us"] = round(timeit(T, 8), 1)
            os.environ.pop("KAD_RT_KERNEL")
    for k in (8, 14, 16, 32):
        res[f"S{n}_k{k}_gl_us"] = round(timeit(T, k), 1)
        a = T.rt_closest(tgs[0], k)[0].clone()
        os.environ["KAD_RT_KERNEL"] = "lane"
        res[f"S{n}_k{k}_lane_us"] = round(timeit(T, k), 1)
        c = T.rt_closest(tgs[0], k)[0].clone()
        os.environ.pop("KAD_RT_KERNEL")
        torch.cuda.synchronize()
        res[f"S{n}_k{k}_equal"] = bool(torch.equal(a, c))
        if k in (14, 16):  # the gl16 lines without their slot copies (gl), the 256-byte count 9..32 lines (gl32)
            for env in ("gl", "gl32"):
                os.environ["KAD_RT_KERNEL"] = env
                res[f"S{n}_k{k}_{env}_only_us"] = round(timeit(T, k), 1)
                c = T.rt_closest(tgs[0], k)[0].clone()
                os.environ.pop("KAD_RT_KERNEL")
                torch.cuda.synchronize()
                res[f"S{n}_k{k}_{env}_only_equal"] = bool(torch.equal(a, c))
    # dual-family batch (af alternating, the table as both families): rt_dual_gl_kernel vs the lane kernel
    from opendht_amd import rt_closest_dual
    afd = (torch.arange(Q, device=dev) % 2).to(torch.uint8)
    for k in (8, 14, 32):
        for j in range(NB):
            rt_closest_dual(T, T, tgs[j], afd, k)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for j in range(24):
            rt_closest_dual(T, T, tgs[j % NB], afd, k)
        b.record()
        torch.cuda.synchronize()
        res[f"S{n}_dual_k{k}_us"] = round(a.elapsed_time(b) / 24 * 1e3, 1)
    T.close()
    sid, _ = S.sort_ids(ids)
    d = max(1, int(round(np.log2(n / 8))))
    fu, ou = S.uniform_buckets(sid, d)
    U = DeviceTable(sid, st, fu, ou, device=0)
    for k in (8, 16, 32):
        res[f"U{d}_{n}_k{k}_wl_us"] = round(timeit(U, k), 1)
    U.close()
    print(json.dumps(res), flush=True)
print(json.dumps(res, indent=1))
