"""In-process A/B timing of RoutingTable kernel variants on the bench workload (one 1/8 shard
of the 100M-node table, 1M queries). Variants are selected per call through KAD_RT_KERNEL
(rounds interleaved, median reported: cdna_hip_programming.md §5.4 rule 24). Results of every
variant must be identical.

    python tools/ab_bench.py [--variants wl,lane] [--rounds 5] [--reps 10] [--count 8]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import opendht_amd._lib as _kl  # noqa: E402

_kl.use_ablation_build()  # the wl_abl* / *_abl1 timing ablations live only in the tools build
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="wl,lane")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--count", type=int, default=8)
    ap.add_argument("--queries", type=int, default=1 << 20)
    ap.add_argument("--batches", type=int, default=8, help="distinct target batches, one per launch in turn")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    spec = config3_spec()
    sh = build_shard(spec, 0)
    tgs = [torch.from_numpy(spec.targets_for(0, args.queries, seed=0x0D470002 + j)).to(dev) for j in range(args.batches)]
    targets = tgs[0]
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    variants = args.variants.split(",")
    outs = {}
    times = {v: [] for v in variants}
    stream = torch.cuda.current_stream(dev)
    for v in variants:  # warm + correctness
        os.environ["KAD_RT_KERNEL"] = v
        idx, cnt = T.rt_closest(targets, args.count)
        torch.cuda.synchronize()
        outs[v] = (idx.cpu().numpy(), cnt.cpu().numpy())
    ref = outs[variants[0]]
    same = {v: bool(np.array_equal(outs[v][0], ref[0]) and np.array_equal(outs[v][1], ref[1])) for v in variants}
    idx = torch.empty((args.queries, args.count), dtype=torch.int32, device=dev)
    cnt = torch.empty((args.queries,), dtype=torch.uint8, device=dev)
    for _ in range(args.rounds):
        for v in variants:
            os.environ["KAD_RT_KERNEL"] = v
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for r in range(args.reps):
                T.rt_closest(tgs[r % args.batches], args.count, idx, cnt, stream=stream.cuda_stream)
            e1.record(stream)
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / args.reps)
    res = {v: {"median_ms": float(np.median(times[v])), "min_ms": float(np.min(times[v])),
               "gq_per_s": args.queries / np.median(times[v]) / 1e6, "identical": same[v]} for v in variants}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
