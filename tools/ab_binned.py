"""Verdict r03 item 6: does binning the targets by bucket pay on the headline? The bench shard, 1M-query batches:
  random     the headline (rotated random batches), graph of K launches
  sorted     the same batches sorted by target outside the timed region: the kernel's time when a wave's
             lines are neighbours (an upper bound on what any binning can give the query kernel itself)
  bin_cost   what a binning step costs inside the step: torch.sort of the 1M top-64 keys + the gather of the
             targets by the order (the scatter of the rows back would come on top)
Prints one JSON object."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


def timed_graph(fn, K, dev):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream(dev)
    s.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.graph(g, stream=s):
        for j in range(K):
            fn(j, s.cuda_stream)
    torch.cuda.current_stream(dev).wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) / K * 1e3)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda", 0)
    spec = config3_spec()
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    Q, NB, K = 1 << 20, 40, 40
    tgs = bench.device_targets(NB, Q, spec.shard_bits, 0, 0x0D470002, dev)
    outs = [torch.empty((Q, 8), dtype=torch.int32, device=dev) for _ in range(NB)]
    ocnt = [torch.empty((Q,), dtype=torch.uint8, device=dev) for _ in range(NB)]

    def key64(t):
        k = torch.zeros(t.shape[0], dtype=torch.int64, device=dev)
        for b in range(8):
            k = (k << 8) | t[:, b].to(torch.int64)
        return k ^ (-(2**63))  # the unsigned order as a signed one

    srt = []
    for t in tgs:
        order = torch.argsort(key64(t))
        srt.append(t[order].contiguous())
    torch.cuda.synchronize()
    res = {"queries": Q}
    res["random_us"] = timed_graph(lambda j, s: T.rt_closest(tgs[j % NB], 8, outs[j % NB], ocnt[j % NB], stream=s), K, dev)
    res["sorted_us"] = timed_graph(lambda j, s: T.rt_closest(srt[j % NB], 8, outs[j % NB], ocnt[j % NB], stream=s), K, dev)
    res["random_again_us"] = timed_graph(lambda j, s: T.rt_closest(tgs[j % NB], 8, outs[j % NB], ocnt[j % NB], stream=s),
                                         K, dev)
    # the binning step's cost: sort the top-64 keys, gather the targets
    ks = [key64(t) for t in tgs[:8]]
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for j in range(8):
        o = torch.argsort(ks[j])
        _ = tgs[j][o]
    b.record()
    torch.cuda.synchronize()
    res["bin_cost_us_sort_gather"] = a.elapsed_time(b) / 8 * 1e3
    # a cheaper bin: 16-bit histogram bins (counting sort by the top 16 bits of the shard-local key)
    a.record()
    for j in range(8):
        top = ((ks[j] ^ (-(2**63))) >> 40) & 0xFFFF
        o = torch.argsort(top, stable=False)
        _ = tgs[j][o]
    b.record()
    torch.cuda.synchronize()
    res["bin_cost_us_top16"] = a.elapsed_time(b) / 8 * 1e3
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
