"""Probe of the north-star step's kernels at N = 8 on one GPU (tools only; run it under rocprofv3 --kernel-trace
--stats for per-kernel times): rank 0's shard of the 100M-node table (global buckets [0, B/8), no halo), the shard
kernel over a replicated 1M batch into 8 home blocks, and the finish (kad_rt_home_finish_reset: gather_scatter_link +
gather_merge) over 8 blocks addressed to home 0, as bench.py's n8_step_model builds them. One JSON line of event
times and row checksums.

    python tools/ns_finish_probe.py [reps]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import ctypes as C  # noqa: E402

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from opendht_amd.global_shard import GlobalShard, build_plain_shard  # noqa: E402
from opendht_amd.sharded import config3_spec  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = config3_spec(1)
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
    gp = np.concatenate([[0], np.cumsum(good.astype(np.int64))])
    B = off.shape[0] - 1
    h8 = B // 8
    n0 = int(off[h8])
    G0 = GlobalShard(ids[:n0], st[:n0], off[:h8 + 1], 0, h8, spec.depth, 0, gp, device=0)
    Q = 1 << 20
    tgs = bench.device_targets(4, Q, 0, 0, 0x0D470002, dev)
    res = {"reps": reps}
    stream = torch.cuda.current_stream(dev)
    s = C.c_void_p(stream.cuda_stream)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for k in (8, 32):
        ex = G0.exchange(Q, k, 8, True, True)
        ex.recv = bench.home0_recv(G0, ex, tgs[0], Q, dev)
        hi_q = -(-(-(-Q // 256)) // 8) * 256
        oi = torch.empty((min(hi_q, Q), k), dtype=torch.int32, device=dev)
        oc = torch.empty((min(hi_q, Q),), dtype=torch.uint8, device=dev)
        ex.home_finish(0, oi, oc, s, reset=True)
        torch.cuda.synchronize()
        a.record(stream)
        for _ in range(reps):
            ex.home_finish(0, oi, oc, s, reset=True)
        b.record(stream)
        torch.cuda.synchronize()
        res[f"finish_k{k}_us"] = a.elapsed_time(b) / reps * 1e3
        res[f"finish_k{k}_rows_sum"] = int(oi.to(torch.int64).sum().item()) * 31 + int(oc.to(torch.int64).sum().item())
        res[f"parts_received_k{k}"] = ex.parts_received()
        ctr = ex.send.view(8, ex.block)[:, ex.ctr_off:ex.ctr_off + 10 * 32]
        a.record(stream)
        for j in range(reps):
            ctr.zero_()
            G0.home_block(tgs[j % 4], ex, zeroed=True)
        b.record(stream)
        torch.cuda.synchronize()
        res[f"shard_k{k}_us_incl_zero"] = a.elapsed_time(b) / reps * 1e3
        del ex
    G0.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
