"""Probe of the native executor's overlap at world 1 (tools only): config 3's rank-0 shard, 1M targets per batch,
kad_route_run serial (one set) and pipelined (three sets) over K batches, and the pieces alone (pack, query, unpack,
the one-rank ncclAllToAll copies) timed with HIP events; one JSON line. Run it in a fresh process per environment
(e.g. GPU_MAX_HW_QUEUES) to see whether the compute and comm streams share a hardware queue.

    python tools/native_pipe_probe.py [K]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.comm import Comm, NativeRoute  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    spec = config3_spec()
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    Q = 1 << 20
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    tgs = []
    for _ in range(4):
        t = torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g)
        t[:, 0] &= 0x1F
        tgs.append(t)
    outs = [(torch.empty((Q, 8), dtype=torch.int32, device=dev), torch.empty((Q,), dtype=torch.uint8, device=dev))
            for _ in range(4)]
    res = {"env": {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES",)}, "K": K}
    with Comm(0, 1, 0) as comm:
        for name, n in (("serial", 1), ("pipelined", 3), ("pipelined5", 5)):
            R = NativeRoute(Q, 8, 1, 3, dev, n_sets=n, comm=comm)
            R.run(T, tgs[:3], outs[:3])
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                R.run(T, [tgs[j % 4] for j in range(K)], [outs[j % 4] for j in range(K)])
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) / K * 1e6)
            res[name + "_us"] = min(ts)
            res[name + "_flags"] = R.flags()
        # the pieces on one stream, HIP events
        R = NativeRoute(Q, 8, 1, 3, dev, n_sets=1, comm=comm)
        S = R.sets[0]
        s = torch.cuda.current_stream(dev).cuda_stream
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def timed(fn, n=10):
            fn()
            torch.cuda.synchronize()
            a.record()
            for _ in range(n):
                fn()
            b.record()
            b.synchronize()
            return a.elapsed_time(b) / n * 1e3

        res["pack_us"] = timed(lambda: S.pack(tgs[0], s))
        res["a2a_targets_us"] = timed(lambda: comm.all_to_all(S.recv, S.send))
        res["query_packed_us"] = timed(lambda: S.answer(T, s))
        res["a2a_rows_us"] = timed(lambda: comm.all_to_all(S.back_prow, S.prow))
        res["unpack_us"] = timed(lambda: S.unpack_packed(*outs[0], s))
        res["d2d_copy_targets_us"] = timed(lambda: S.recv.copy_(S.send))
    T.close()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
