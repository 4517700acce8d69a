"""Where the time of bench.py's `live` object goes (round 4): the bench shard with live-table node times, then
  graph    K query steps as one HIP graph (the headline's form)
  eager    K eager query steps through direct ctypes calls (no refresh)
  live     K steps of refresh_status(now = start + elapsed) + one query batch, direct ctypes, no events
  live_ev  the same with HIP events around every refresh (bench.py's form)
  tick     single refreshes passing 1, 4, 16, 64, 256 deadlines: GPU time between events and host time
Prints one JSON object. Usage: python tools/live_diag.py [K]"""
import ctypes as C
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
from opendht_amd._lib import lib  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    dev = torch.device("cuda", 0)
    spec = config3_spec()
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    Q, NB = 1 << 20, 64
    tgs = bench.device_targets(NB, Q, spec.shard_bits, 0, 0x0D470002, dev)
    outs = [torch.empty((Q, 8), dtype=torch.int32, device=dev) for _ in range(NB)]
    ocnt = [torch.empty((Q,), dtype=torch.uint8, device=dev) for _ in range(NB)]
    stream = torch.cuda.current_stream(dev)
    s = C.c_void_p(stream.cuda_stream)
    L = lib()
    h = T._h
    rt, rf = L.kad_rt_closest_batch, L.kad_table_refresh_status
    P = [(C.c_void_p(tgs[j].data_ptr()), C.c_void_p(outs[j].data_ptr()), C.c_void_p(ocnt[j].data_ptr()))
         for j in range(NB)]
    now = 10**15
    t, r, ex = bench.node_times(sh.status, now)
    T.set_times(t, r, ex)
    T.refresh_status(now, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    MIN = 60 * 10**9
    D = np.unique(np.minimum(t + 10 * MIN, r + 120 * MIN)[ex == 0])
    res = {}

    # graph
    g = torch.cuda.CUDAGraph()
    cs = torch.cuda.Stream(dev)
    cs.wait_stream(stream)
    with torch.cuda.graph(g, stream=cs):
        for j in range(K):
            rt(h, P[j % NB][0], Q, 8, P[j % NB][1], P[j % NB][2], C.c_void_p(cs.cuda_stream))
    stream.wait_stream(cs)
    g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    res["graph_us_per_step"] = (time.perf_counter() - t0) / K * 1e6

    def eager(with_refresh, events):
        nonlocal now
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
        torch.cuda.synchronize()
        start = now
        host = 0.0
        t0 = time.perf_counter()
        for j in range(K):
            a = time.perf_counter()
            if with_refresh:
                now = start + int((a - t0) * 1e9)
                if events:
                    evs[j][0].record(stream)
                assert rf(h, C.c_int64(now), s) == 0
                if events:
                    evs[j][1].record(stream)
            tp, op, cp = P[j % NB]
            assert rt(h, tp, Q, 8, op, cp, s) == 0
            host += time.perf_counter() - a
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        out = {"us_per_step": wall / K * 1e6, "host_issue_us_per_step": host / K * 1e6}
        if with_refresh:
            out["deadlines_passed"] = int(np.searchsorted(D, now) - np.searchsorted(D, start))
        if events:
            rfms = np.array([a.elapsed_time(b) for a, b in evs])
            out["refresh_event_us_median"] = float(np.median(rfms)) * 1e3
            out["refresh_event_us_max"] = float(rfms.max()) * 1e3
        now += 1
        return out

    eager(False, False)
    res["eager"] = eager(False, False)
    res["live"] = eager(True, False)
    res["live_ev"] = eager(True, True)
    # single refreshes passing k deadlines: GPU time between events, host time of the call
    ticks = {}
    for k in (0, 1, 4, 16, 64, 100, 128, 256, 2048):
        i0 = int(np.searchsorted(D, now, "right"))
        target = now + 1 if k == 0 else int(D[i0 + k - 1]) + 1
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        tp, op, cp = P[k % NB]  # queued behind a query batch: the events bracket the refresh's device time
        assert rt(h, tp, Q, 8, op, cp, s) == 0
        a.record(stream)
        h0 = time.perf_counter()
        assert rf(h, C.c_int64(target), s) == 0
        h1 = time.perf_counter()
        b.record(stream)
        torch.cuda.synchronize()
        ticks[str(k)] = {"event_us": a.elapsed_time(b) * 1e3, "host_us": (h1 - h0) * 1e6}
        now = target
    res["ticks"] = ticks
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
