"""Round-6 path workload for per-kernel timings and PMC passes (tools/gpu_pmc_r06.sh; round 5's tools/paths_pmc_r05.py
with the round-6 owner-routing kernels: the 20-byte and the key-only pack, the owner's packed query from 20-byte
targets and from 8-byte keys, the packed unpack with and without the counter fold). One mode per run, so that each
rocprofv3 --pmc pass stays short:
  lines    bench shard (1/8 of the 100M-node U(24) table): rt_ws_kernel (k=8), rt_wl16_kernel (k=16),
           rt_wl32q_kernel (k=32), nc_line_kernel (NodeCache k=14), nc32_line_kernel (NodeCache k=32);
           split-policy table of 4M nodes: rt_sl_kernel (k=8), rt_sl16_kernel (k=14), rt_gl32q_kernel (k=32)
  shard    the north-star step at N = 8 on rank 0's shard of the 100M-node table: rt_shard_kernel over the replicated
           1M batch into 8 home blocks (k = 8 and 32), gather_scatter_link_kernel + gather_merge_kernel over 8 blocks
  swarm    config 5 at 2M peers, 10 % offline: search_init / search_query / search_merge over 256k lookups to convergence
  swarm0   the same with every peer online (the 16-register merge)
  refresh  the live refresh: rf_nodes_kernel over 300 refreshes of the bench shard at a moving `now`
  route    the owner-routed serving form: route_pack_kernel (N = 8), route_unpack_kernel (k = 8), the owner's query with
           packed rows (rt_ws_packed_kernel) over 8 received blocks, route_unpack_packed4_kernel
Every launch reads a different batch (8 rotated batches of 1M targets). Prints the per-launch times (HIP events,
median of REPS) as one JSON object."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

REPS, NB, Q = 6, 8, 1 << 20
dev = torch.device("cuda:0")
res = {}


def batches(top3=None, seed=9):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    out = [torch.randint(0, 256, (Q, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
    if top3 is not None:
        for t in out:
            t[:, 0] = (t[:, 0] & 0x1F) | (top3 << 5)
    return out


def run(name, fn, tgs):
    ts = []
    for j in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(tgs[j % NB])
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    res[name] = round(float(np.median(ts)), 2)


def mode_lines():
    tgs = batches(top3=0)
    sh = build_shard(config3_spec(), 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True, eager=True)
    run("U24shard_rt_k8_us", lambda t: T.rt_closest(t, 8), tgs)
    run("U24shard_rt_k16_us", lambda t: T.rt_closest(t, 16), tgs)
    run("U24shard_rt_k32_us", lambda t: T.rt_closest(t, 32), tgs)
    run("U24shard_nc_k14_us", lambda t: T.nc_closest(t, 14), tgs)
    run("U24shard_nc_k32_us", lambda t: T.nc_closest(t, 32), tgs)
    T.close()
    del sh
    n = 4_000_000
    ids = S.random_ids(n, 0xB5)
    st = S.random_status(n, 0xB6)
    perm, first, off = S.split_table(ids)
    T = DeviceTable(ids[perm], st[perm], first, off, device=0, eager=True)
    tgs = batches(seed=10)
    run("S4M_rt_k8_us", lambda t: T.rt_closest(t, 8), tgs)
    run("S4M_rt_k14_us", lambda t: T.rt_closest(t, 14), tgs)
    run("S4M_rt_k32_us", lambda t: T.rt_closest(t, 32), tgs)
    T.close()


def mode_shard():
    import bench
    from opendht_amd.global_shard import GlobalShard, build_plain_shard

    spec = config3_spec(1)  # the whole 100M-node table, then rank 0's eighth of it (as bench.n8_step_model)
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
    gp = np.concatenate([[0], np.cumsum(good.astype(np.int64))])
    B = off.shape[0] - 1
    h8 = B // 8
    n0 = int(off[h8])
    G0 = GlobalShard(ids[:n0], st[:n0], off[:h8 + 1], 0, h8, spec.depth, 0, gp, device=0)
    del ids, st
    tgs = batches(seed=11)
    s = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    far = batches(seed=13)
    for t in far:
        t[:, 0] |= 0x80  # beyond rank 0's reach: reading and testing the batch is all the kernel does
    ex = G0.exchange(Q, 8, 8)
    run("shard_reach0_us", lambda t: G0.home_block(t, ex), far)
    own = batches(top3=0, seed=14)  # every query in reach (what one rank holding its own queries would see)
    ex1 = G0.exchange(Q, 8, 1)
    run("shard_allreach_k8_us", lambda t: G0.home_block(t, ex1), own)
    del far, own, ex1
    for k in (8, 32):
        ex = G0.exchange(Q, k, 8)
        run(f"shard_k{k}_us", lambda t: G0.home_block(t, ex), tgs)
        ex.recv = bench.home0_recv(G0, ex, tgs[0], Q, dev)
        hq = -(-(-(-Q // 256)) // 8) * 256
        oi = torch.empty((hq, k), dtype=torch.int32, device=dev)
        oc = torch.empty((hq,), dtype=torch.uint8, device=dev)
        run(f"finish_k{k}_us", lambda t: ex.home_finish(0, oi, oc, s), tgs)
    G0.close()


def mode_swarm():
    from opendht_amd.swarm import Swarm

    peers, lookups = 2_000_000, 1 << 18
    ids, _ = S.sort_ids(S.random_ids(peers, 0x0D470500))
    W = Swarm(ids, device=0)
    rng = np.random.default_rng(9)
    src = torch.from_numpy(rng.integers(0, peers, lookups).astype(np.int32)).to(dev)
    tg = torch.from_numpy(S.random_targets(lookups, seed=0x0D470501)).to(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    X = W.search(src, tg, 1000)
    hops = X.run()
    b.record()
    torch.cuda.synchronize()
    res["swarm_2M_256k_ms"] = round(a.elapsed_time(b), 3)
    res["swarm_hops"] = int(hops)
    X.close()
    W.close()


def mode_swarm0():
    """config 5 at 2M peers with every peer online (the 16-register merge), 256k lookups to convergence"""
    from opendht_amd.swarm import Swarm

    peers, lookups = 2_000_000, 1 << 18
    ids, _ = S.sort_ids(S.random_ids(peers, 0x0D470500))
    W = Swarm(ids, device=0)
    rng = np.random.default_rng(9)
    src = torch.from_numpy(rng.integers(0, peers, lookups).astype(np.int32)).to(dev)
    tg = torch.from_numpy(S.random_targets(lookups, seed=0x0D470501)).to(dev)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    X = W.search(src, tg, 0)
    hops = X.run()
    b.record()
    torch.cuda.synchronize()
    res["swarm0_2M_256k_ms"] = round(a.elapsed_time(b), 3)
    res["swarm0_hops"] = int(hops)
    X.close()
    W.close()


def mode_refresh():
    import bench

    spec = config3_spec()
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    now = 1_000_000 * 10**9
    t, rt, ex = bench.node_times(sh.status, now)
    T.set_times(t, rt, ex)
    T.refresh_status(now)
    torch.cuda.synchronize()
    d = np.sort(np.minimum(t + 600 * 10**9, rt + 7200 * 10**9)[(sh.status & 1) == 1])
    d = d[d >= now]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts, j = [], 0
    for step in range(300):  # 1 .. 100 deadlines per refresh, as a live table between query batches
        j += 1 + (step * 37) % 100
        a.record()
        T.refresh_status(int(d[min(j, d.shape[0] - 1)]) + 1)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    res["refresh_event_us_median"] = round(float(np.median(ts)), 2)
    res["refresh_deadlines_passed"] = j
    res["refresh_diag"] = T.refresh_diag()
    T.close()


def mode_route():
    from opendht_amd._lib import check, lib, ptr
    from opendht_amd.sharded import OwnerRoute

    tgs = batches(seed=12)
    s = torch.cuda.current_stream(dev).cuda_stream
    R = OwnerRoute(Q, 8, 8, 3, dev, collective=False, keys=False)
    run("route_pack_n8_us", lambda t: R.pack(t, s), tgs)  # route_pack_kernel<false>
    RK = OwnerRoute(Q, 8, 8, 3, dev, collective=False, keys=True)
    run("route_pack_keys_n8_us", lambda t: RK.pack(t, s), tgs)  # route_pack_kernel<true>
    oi = torch.empty((Q, 8), dtype=torch.int32, device=dev)
    oc = torch.empty((Q,), dtype=torch.uint8, device=dev)
    R.rows.random_(0, 1 << 20)
    R.cnt.fill_(8)
    run("route_unpack_k8_us", lambda t: R.unpack(oi, oc, s), tgs)
    # the owner's query with packed rows over the 8 blocks it receives: from 20-byte targets, then from 8-byte keys
    sh = build_shard(config3_spec(), 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    own = batches(top3=0, seed=15)
    R.recv = R.send = torch.cat([t[:R.cap] for t in own])[:8 * R.cap]
    run("route_answer_packed_k8_us", lambda t: R.answer(T, s), tgs)  # rt_ws_packed_kernel<false>
    res["route_answer_fused"] = bool(R.fused)
    RK.recv_keys = R.recv[:, :8].flip(1).contiguous().view(torch.int64).view(-1)
    run("route_answer_keys_k8_us", lambda t: RK.answer(T, s), tgs)  # rt_ws_packed_kernel<true>
    res["route_answer_keys_tailed"] = bool(RK.tailed(combine=False))
    run("route_unpack_packed_k8_us", lambda t: R.unpack_packed(oi, oc, s), tgs)  # route_unpack_packed4, case 0
    RK.back_prow = R.prow
    flags = torch.zeros((4,), dtype=torch.int32, device=dev)

    def unpack_fold(t):  # case 1: the same unpack folding and zeroing the batch's counters (the native executor's)
        check(lib().kad_route_unpack_packed_fold(ptr(RK.slot), Q, 8, ptr(RK.back_prow), ptr(oi), ptr(oc), ptr(RK.ctr), 8,
                                                 ptr(flags), 0, C.c_void_p(s)), "kad_route_unpack_packed_fold")

    run("route_unpack_packed_fold_k8_us", unpack_fold, tgs)
    T.close()


if __name__ == "__main__":
    {"lines": mode_lines, "shard": mode_shard, "swarm": mode_swarm, "swarm0": mode_swarm0, "refresh": mode_refresh,
     "route": mode_route}[sys.argv[1] if len(sys.argv) > 1 else "lines"]()
    print(json.dumps(res), flush=True)
