"""Headline bench: k=8 closest-node queries/sec at a 100M-node table (1/8 per GPU) + % HBM roofline.

Workload (BASELINE.json config 3, per GPU): rank r holds shard r of the 100M-node U(24)
routing table (2^21 owned buckets, ~12.5M nodes, plus the exact halo from its neighbours) in
HBM and answers a batch of 1,048,576 RoutingTable::findClosestNodes(target, now, 8) queries
whose targets it owns. One step = one batched kernel launch over that batch; inputs are
resident in HBM before the timed region. Weak scaling: per-GPU work is fixed as N grows; at
N=8 the shards cover the whole 100M-node table and a step answers 8M queries. No data-path
collective (owner routing, DESIGN.md "Multi-GPU").

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd._lib import KAD_INFO_WINDOW_LINES  # noqa: E402
from opendht_amd.metrics import rt_algorithmic_bytes  # noqa: E402
from opendht_amd.sharded import ShardSpec, build_shard  # noqa: E402

METRIC = "k=8 closest-node queries/sec at 100M-node table (1/8 GPU) + % HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md


def cpu_baseline(sh, targets, count, budget_s, nthreads):
    """The oracle's structure-faithful restatement of RoutingTable::findClosestNodes (std::list
    buckets, linear findBucket, insertion sort: the "port" CPU baseline) on this rank's shard,
    timed on host cores over a bounded sample of the same queries."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    t0 = time.perf_counter()
    F = O.FaithfulTable(sh.ids, sh.status, sh.first, sh.off)
    build_s = time.perf_counter() - t0
    # time successive slices of the same queries (doubling) until the budget is spent: the
    # first slice also warms the table's pages, so no single-probe extrapolation is needed
    n, dt, chunk = 0, 0.0, max(nthreads, 16)
    while n < targets.shape[0] and dt < budget_s:
        sl = targets[n:n + chunk]
        t0 = time.perf_counter()
        F.rt_closest(sl, count, nthreads=nthreads)
        dt += time.perf_counter() - t0
        n += sl.shape[0]
        chunk = min(2 * chunk, max(16, int(n * (budget_s - dt) / max(dt, 1e-9))))
    F.close()
    return {"value": n / dt, "unit": "queries/s", "cores": nthreads, "kind": "port",
            "sample": f"{n} of the {targets.shape[0]} queries of rank 0's step (same shard table, "
                      f"{sh.first.shape[0]} buckets, {sh.ids.shape[0]} nodes); structure-faithful "
                      f"oracle build {build_s:.1f}s excluded"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--count", type=int, default=8)
    ap.add_argument("--queries", type=int, default=1 << 20, help="queries per GPU per step")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU baseline sampling")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-graph", action="store_true", help="issue the K steps one by one instead of one HIP graph")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_r01.json"))
    ap.add_argument("--mode", choices=("owner", "allgather"), default="owner",
                    help="owner: weak scaling, owner-routed shards with halo (the headline); allgather: the "
                         "north-star variant, 1M global queries against the 100M-node table split over the N "
                         "GPUs without halo, RCCL all-gather + on-device merge (strong scaling)")
    args = ap.parse_args()
    if args.mode == "allgather":
        return main_allgather(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 8:
        raise SystemExit("the 100M-node table has 8 shards: at most 8 GPUs")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)

    spec = ShardSpec()  # 100M-node U(24), 8 shards, k_max 32
    t0 = time.perf_counter()
    sh = build_shard(spec, rank)
    targets = spec.targets_for(rank, args.queries, seed=0x0D470002)
    build_s = time.perf_counter() - t0

    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=local, index_base=sh.index_base, sorted=True)
    tg = torch.from_numpy(targets).to(dev)
    out_idx = torch.empty((args.queries, args.count), dtype=torch.int32, device=dev)
    out_cnt = torch.empty((args.queries,), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    wl = bool(T.info()["flags"] & KAD_INFO_WINDOW_LINES)  # the shard's U(24) table carries all three line sets
    kernel = (("rt_wl_kernel<0>" if args.count <= 8 else "rt_wl16_kernel" if args.count <= 16 else "rt_wl32_kernel")
              if wl else f"rt_closest_kernel<{8 if args.count <= 8 else 16 if args.count <= 16 else 32}>")

    # algorithmic bytes of one launch (exact, host side; target buckets from the engine's findBucket)
    tb = T.find_bucket(tg).cpu().numpy().view(np.uint32).astype(np.int64)
    alg_bytes, mb, mn, mg = rt_algorithmic_bytes(sh.status, sh.off, tb, args.count)

    for _ in range(args.warmup):
        T.rt_closest(tg, args.count, out_idx, out_cnt, stream=stream.cuda_stream)
    torch.cuda.synchronize(dev)

    # The K steps go out as one HIP graph of K launches (the step is ~30 us; issuing them one by one
    # from Python leaves ~3 us gaps). --no-graph issues them one by one with an event per step.
    graph = None
    if not args.no_graph:
        try:
            g = torch.cuda.CUDAGraph()
            cs = torch.cuda.Stream(dev)
            cs.wait_stream(stream)
            with torch.cuda.graph(g, stream=cs):
                for _ in range(args.steps):
                    T.rt_closest(tg, args.count, out_idx, out_cnt, stream=cs.cuda_stream)
            stream.wait_stream(cs)
            g.replay()  # untimed: the graph's first launch uploads it
            torch.cuda.synchronize(dev)
            graph = g
        except Exception as e:  # capture unsupported: fall back to eager launches
            print(f"graph capture failed ({e}); eager launches", file=sys.stderr)
            graph = None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    ev[0].record(stream)
    if graph is not None:
        graph.replay()
        ev[-1].record(stream)
    else:
        for i in range(args.steps):
            T.rt_closest(tg, args.count, out_idx, out_cnt, stream=stream.cuda_stream)
            ev[i + 1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t_start
    if graph is not None:
        kern_ms = [ev[0].elapsed_time(ev[-1]) / args.steps]
    else:
        kern_ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(args.steps)]
    t_max = wall
    if dist:
        x = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        t_max = float(x.item())

    avg_kernel_s = float(np.mean(kern_ms)) / 1e3
    achieved = alg_bytes / avg_kernel_s / 1e9
    total_q = world * args.queries * args.steps
    value = total_q / t_max

    traffic = None
    if os.path.exists(args.traffic_json):
        try:
            traffic = json.load(open(args.traffic_json)).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(sh, targets, args.count, args.cpu_budget, min(16, os.cpu_count() or 1))

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": t_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic (counter-based uniform 160-bit IDs, 80/10/10 good/expired/dubious)",
            "config": {
                "workload": "config3: 100M-node U(24) routing table, 1/8 shard per GPU (2^21 owned buckets "
                            f"+ halo, {sh.ids.shape[0]} nodes on rank 0), {args.queries} owned queries per GPU "
                            f"per step, k={args.count}",
                "table_nodes_per_gpu": int(sh.ids.shape[0]),
                "buckets_per_gpu": int(sh.first.shape[0]),
                "queries_per_gpu": args.queries,
                "k": args.count,
                "parallelism": f"id-range shards x{world}, owner routing (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kernel,
                "launch": "hip graph of K launches" if graph is not None else "K eager launches",
                "avg_kernel_ms": avg_kernel_s * 1e3,
                "alg_bytes_per_launch": alg_bytes,
                "alg_bytes_per_query": alg_bytes / args.queries,
                "window_means": {"buckets": mb, "nodes": mn, "good": mg},
            },
            "cpu_baseline": cpu,
            "setup_s": build_s,
        }
        print(json.dumps(line), flush=True)
    T.close()
    if dist:
        dist.destroy_process_group()


def main_allgather(args):
    """North-star variant (opendht_amd/global_shard.py): every rank holds 1/N of the 100M-node U(24)
    table without halo and the global good prefix sums; one step answers the same 1M global queries
    on every rank: local rows/parts, RCCL all-gather, device scatter + merge. Strong scaling."""
    from opendht_amd.global_shard import GlobalShard, build_plain_shard, global_good_prefix
    from opendht_amd import synth as S

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus or world & (world - 1) or world > 8:
        raise SystemExit("allgather mode: --gpus must equal WORLD_SIZE, a power of two <= 8")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist

        dist.init_process_group("nccl", device_id=dev)
    spec = ShardSpec(n_shards=world)  # the 100M-node U(24) table in `world` shards
    t0 = time.perf_counter()
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, rank)
    gp = global_good_prefix(good, device=dev if world > 1 else None)
    G = GlobalShard(ids, st, off, lo, hi, spec.depth, base, gp, device=local)
    n_local = ids.shape[0]
    del ids, st
    targets = torch.from_numpy(S.random_targets(args.queries, seed=0x0D470002)).to(dev)
    build_s = time.perf_counter() - t0
    out_idx = torch.empty((args.queries, args.count), dtype=torch.int32, device=dev)
    out_cnt = torch.empty((args.queries,), dtype=torch.uint8, device=dev)
    for _ in range(args.warmup):
        G.query(targets, args.count, out_idx=out_idx, out_cnt=out_cnt)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    for _ in range(args.steps):
        G.query(targets, args.count, out_idx=out_idx, out_cnt=out_cnt)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    wall = time.perf_counter() - t_start
    t_max = wall
    if dist:
        x = torch.tensor([wall], dtype=torch.float64, device=dev)
        dist.all_reduce(x, op=dist.ReduceOp.MAX)
        t_max = float(x.item())
    if rank == 0:
        print(json.dumps({
            "metric": "k=8 closest-node queries/sec, 1M queries vs the 100M-node table split over N GPUs "
                      "(north-star all-gather + merge variant)",
            "value": args.queries * args.steps / t_max, "unit": "queries/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": t_max / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u64",
            "data": "synthetic (counter-based uniform 160-bit IDs, 80/10/10 good/expired/dubious)",
            "config": {"workload": f"config3 north-star: 100M-node U(24) table, 1/{world} per GPU without halo "
                                   f"({n_local} nodes on rank 0), {args.queries} global queries per step, "
                                   f"k={args.count}, RCCL all-gather of rows + device merge",
                       "parallelism": f"id-range shards x{world}, replicated batch, all-gather"},
            "setup_s": build_s}), flush=True)
    G.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
