"""Child process of tests/test_rccl_world1.py: a real RCCL ("nccl") process group of one rank on this box's GPU,
so that the multi-GPU code's RCCL branches run on the device at least once (the CPU tests use gloo):

  * the north-star step (global_shard.GlobalShard.query with force_collective): kad_rt_shard_batch_home, then
    all_to_all_single of the send blocks through RCCL, kad_rt_home_finish; the all-gather form through
    all_gather_into_tensor; both started with capacities of 1, so the sticky overflow word is combined with a
    device-tensor all_reduce(MAX) and the needed capacities with another, the layout grows and the batch reruns;
  * owner routing (sharded.route_queries / return_results): all_to_all_single of the split sizes, the targets,
    the rows and the counts, on device tensors; and its device-only form (sharded.OwnerRoute through serve_owner:
    kad_route_pack, all_to_all_single of the fixed-size blocks, kad_route_unpack, the overflow combine).

Every row is compared with the oracle on the whole table (routing_table.cpp:67-111; the windows of
routing_table.cpp:89-104). Prints RCCL_WORLD1_OK and one JSON line of step timings."""
import json
import os
import socket
import sys
import time
import types

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle as O  # noqa: E402
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.global_shard import Exchange, GlobalShard, build_plain_shard  # noqa: E402
from opendht_amd.sharded import (OwnerPipeline, OwnerRoute, ShardSpec, return_results, route_queries,  # noqa: E402
                                 serve_owner, serve_pipelined)
from opendht_amd.table import DeviceTable  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    from datetime import timedelta

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev,
                            timeout=timedelta(seconds=60))
    assert dist.get_backend() == "nccl"
    spec = ShardSpec(n_shards=1, depth=12, mean_per_bucket=6.0, seed=0x6A7 + 12, good_pct=80, expired_pct=10)
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
    first = S.bucket_firsts(spec.depth, lo, hi)
    gp = np.concatenate([[0], np.cumsum(good)])
    G = GlobalShard(ids, st, off, lo, hi, spec.depth, base, gp, device=0)
    targets = np.ascontiguousarray(np.concatenate([S.random_targets(20000, seed=77), ids[::97]]), np.uint8)
    tg = torch.from_numpy(targets).to(dev)
    q = targets.shape[0]
    timings = {}
    try:
        for count in (1, 8, 14, 32):
            want, wcnt = O.flat_rt_closest(ids, st, first, off, targets, count, nthreads=8)
            for home in (True, False):
                # capacities of 1: the first step overflows, the combine and the growth go through RCCL
                G._ex[(q, count, 1, home, True)] = Exchange(q, count, 1, dev, row_cap=1, part_cap=1, home=home,
                                                            collective=True)
                lo_q, idx, cnt = G.query(tg, count, home=home, force_collective=True)
                torch.cuda.synchronize()
                assert lo_q == 0 and idx.shape[0] == q
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"k={count} home={home} counts")
                np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"k={count} home={home}")
                assert len(G.tries) >= 2 and G.tries[0] == (1, 1), G.tries  # it grew and ran again
        # step time with and without the collective (k = 8, the grown layouts, 20 eager steps each)
        for coll in (False, True):
            ex = G.exchange(q, 8, 1, True, coll)
            out_i = torch.empty((q, 8), dtype=torch.int32, device=dev)
            out_c = torch.empty((q,), dtype=torch.uint8, device=dev)
            for _ in range(3):
                G.step(tg, ex, out_i, out_c, rank=0)
                if not ex.overflowed():
                    break
                ex = G._ex[(q, 8, 1, True, coll)] = ex.grown()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                G.step(tg, ex, out_i, out_c, rank=0)
            torch.cuda.synchronize()
            timings["step_us_rccl" if coll else "step_us_no_collective"] = (time.perf_counter() - t0) / 20 * 1e6
            assert not ex.overflowed()
        # owner routing through RCCL: route, answer on the device, route the rows back
        T = DeviceTable(ids, st, first, off, device=0, sorted=True)
        for count in (8, 14):
            want, wcnt = O.flat_rt_closest(ids, st, first, off, targets, count, nthreads=8)
            local, ctx = route_queries(tg, types.SimpleNamespace(shard_bits=3))
            assert local.device.type == "cuda" and local.shape[0] == q
            li, lc = T.rt_closest(local, count)
            oi, oc = return_results(li, lc, ctx)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(oc.cpu().numpy(), wcnt, err_msg=f"routed k={count} counts")
            np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want, err_msg=f"routed k={count}")
            # the device-only owner routing (kad_route_pack / unpack) with its all_to_alls through RCCL, started
            # with blocks of one record: the overflow and the block counts are combined through RCCL all_reduces
            route = OwnerRoute(q, count, 1, 0, dev, cap=1, collective=True)
            oi, oc, route = serve_owner(T, tg, count, route=route)
            torch.cuda.synchronize()
            assert route.cap > 1
            np.testing.assert_array_equal(oc.cpu().numpy(), wcnt, err_msg=f"owner route k={count} counts")
            np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want, err_msg=f"owner route k={count}")
        # the overlapped forms through RCCL: 5 consecutive distinct batches each
        batches = [np.ascontiguousarray(S.random_targets(6000, seed=300 + j), np.uint8) for j in range(5)]
        dbs = [torch.from_numpy(b).to(dev) for b in batches]
        for count in (8, 14):
            wants = [O.flat_rt_closest(ids, st, first, off, b, count, nthreads=8) for b in batches]
            pipe = OwnerPipeline(6000, count, 1, 0, dev, cap=8, collective=True)
            outs, pipe = serve_pipelined(T, dbs, count, pipe=pipe)
            torch.cuda.synchronize()
            assert pipe.cap > 8 and pipe.collective
            for j, (want, wcnt) in enumerate(wants):
                np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"owner pipe k={count} b{j}")
                np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                              err_msg=f"owner pipe k={count} b{j}")
            like = Exchange(6000, count, 1, dev, row_cap=1 << 20, part_cap=4096, collective=True)
            exs = G.pipeline(6000, count, 1, like=like)
            outs = [(torch.empty((6000, count), dtype=torch.int32, device=dev),
                     torch.empty((6000,), dtype=torch.uint8, device=dev)) for _ in dbs]
            G.run_pipelined(dbs, exs, outs, rank=0)
            torch.cuda.synchronize()
            assert not any(e.overflowed() for e in exs)
            for j, (want, wcnt) in enumerate(wants):
                np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"ns pipe k={count} b{j}")
                np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                              err_msg=f"ns pipe k={count} b{j}")
        # the native executor (opendht_amd.comm: kad_route_run / kad_shard_run over the engine's own RCCL
        # communicator), serial and pipelined, blocks of one record first for the owner routing
        from opendht_amd.comm import Comm, NativeRoute, serve_native, shard_run

        with Comm(0, 1, 0) as comm:
            for count in (8, 14, 32):
                wants = [O.flat_rt_closest(ids, st, first, off, b, count, nthreads=8) for b in batches]
                for n_sets in (1, 3):
                    route = NativeRoute(6000, count, 1, 0, dev, cap=8, n_sets=n_sets, comm=comm)
                    outs, route = serve_native(T, dbs, count, route)
                    torch.cuda.synchronize()
                    assert route.cap > 8
                    for j, (want, wcnt) in enumerate(wants):
                        np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"native k={count} "
                                                      f"sets={n_sets} b{j} counts")
                        np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                                      err_msg=f"native k={count} sets={n_sets} b{j}")
                    like = Exchange(6000, count, 1, dev, row_cap=1 << 20, part_cap=4096, collective=True)
                    exs = G.pipeline(6000, count, 1, like=like)[:n_sets]
                    outs = [(torch.empty((6000, count), dtype=torch.int32, device=dev),
                             torch.empty((6000,), dtype=torch.uint8, device=dev)) for _ in dbs]
                    shard_run(G, comm, dbs, exs, outs)
                    torch.cuda.synchronize()
                    assert not exs[0].overflowed()
                    for j, (want, wcnt) in enumerate(wants):
                        np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"native ns k={count} "
                                                      f"sets={n_sets} b{j} counts")
                        np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                                      err_msg=f"native ns k={count} sets={n_sets} b{j}")
            # kad_comm_all_to_all at world 1: a copy
            x = torch.randint(0, 1 << 30, (4096,), dtype=torch.int32, device=dev)
            y = torch.empty_like(x)
            comm.all_to_all(y, x)
            torch.cuda.synchronize()
            assert torch.equal(x, y)
        T.close()
    finally:
        G.close()
        dist.destroy_process_group()
    print(json.dumps({"rccl_world1": timings, "queries": q}), flush=True)
    print("RCCL_WORLD1_OK", flush=True)


if __name__ == "__main__":
    main()
