"""Multi-process path on CPU (gloo, world_size 2): serving-mode query routing -- targets go to
their owner shard with all_to_all_single, each rank answers from its own shard table (oracle on
CPU; the GPU engine on a GPU box) and results come back in the original order. Bit-exact against
the whole table."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    import torch.distributed as dist

    import oracle as O
    from opendht_amd import synth as S
    from opendht_amd.sharded import ShardSpec, build_shard, return_results, route_queries

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok = False
    try:
        spec = ShardSpec(n_shards=world, depth=10, mean_per_bucket=6.0, seed=991)
        sh = build_shard(spec, rank)
        # each rank receives a batch of arbitrary targets (any owner)
        tg = S.random_targets(3000, seed=1000 + rank)
        local, ctx = route_queries(tg, spec)
        ltg = local.numpy()
        assert (ltg[:, 0] >> (8 - spec.shard_bits) == rank).all()
        idx, cnt = O.flat_rt_closest(sh.ids, sh.status, sh.first, sh.off, ltg, 8)
        idx = np.where(idx != 0xFFFFFFFF, idx + np.uint32(sh.index_base), idx).astype(np.uint32)
        out_idx, out_cnt = return_results(idx, cnt, ctx)
        out_idx, out_cnt = out_idx.numpy().view(np.uint32), out_cnt.numpy()
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, tg, 8)
        ok = np.array_equal(out_idx, want) and np.array_equal(out_cnt, wcnt)
    finally:
        q.put((rank, bool(ok)))
        dist.destroy_process_group()


def test_route_queries_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True}
