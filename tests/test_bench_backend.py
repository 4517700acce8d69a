"""bench.py's owner-routed serving step puts its data path (the all_to_alls of the target blocks and the rows) on
RCCL whenever the ranks have a GPU each: data_backend() picks nccl for world > 1 on CUDA
devices, gloo only in the one-GPU rehearsal, and owner_routed_pass refuses to run the data path on any other
backend. CPU only: two gloo ranks, the device only named (nothing touches a GPU before the refusal)."""
import importlib
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(one_gpu: bool):
    os.environ.pop("KADGPU_BENCH_ONE_GPU", None)
    if one_gpu:
        os.environ["KADGPU_BENCH_ONE_GPU"] = "1"
    sys.path.insert(0, ROOT)
    import bench

    try:
        return importlib.reload(bench)
    finally:
        os.environ.pop("KADGPU_BENCH_ONE_GPU", None)


def test_data_backend_selects_rccl_on_gpus():
    b = _bench(False)
    cuda = torch.device("cuda", 0)
    assert b.data_backend(1, cuda) is None
    for n in (2, 4, 8):
        assert b.data_backend(n, cuda) == "nccl"
        assert b.data_backend(n, torch.device("cpu")) == "gloo"
    r = _bench(True)  # the rehearsal: every rank on cuda:0, RCCL impossible
    assert r.data_backend(2, cuda) == "gloo"


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench(False)
        try:
            b.owner_routed_pass(None, None, None, 1 << 10, 8, 2, 1, torch.device("cuda", rank), dist, world, rank)
            q.put((rank, "ran"))
        except RuntimeError as e:
            q.put((rank, str(e)))
    finally:
        dist.destroy_process_group()


def test_owner_routed_pass_refuses_gloo_between_gpus():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert "must run on nccl" in got[r], got


@pytest.mark.parametrize("world,bits", [(1, 0), (2, 1), (4, 2), (8, 3)])
def test_owner_shard_bits(world, bits):
    from opendht_amd.sharded import ShardSpec, owner_shard_bits

    assert owner_shard_bits(world) == bits
    assert owner_shard_bits(world, ShardSpec(n_shards=world)) == bits


@pytest.mark.parametrize("world,n_shards", [(3, 3), (6, 8), (2, 8), (8, 4)])
def test_owner_shard_bits_refuses_mismatch(world, n_shards):
    """world 3: rank 2 would get no targets; n_shards > world: shard r + world's targets would go to rank r, which
    does not hold that shard. Both raise instead of answering from the wrong shard."""
    from opendht_amd.sharded import ShardSpec, owner_shard_bits

    with pytest.raises(ValueError):
        owner_shard_bits(world, ShardSpec(n_shards=n_shards) if n_shards & (n_shards - 1) == 0 else None)


def _verify_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import numpy as np
    import torch.distributed as dist

    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import oracle as O
    from opendht_amd import synth as S
    from opendht_amd.sharded import ShardSpec, build_shard

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b = _bench(False)
        spec = ShardSpec(n_shards=world, depth=8, mean_per_bucket=6.0, seed=0xA11 + 3, good_pct=70, expired_pct=15)
        sh = build_shard(spec, rank)
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        tg = S.random_targets(600, seed=50 + rank)  # targets of both shards: half answered by the other rank
        want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, tg, 8)
        idx = torch.from_numpy(want.view(np.int32).copy())
        cnt = torch.from_numpy(wcnt.copy())
        good = b.verify_routed(dist, sh, spec, rank, world, torch.from_numpy(tg), idx, cnt, 8)
        # rank 1 corrupts one returned row whose target rank 0 owns: rank 0 must be the one to catch it
        if rank == 1:
            j = int(np.flatnonzero((tg[:, 0] >> 7) == 0)[0])
            idx[j, 0] = idx[j, 0] + 1
        bad = b.verify_routed(dist, sh, spec, rank, world, torch.from_numpy(tg), idx, cnt, 8)
        q.put((rank, good, bad))
    except Exception as e:  # reported through the queue
        q.put((rank, {"error": repr(e)}, None))
    finally:
        dist.destroy_process_group()


def test_verify_routed_checks_rows_answered_elsewhere():
    """bench.verify_routed: every rank's returned rows are all-gathered and each is checked by the rank
    owning its target, so a wrong row that came back from another rank is counted. Two gloo ranks on the CPU, rows
    from the oracle on the whole table, then one row of a rank-0 target corrupted on rank 1."""
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_verify_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = {r: (g, b) for r, g, b in (q.get(timeout=180) for _ in ps)}
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        g, b = got[r]
        assert "error" not in g, g
        assert g["rows"] == 1200 and g["mismatches"] == 0 and g["rows_answered_by_another_rank"] > 0, g
        assert b["mismatches"] == 1, b
