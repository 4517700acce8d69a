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
