"""Owner routing of a serving front end, device-only (kad_route_pack / kad_route_unpack, sharded.OwnerRoute;
DESIGN.md §6.1): every rank sends its batch's targets to the ranks owning them, the owners answer from their
halo shards, the rows come back to the senders' positions. The reference answers each request where it arrives
(Dht::onFindNode / onGetValues, dht.cpp:3189-3217), every answer the whole table's findClosestNodes
(routing_table.cpp:67-111). Checked bit-exact against the oracle on the whole table: N = 1, 2, 4, 8 ranks simulated
on one GPU (blocks concatenated as all_to_all_single delivers them), capacities of 1 (overflow, growth, rerun), rows
back plain and packed (kad_route_compress, and the unpacked rerun when a row cannot be packed), and two real gloo
ranks sharing the GPU."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd.sharded import OwnerRoute, ShardSpec, build_shard, route_simulated

pytestmark = pytest.mark.gpu


def _batch(spec, n, seed):
    """Targets over the whole ID space plus node IDs and bucket firsts next to every shard edge."""
    rng = np.random.default_rng(seed)
    parts = [S.random_targets(n, seed=seed)]
    per = spec.n_buckets // spec.n_shards
    for e in range(0, spec.n_buckets + 1, per):
        for b in (e - 1, e):
            if 0 <= b < spec.n_buckets:
                f = S.bucket_firsts(spec.depth, b, b + 1).copy()
                f[0, 8:] = rng.integers(0, 256, 12, dtype=np.uint8)
                parts.append(f)
    return np.ascontiguousarray(np.concatenate(parts), np.uint8)


@pytest.mark.parametrize("world", [1, 2, 4, 8])
@pytest.mark.parametrize("small_cap", [False, True], ids=["", "cap1"])
@pytest.mark.parametrize("packed", [False, True], ids=["rows", "packed"])
def test_owner_route_simulated(gpu, world, small_cap, packed):
    spec = ShardSpec(n_shards=world, depth=10, mean_per_bucket=6.0, seed=0x0A0 + world, good_pct=60, expired_pct=20)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    shards = [build_shard(spec, s) for s in range(world)]
    tables = [DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
              for sh in shards]
    try:
        batches = [_batch(spec, 3000, seed=world * 16 + r) for r in range(world)]
        n = min(b.shape[0] for b in batches)
        batches = [b[:n] for b in batches]
        tgs = [torch.from_numpy(b).to(gpu) for b in batches]
        for count in (1, 8, 14, 32):
            out, r0 = route_simulated(tables, tgs, count, spec.shard_bits, cap=1 if small_cap else None,
                                      packed=packed)
            torch.cuda.synchronize()
            if small_cap:
                assert r0.cap > 8  # it grew (cap 1 -> one record per sub-block)
            if packed:
                assert not r0.sim_escaped  # (60 % good: every window spans far fewer than 255 nodes)
            for r, (oi, oc) in enumerate(out):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, batches[r], count, nthreads=8)
                np.testing.assert_array_equal(oc.cpu().numpy(), wcnt, err_msg=f"N={world} rank {r} k={count} counts")
                np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want,
                                              err_msg=f"N={world} rank {r} k={count}")
    finally:
        for T in tables:
            T.close()


def test_route_pack_layout(gpu):
    """kad_route_pack places every target in its owner's block once (in its workgroup's sub-block), counts each
    sub-block, flags a full one."""
    q, world, bits = 5000, 4, 2
    t = torch.randint(0, 256, (q, 20), dtype=torch.uint8, device=gpu)
    R = OwnerRoute(q, 8, world, bits, gpu, cap=8 * 1024, keys=False)
    s = torch.cuda.current_stream(gpu).cuda_stream
    R.pack(t, s)
    torch.cuda.synchronize()
    owner = (t[:, 0].to(torch.int64) >> (8 - bits)) % world
    slot = R.slot.cpu().numpy().view(np.uint32).astype(np.int64)
    subs = R.ctr[:world * 8 * 32].view(world * 8, 32)[:, 0].cpu().numpy().reshape(world, 8)
    assert not R.overflowed(combine=False)
    np.testing.assert_array_equal(subs.sum(1), torch.bincount(owner, minlength=world).cpu().numpy())
    cap = R.cap
    np.testing.assert_array_equal(slot // cap, owner.cpu().numpy())
    # workgroup w (1,024 targets) appends to sub-block w % 8 of its owner's block
    np.testing.assert_array_equal((slot % cap) // (cap // 8), (np.arange(q) // 1024) % 8)
    assert int(subs[:, 5:].sum()) == 0  # (5,000 targets: workgroups 0..4)
    assert np.unique(slot).size == q
    np.testing.assert_array_equal(R.send[torch.from_numpy(slot).to(gpu)].cpu().numpy(), t.cpu().numpy())
    # kad_route_pack_keys: the same places, each record the target's top 64 bits as one native key
    RK = OwnerRoute(q, 8, world, bits, gpu, cap=8 * 1024, keys=True)
    RK.pack(t, s)
    torch.cuda.synchronize()
    kslot = RK.slot.cpu().numpy().view(np.uint32).astype(np.int64)  # (the order inside a sub-block is unspecified)
    np.testing.assert_array_equal(kslot // cap, owner.cpu().numpy())
    assert np.unique(kslot).size == q
    want = t.cpu().numpy()[:, :8].copy().view(">u8").reshape(-1)
    got = RK.send_keys[torch.from_numpy(kslot).to(gpu)].cpu().numpy().view(np.uint64)
    np.testing.assert_array_equal(got, want)
    R2 = OwnerRoute(q, 8, world, bits, gpu, cap=8 * 100)
    R2.pack(t, s)
    torch.cuda.synchronize()
    assert R2.overflowed(combine=False)
    assert int((R2.slot.cpu().numpy().view(np.uint32) == 0xFFFFFFFF).sum()) > 0


def test_owner_route_packed_escape(gpu):
    """A mostly-bad table: count-32 windows span more than 254 nodes, so the packed rows escape and the way back
    runs unpacked; every row still equals the whole table's answer. kad_route_compress / kad_route_unpack_packed
    round trip on rows that do pack."""
    world = 2
    spec = ShardSpec(n_shards=world, depth=8, mean_per_bucket=12.0, seed=0xE5C, good_pct=2, expired_pct=90)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    shards = [build_shard(spec, s) for s in range(world)]
    tables = [DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
              for sh in shards]
    try:
        batches = [_batch(spec, 800, seed=70 + r)[:800] for r in range(world)]
        tgs = [torch.from_numpy(b).to(gpu) for b in batches]
        seen = set()
        for count in (4, 32):
            out, r0 = route_simulated(tables, tgs, count, spec.shard_bits, packed=True)
            torch.cuda.synchronize()
            seen.add(r0.sim_escaped)
            for r, (oi, oc) in enumerate(out):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, batches[r], count, nthreads=8)
                np.testing.assert_array_equal(oc.cpu().numpy(), wcnt, err_msg=f"rank {r} k={count} counts")
                np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want, err_msg=f"rank {r} k={count}")
        assert True in seen  # count 32 escaped
    finally:
        for T in tables:
            T.close()


@pytest.mark.parametrize("good_pct", [80, 2], ids=["u80", "mostly_bad"])
def test_owner_route_fused_packed_rows(gpu, good_pct):
    """Count 8 on a table with short window lines: the query kernel writes the rows packed
    (kad_rt_closest_batch_packed, no compress pass). On a 2 %-good table most windows span hundreds of nodes, the
    rows escape packing and serve_owner answers the batch again unpacked. One rank, every row against the oracle."""
    from opendht_amd.sharded import serve_owner

    spec = ShardSpec(n_shards=1, depth=10, mean_per_bucket=6.0, seed=0xF5 + good_pct, good_pct=good_pct,
                     expired_pct=(100 - good_pct) // 2)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    try:
        targets = _batch(spec, 3000, seed=90 + good_pct)
        tg = torch.from_numpy(targets).to(gpu)
        R = OwnerRoute(tg.shape[0], 8, 1, 0, gpu)
        oi, oc, R = serve_owner(T, tg, 8, route=R)
        torch.cuda.synchronize()
        if good_pct == 2:
            assert R.last_escaped and not R.fused  # could not pack them: answered again unpacked
        else:
            assert R.fused and not R.last_escaped  # the kernel wrote the packed rows
        want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, 8, nthreads=8)
        np.testing.assert_array_equal(oc.cpu().numpy(), wcnt)
        np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want)
    finally:
        T.close()


@pytest.mark.parametrize("good_pct", [60, 2], ids=["u60", "mostly_bad"])
def test_owner_pipeline_one_rank(gpu, good_pct):
    """sharded.OwnerPipeline without a collective (one rank): 6 consecutive distinct batches through three buffer
    sets on two streams, blocks of one record first (the folded overflow word makes every batch run again grown);
    on the 2 %-good table rows escape packing and the batches run again unpacked. Every row against the oracle."""
    from opendht_amd.sharded import OwnerPipeline, serve_pipelined

    spec = ShardSpec(n_shards=1, depth=10, mean_per_bucket=6.0, seed=0x91 + good_pct, good_pct=good_pct,
                     expired_pct=(100 - good_pct) // 2)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    try:
        batches = [_batch(spec, 2500, seed=200 + j)[:2500] for j in range(6)]
        for count in (8, 14, 32):
            pipe = OwnerPipeline(2500, count, 1, 0, gpu, cap=8)
            outs, pipe = serve_pipelined(T, [torch.from_numpy(b).to(gpu) for b in batches], count, pipe=pipe)
            torch.cuda.synchronize()
            assert pipe.cap > 8
            for j, b in enumerate(batches):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, b, count, nthreads=8)
                np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"k={count} batch {j} counts")
                np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                              err_msg=f"k={count} batch {j}")
    finally:
        T.close()


def test_native_route_one_rank_no_comm(gpu):
    """kad_route_run without a communicator (world 1, one buffer set, every batch in order on the stream): rows
    packed (count 8, 32) and plain (14), blocks of one record first; every row against the oracle."""
    from opendht_amd.comm import NativeRoute, serve_native

    spec = ShardSpec(n_shards=1, depth=10, mean_per_bucket=6.0, seed=0x93, good_pct=70, expired_pct=15)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    try:
        batches = [_batch(spec, 2500, seed=300 + j)[:2500] for j in range(4)]
        for count in (8, 14, 32):
            route = NativeRoute(2500, count, 1, 0, gpu, cap=8, n_sets=1)
            outs, route = serve_native(T, [torch.from_numpy(b).to(gpu) for b in batches], count, route)
            torch.cuda.synchronize()
            assert route.cap > 8
            for j, b in enumerate(batches):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, b, count, nthreads=8)
                np.testing.assert_array_equal(outs[j][1].cpu().numpy(), wcnt, err_msg=f"k={count} batch {j} counts")
                np.testing.assert_array_equal(outs[j][0].cpu().numpy().view(np.uint32), want,
                                              err_msg=f"k={count} batch {j}")
        with pytest.raises(ValueError):
            NativeRoute(2500, 8, 1, 0, gpu, n_sets=3)  # the pipelined form needs a communicator
    finally:
        T.close()


def _tie_tables():
    import tables as TB

    return TB.tie_table() + TB.tie_table(groups=24, per=48, seed=8, tag="48") + [TB.uniform_config(20_000, 10),
                                                                              TB.split_config(4000)]


@pytest.mark.parametrize("ti", range(6), ids=["ties", "dups", "ties48", "dups48", "uniform", "split"])
def test_owner_route_keys_ties(gpu, ti):
    """Key-only owner routing (8-byte keys on the links, kad_rt_closest_keys_packed): on tables whose nodes share
    their top 64 bits (tests/tables.py tie_table: ties / ties48, and the unsorted dups tables without short lines)
    the key-only answer cannot order the window, sets the tail word, and serve_owner answers the batch again from
    full targets; on a uniform table the keys answer every query. Every row bit-exact against the oracle
    (infohash.h:131-146: xorCmp reads all 20 bytes)."""
    import tables as TB
    from opendht_amd.sharded import serve_owner

    t = _tie_tables()[ti]
    rng = np.random.default_rng(40 + ti)
    tg = TB.adversarial_targets(t, extra=2000, seed=ti)
    heads = t["ids"][rng.integers(0, t["ids"].shape[0], 300)].copy()
    heads[:, 8:] = rng.integers(0, 256, (300, 12), dtype=np.uint8)  # the tied heads with other tails
    tg = np.ascontiguousarray(np.concatenate([tg, heads]), np.uint8)
    tg = tg[:tg.shape[0] // 8 * 8]
    T = DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=0, sorted=t.get("sorted", False))
    try:
        d = torch.from_numpy(tg).to(gpu)
        R = OwnerRoute(tg.shape[0], 8, 1, 0, gpu)
        assert R.keys and R.record_bytes == 8
        oi = torch.empty((tg.shape[0], 8), dtype=torch.int32, device=gpu)
        oc = torch.empty((tg.shape[0],), dtype=torch.uint8, device=gpu)
        R.step(T, d, oi, oc)
        tailed = R.tailed(combine=False)
        if ti != 4:
            assert tailed, "a top-64 tie (or a table without short lines) must ask for the full targets"
        oi, oc, R = serve_owner(T, d, 8, route=R)
        torch.cuda.synchronize()
        want, wcnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], tg, 8, nthreads=8)
        np.testing.assert_array_equal(oc.cpu().numpy(), wcnt)
        np.testing.assert_array_equal(oi.cpu().numpy().view(np.uint32), want)
    finally:
        T.close()


def test_padding_records_pack(gpu):
    """The send blocks start filled with a padding target of each block's owner: an owner answering
    whole blocks never meets uninitialised records, so the rows of the padding pack (no escape)."""
    from opendht_amd.sharded import pad_blocks

    R = OwnerRoute(3000, 8, 4, 2, gpu)
    v = R.send.view(4, R.cap, 20).cpu().numpy()
    for d in range(4):
        assert (v[d, :, 0] == ((d << 6) | 0x20)).all() and not v[d, :, 1:].any()
    t = torch.empty((2, 8, 20), dtype=torch.uint8, device=gpu)
    pad_blocks(t.view(16, 20), 2, 8, 8)
    assert t[1, :, 0].eq(1).all() and t[1, :, 1].eq(0x80).all()


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def _serve_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    import torch.distributed as dist

    import oracle as O
    from opendht_amd import DeviceTable
    from opendht_amd import synth as S
    from opendht_amd.sharded import OwnerPipeline, OwnerRoute, ShardSpec, build_shard, serve_owner, serve_pipelined

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)  # both ranks on cuda:0: gloo through the host
    ok, why = False, "did not finish"
    try:
        dev = torch.device("cuda:0")
        spec = ShardSpec(n_shards=world, depth=9, mean_per_bucket=6.0, seed=0x5B, good_pct=50, expired_pct=25)
        sh = build_shard(spec, rank)
        T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        targets = _batch(spec, 1500, seed=40 + rank)[:1500]
        tg = torch.from_numpy(targets).to(dev)
        ok, why = True, ""
        for count in (1, 8, 14, 32):
            for cap, packed in ((None, True), (1, True), (None, False)):
                route = OwnerRoute(tg.shape[0], count, world, spec.shard_bits, dev, cap=cap, packed=packed)
                oi, oc, route = serve_owner(T, tg, count, route=route)
                torch.cuda.synchronize()
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, count)
                if not (np.array_equal(oi.cpu().numpy().view(np.uint32), want) and np.array_equal(oc.cpu().numpy(), wcnt)):
                    ok, why = False, f"rank {rank} k={count} cap={cap} packed={packed}"
        # the overlapped pipeline (sharded.OwnerPipeline: gloo all_to_alls on the comm stream), 5 consecutive
        # distinct batches, blocks of one record first (overflow combined over the ranks, grown, all run again)
        batches = [_batch(spec, 1200, seed=100 + 7 * rank + j)[:1200] for j in range(5)]
        for count in (8, 14):
            pipe = OwnerPipeline(1200, count, world, spec.shard_bits, dev, cap=8)
            outs, pipe = serve_pipelined(T, [torch.from_numpy(b).to(dev) for b in batches], count, pipe=pipe)
            torch.cuda.synchronize()
            if pipe.cap <= 8:
                ok, why = False, f"rank {rank} pipelined k={count}: did not grow"
            for j, b in enumerate(batches):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, b, count)
                if not (np.array_equal(outs[j][0].cpu().numpy().view(np.uint32), want) and
                        np.array_equal(outs[j][1].cpu().numpy(), wcnt)):
                    ok, why = False, f"rank {rank} pipelined k={count} batch {j}"
        T.close()
    except Exception as e:  # reported through the queue
        ok, why = False, f"{type(e).__name__}: {e}"
    finally:
        q.put((rank, ok, why))
        dist.destroy_process_group()


def test_serve_owner_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, ok, why = q.get(timeout=240)
        res[r] = (ok, why)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: (True, ""), 1: (True, "")}, res
