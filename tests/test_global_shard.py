"""North-star multi-GPU variant (opendht_amd/global_shard.py): shards without halo answer their part
of every query's global window; complete rows are scattered and partial rows merged on the device.
The GPU tests simulate the all-gather by concatenating the shards' outputs on one GPU (one process
cannot open RCCL on one device twice); the gloo test runs the gather plumbing with world_size 2.
Bit-exact against the oracle on the whole table."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import oracle as O
from opendht_amd import DeviceTable
from opendht_amd import synth as S
from opendht_amd._lib import check, lib, part_words, ptr, row_words
from opendht_amd.global_shard import Exchange, GlobalShard, build_plain_shard, merge_parts, query_simulated, reach
from opendht_amd.metrics import good_counts, window_radii
from opendht_amd.sharded import ShardSpec

CASES = [  # (n_shards, depth, mean nodes per bucket, good %)
    (4, 10, 6.0, 80),
    (8, 8, 6.0, 30),
    (8, 6, 2.0, 8),     # windows spanning several whole shards: up to 8 parts per query
    (1, 9, 6.0, 80),    # one shard = the whole table
]


def _targets(spec, n, seed):
    """Random targets plus targets in the buckets around every shard edge."""
    rng = np.random.default_rng(seed)
    parts = [S.random_targets(n, seed=seed)]
    B = spec.n_buckets
    per = B // spec.n_shards
    edges = np.unique(np.clip(np.concatenate([[0, B - 1]] + [np.arange(e - 5, e + 5) for e in range(per, B, per)]),
                              0, B - 1))
    for b in edges:
        f = S.bucket_firsts(spec.depth, int(b), int(b) + 1).copy()
        f[0, 8:] = rng.integers(0, 256, 12, dtype=np.uint8)
        # random low bits below the bucket prefix
        pre = int.from_bytes(f[0, :8].tobytes(), "big")
        pre |= int(rng.integers(0, 1 << 62)) >> spec.depth
        f[0, :8] = np.frombuffer(pre.to_bytes(8, "big"), np.uint8)
        parts.append(f)
    return np.ascontiguousarray(np.concatenate(parts), np.uint8)


def _build(spec, device):
    built = [build_plain_shard(spec, s) for s in range(spec.n_shards)]
    gp = np.concatenate([[0], np.cumsum(np.concatenate([b[6] for b in built]))])
    shards = [GlobalShard(ids, st, off, lo, hi, spec.depth, base, gp, device=device)
              for ids, st, off, lo, hi, base, _ in built]
    return shards


def _compact_path(shards, tg, count, gpu):
    """The per-rank-compacted exchange through kad_rt_scatter_rows + kad_rt_merge_parts (the ABI's other
    finish): every shard's rows and parts read out of its send block on the host side."""
    q = tg.shape[0]
    rw, pw = row_words(count), part_words(count)
    rows, parts = [], []
    for sh in shards:
        ex = Exchange(q, count, len(shards), gpu, row_cap=2 * -(-(-(-q // 2048)) // 8) * 2048, part_cap=max(4096, 8 * q),
                      home=False)
        sh.local_block(tg, ex)
        c = ex.counters().cpu().numpy().reshape(-1, 32)[:, 0]
        assert c[9] == 0
        reg = ex.send[:ex.parts_off].view(8, ex.row_cap, rw)
        rows.append(torch.cat([reg[r, :c[r]] for r in range(8)]))
        parts.append(ex.send[ex.parts_off:ex.ctr_off].view(ex.part_cap, pw)[:c[8]])
    out_idx = torch.full((q, count), -1, dtype=torch.int32, device=gpu)
    out_cnt = torch.full((q,), 255, dtype=torch.uint8, device=gpu)
    nr = [r.shape[0] for r in rows]
    maxr = max(nr)
    g_rows = torch.stack([torch.cat([r, r.new_zeros((maxr - r.shape[0], rw))]) for r in rows]).contiguous()
    n_rows = torch.tensor(nr, dtype=torch.int32, device=gpu)
    s = torch.cuda.current_stream(gpu).cuda_stream
    check(lib().kad_rt_scatter_rows(ptr(g_rows), ptr(n_rows), 1, len(shards), maxr, count, ptr(out_idx),
                                    ptr(out_cnt), gpu.index or 0, s), "scatter")
    npart = [p.shape[0] for p in parts]
    if max(npart):
        maxp = max(npart)
        g_parts = torch.stack([torch.cat([p, p.new_zeros((maxp - p.shape[0], pw))]) for p in parts])
        merge_parts(g_parts, npart, count, out_idx, out_cnt, gpu.index or 0)
    return out_idx, out_cnt, sum(npart)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=lambda c: f"N{c[0]}_U{c[1]}_g{c[3]}")
def test_global_shards_simulated_gather(gpu, case):
    """N shards on one GPU: the home-rank exchange (kad_rt_shard_batch_home + kad_rt_home_finish, what rank r
    runs after all_to_all_single: the rows of its home queries), the all-gather exchange (kad_rt_gather_finish,
    what every rank runs after all_gather_into_tensor), both started with capacities too small so that the
    overflow word makes them grow and run again, and the compacted exchange (kad_rt_scatter_rows +
    kad_rt_merge_parts); all bit-exact against the oracle on the whole table."""
    n_shards, depth, mean, good = case
    spec = ShardSpec(n_shards=n_shards, depth=depth, mean_per_bucket=mean, seed=0x6A7 + depth, good_pct=good,
                     expired_pct=(100 - good) // 2)
    gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
    gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    targets = _targets(spec, 3000, seed=depth)
    tg = torch.from_numpy(targets).to(gpu)
    shards = _build(spec, gpu.index or 0)
    grew = False
    try:
        for count in (1, 3, 8, 9, 14, 16, 24, 32):
            want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, count, nthreads=8)
            for home in (True, False):
                for caps in ((None, None), (1, 1)):
                    idx, cnt, ex = query_simulated(shards, tg, count, row_cap=caps[0], part_cap=caps[1], home=home)
                    torch.cuda.synchronize()
                    what = f"{case} k={count} {caps} home={home}"
                    np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{what} counts")
                    np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=what)
                    if caps[0] == 1:
                        grew = grew or ex.row_cap > 1 or ex.part_cap > 1
            idx, cnt, nparts = _compact_path(shards, tg, count, gpu)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"{case} k={count} compacted counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"{case} k={count} compacted")
            if n_shards == 1:  # the single-rank paths: the plain batch, the shard kernel + finish (no host sync)
                for sk in (False, True):
                    _, i2, c2 = shards[0].query(tg, count, single_rank_shard_kernel=sk)
                    torch.cuda.synchronize()
                    np.testing.assert_array_equal(i2.cpu().numpy().view(np.uint32), want)
                    np.testing.assert_array_equal(c2.cpu().numpy(), wcnt)
            if n_shards > 1 and count == 8:
                assert nparts > 0  # the edge targets produced parts
        assert grew  # capacities of 1 overflowed and grew
    finally:
        for sh in shards:
            sh.close()


@pytest.fixture(scope="module")
def table_100M():
    """Config 3's 100M-node U(24) table from the SURVEY §8d recipe (what every rank's shard is cut from)."""
    from opendht_amd.sharded import config3_spec

    spec = config3_spec(1)
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
    assert (lo, hi, base) == (0, spec.n_buckets, 0) and ids.shape[0] == 100_000_000
    return spec, ids, st, off, good


def _random_and_edge_targets(n_shards, depth, q, seed, gpu):
    """q uniform random targets plus, for every shard edge, targets in the 5 buckets either side of it."""
    g = torch.Generator(device=gpu).manual_seed(seed)
    tg = torch.randint(0, 256, (q, 20), dtype=torch.uint8, device=gpu, generator=g)
    edge = ShardSpec(n_shards=n_shards, depth=depth, mean_per_bucket=1.0, seed=1)
    et = _targets(edge, 0, seed=seed)
    return torch.cat([tg, torch.from_numpy(et).to(gpu)]).contiguous()


@pytest.mark.gpu
def test_whole_100M_table_one_gpu(gpu, table_100M):
    """The north-star table whole on one GPU (what GlobalShard.query answers at N = 1): 1M random targets plus
    the targets next to the 8-shard edges, EVERY query bit-exact against the oracle's closed form for k = 8,
    14 and 32, through the plain batch and through the shard kernel + kad_rt_gather_finish
    (single_rank_shard_kernel, what each rank runs at N > 1 minus the collective)."""
    spec, ids, st, off, good = table_100M
    first = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    gp = np.concatenate([[0], np.cumsum(good)])
    tg = _random_and_edge_targets(8, spec.depth, 1 << 20, 0x100, gpu)
    targets = tg.cpu().numpy()
    G = GlobalShard(ids, st, off, 0, spec.n_buckets, spec.depth, 0, gp, device=gpu.index or 0)
    try:
        for k in (8, 14, 32):
            want, wcnt = O.flat_rt_closest(ids, st, first, off, targets, k, nthreads=16)
            for sk in (False, True):
                _, idx, cnt = G.query(tg, k, single_rank_shard_kernel=sk)
                torch.cuda.synchronize()
                np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"k={k} shard_kernel={sk} counts")
                np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"k={k} sk={sk}")
    finally:
        G.close()


@pytest.mark.gpu
def test_north_star_8_shards_100M(gpu, table_100M):
    """BASELINE config 3 as the north star states it: the 100M-node table in 8 halo-free shards (the shards
    bench.py's allgather variant builds at N = 8; all 8 on one GPU here), each answering its part of every
    query's global window into the send block of the query's home rank, for every rank the blocks addressed to
    it concatenated as the RCCL all_to_all delivers them, the device scatter + merge of its home range. EVERY one
    of 1M random targets plus the shard-edge targets bit-exact against the oracle on the whole table, k = 8, 14
    and 32 (routing_table.cpp:89-104: windows that cross shard edges); at k = 8 a rank receives at most 8 MB
    per step (the all-gather layout: every row, ~50 MB)."""
    from opendht_amd.sharded import config3_spec

    spec, ids, st, off, good = table_100M
    first = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
    gp = np.concatenate([[0], np.cumsum(good)])
    s8 = config3_spec(8)
    per = spec.n_buckets // 8
    # shard 5 as rank 5 of an 8-GPU run builds it (its own pass over the recipe) = the slice of the whole table
    i5, st5, off5, lo5, hi5, base5, _ = build_plain_shard(s8, 5)
    assert (lo5, hi5, base5) == (5 * per, 6 * per, int(off[5 * per]))
    np.testing.assert_array_equal(i5, ids[off[lo5]:off[hi5]])
    np.testing.assert_array_equal(st5, st[off[lo5]:off[hi5]])
    np.testing.assert_array_equal(off5, (off[lo5:hi5 + 1] - off[lo5]).astype(np.uint32))
    del i5, st5, off5
    tg = _random_and_edge_targets(8, spec.depth, 1 << 20, 0x800, gpu)
    targets = tg.cpu().numpy()
    shards = []
    try:
        for s in range(8):
            a, e = s * per, (s + 1) * per
            n0, n1 = int(off[a]), int(off[e])
            shards.append(GlobalShard(ids[n0:n1], st[n0:n1], (off[a:e + 1] - n0).astype(np.uint32), a, e, spec.depth,
                                      n0, gp, device=gpu.index or 0))
        for k in (8, 14, 32):
            idx, cnt, ex = query_simulated(shards, tg, k)
            want, wcnt = O.flat_rt_closest(ids, st, first, off, targets, k, nthreads=16)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"k={k} counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"k={k}")
            assert ex.parts_total > 0, "edge targets must produce parts"
            if k == 8:
                assert ex.gathered_bytes <= 8 * 2**20, ex.gathered_bytes
    finally:
        for sh in shards:
            sh.close()


def test_reach_covers_every_touching_bucket():
    """reach() against the brute-force set of buckets whose window touches [lo, hi)."""
    rng = np.random.default_rng(4)
    for trial in range(30):
        B = 256
        good = rng.poisson(rng.choice([0.3, 1.0, 5.0]), B)
        gp = np.concatenate([[0], np.cumsum(good)])
        lo = int(rng.integers(0, B - 1))
        hi = int(rng.integers(lo + 1, B + 1))
        rlo, rhi = reach(gp, lo, hi, 32)
        for count in (1, 8, 32):
            R = window_radii(good, count)
            b = np.arange(B)
            wlo, whi = np.maximum(0, b - 1 - R), np.minimum(B - 1, b + R)
            touch = (whi >= lo) & (wlo < hi)
            assert touch[:rlo].sum() == 0 and touch[rhi:].sum() == 0, (trial, count)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _gather_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), here]
    import torch.distributed as dist

    from opendht_amd.global_shard import allgather_padded, exchange_into, gather_into, global_good_prefix

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 3 + 4 * rank  # ragged row counts
        rows = torch.arange(100 * 6, dtype=torch.int32).reshape(100, 6) + 1000 * rank
        g, counts = allgather_padded(rows, n)
        ok = counts == [3 + 4 * r for r in range(world)] and g.shape == (world, max(counts), 6)
        for r in range(world):
            exp = torch.arange(100 * 6, dtype=torch.int32).reshape(100, 6)[:counts[r]] + 1000 * r
            ok = ok and torch.equal(g[r, :counts[r]], exp)
        recv = torch.full((world * 7,), -1, dtype=torch.int32)
        gather_into(recv, torch.arange(7, dtype=torch.int32) + 100 * rank)
        ok = ok and torch.equal(recv, torch.cat([torch.arange(7, dtype=torch.int32) + 100 * r for r in range(world)]))
        # the home exchange's collective: block d of every rank's send buffer lands in rank d's recv, in rank order
        send = torch.arange(world * 5, dtype=torch.int32) + 1000 * rank
        recv = torch.full((world * 5,), -1, dtype=torch.int32)
        exchange_into(recv, send)
        ok = ok and torch.equal(recv, torch.cat([torch.arange(5 * rank, 5 * rank + 5, dtype=torch.int32) + 1000 * r
                                                 for r in range(world)]))
        gp = global_good_prefix(np.full(5, rank + 1))
        ok = ok and np.array_equal(gp, np.concatenate([[0], np.cumsum(np.repeat(np.arange(1, world + 1), 5))]))
        q.put((rank, bool(ok)))
    finally:
        dist.destroy_process_group()


def test_allgather_padded_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gather_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: True, 1: True}


def _query_worker(rank, world, port, q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [os.path.dirname(here), os.path.join(os.path.dirname(here), "oracle"), here]
    import torch.distributed as dist

    import oracle as O
    from opendht_amd import synth as S
    from opendht_amd.global_shard import GlobalShard, build_plain_shard, global_good_prefix
    from opendht_amd.sharded import ShardSpec

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    # both ranks share cuda:0 (one GPU box): gloo stages the gathers through the host
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ok, why = False, "did not finish"
    try:
        dev = torch.device("cuda:0")
        spec = ShardSpec(n_shards=world, depth=9, mean_per_bucket=6.0, seed=0x5A, good_pct=40, expired_pct=30)
        ids, st, off, lo, hi, base, good = build_plain_shard(spec, rank)
        gp = global_good_prefix(good)
        G = GlobalShard(ids, st, off, lo, hi, spec.depth, base, gp, device=0)
        targets = _targets(spec, 2000, seed=3)
        tg = torch.from_numpy(targets).to(dev)
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        ok = True
        for count in (1, 8, 14, 32):
            want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, count)
            for home in (True, False):  # home rows (all_to_all) / every row on every rank (all-gather)
                lo, idx, cnt = G.query(tg, count, home=home)
                torch.cuda.synchronize()
                m = idx.shape[0]
                what = f"rank {rank} count {count} home {home} lo {lo} m {m}"
                if not (m < targets.shape[0] if home else m == targets.shape[0]):
                    ok, why = False, f"{what}: wrong row count"
                bad_i = int((idx.cpu().numpy().view(np.uint32) != want[lo:lo + m]).any(1).sum())
                bad_c = int((cnt.cpu().numpy() != wcnt[lo:lo + m]).sum())
                if ok and (bad_i or bad_c):
                    j = int(np.flatnonzero((idx.cpu().numpy().view(np.uint32) != want[lo:lo + m]).any(1))[0])
                    ok, why = False, (f"{what}: {bad_i} rows and {bad_c} counts differ; steps {G.tries}; row {j}: "
                                      f"{idx[j].cpu().numpy().view(np.uint32)[:6].tolist()} cnt {int(cnt[j])} against "
                                      f"{want[lo + j][:6].tolist()} cnt {int(wcnt[lo + j])}")
                    # the same batch again with room for everything from the start (no growth)
                    from opendht_amd.global_shard import Exchange
                    G._ex[(targets.shape[0], count, world, home, world > 1)] = Exchange(targets.shape[0], count, world, dev,
                                                                             row_cap=1 << 20, part_cap=4096, home=home)
                    _, idx2, cnt2 = G.query(tg, count, home=home)
                    torch.cuda.synchronize()
                    bad2 = int((idx2.cpu().numpy().view(np.uint32) != want[lo:lo + m]).any(1).sum())
                    why += f"; with room from the start: {bad2} rows differ, steps {G.tries}"
        # the pipelined step (GlobalShard.run_pipelined: three buffer sets, the all_to_all of batch i+1 on a comm
        # stream under batch i's finish) over 5 consecutive distinct batches, every home row against the oracle
        from opendht_amd.global_shard import Exchange, home_range
        batches = [_targets(spec, 2000, seed=50 + j)[:2000] for j in range(5)]
        nq = batches[0].shape[0]
        hlo, hhi = home_range(nq, world, rank)
        for count in (8, 14):
            like = Exchange(nq, count, world, dev, row_cap=1 << 20, part_cap=4096, collective=True)
            exs = G.pipeline(nq, count, world, like=like)
            outs = [(torch.empty((hhi - hlo, count), dtype=torch.int32, device=dev),
                     torch.empty((hhi - hlo,), dtype=torch.uint8, device=dev)) for _ in batches]
            G.run_pipelined([torch.from_numpy(b).to(dev) for b in batches], exs, outs, rank=rank)
            torch.cuda.synchronize()
            if any(e.overflowed() for e in exs) and ok:
                ok, why = False, f"rank {rank} pipelined count {count}: overflow"
            for j, b in enumerate(batches):
                want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, b, count)
                if ok and not (np.array_equal(outs[j][0].cpu().numpy().view(np.uint32), want[hlo:hhi]) and
                               np.array_equal(outs[j][1].cpu().numpy(), wcnt[hlo:hhi])):
                    ok, why = False, f"rank {rank} pipelined count {count} batch {j}: rows differ"
        G.close()
        if ok:
            why = ""
    except Exception as e:  # reported through the queue
        ok, why = False, f"rank {rank}: {type(e).__name__}: {e}"
    finally:
        q.put((rank, (bool(ok), why)))
        dist.destroy_process_group()


@pytest.mark.gpu
def test_global_shard_query_world2_gloo_gpu(gpu):
    """The whole query() protocol with two ranks (gloo, both on cuda:0): kernels, the home exchange (each rank
    gets its home queries' rows) and the all-gather (every rank gets every row), scatter, merge."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_query_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: (True, ""), 1: (True, "")}, res
