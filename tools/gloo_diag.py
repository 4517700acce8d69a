"""Diagnostic: the two-rank gloo query of tests/test_global_shard.py::test_global_shard_query_world2_gloo_gpu at
count 32, home exchange. Every rank also builds both shards locally and runs the one-process simulation of the
same step, then prints the counters of its real send / receive blocks beside the simulated ones and the rows that
differ from the oracle, so a wrong row can be placed in the shard kernel, the collective or the finish."""
import json
import os
import socket
import sys

import numpy as np
import torch
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def worker(rank, world, port, out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist

    import oracle as O
    from opendht_amd import synth as S
    from opendht_amd.global_shard import (Exchange, GlobalShard, build_plain_shard, exchange_into,
                                          global_good_prefix, home_range)
    from opendht_amd.sharded import ShardSpec
    from test_global_shard import _targets

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = {"rank": rank}
    try:
        dev = torch.device("cuda:0")
        spec = ShardSpec(n_shards=world, depth=9, mean_per_bucket=6.0, seed=0x5A, good_pct=40, expired_pct=30)
        built = [build_plain_shard(spec, s) for s in range(world)]
        ids, st, off, lo_b, hi_b, base, good = built[rank]
        gp = global_good_prefix(good)
        gp_local = np.concatenate([[0], np.cumsum(np.concatenate([b[6] for b in built]))])
        rec["gp_equal"] = bool(np.array_equal(gp, gp_local))
        G = GlobalShard(ids, st, off, lo_b, hi_b, spec.depth, base, gp, device=0)
        Gs = [GlobalShard(b[0], b[1], b[2], b[3], b[4], spec.depth, b[5], gp_local, device=0) for b in built]
        targets = _targets(spec, 2000, seed=3)
        tg = torch.from_numpy(targets).to(dev)
        q = targets.shape[0]
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        rec["reach_real"] = list(G.reach)
        rec["reach_sim"] = [list(g.reach) for g in Gs]
        for count in (14, 32):
            want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, count)
            lo, hi = home_range(q, world, rank)
            # the real step, by hand
            ex = Exchange(q, count, world, dev)
            out_idx = torch.full((hi - lo, count), -7, dtype=torch.int32, device=dev)
            out_cnt = torch.full((hi - lo,), 77, dtype=torch.uint8, device=dev)
            G.home_block(tg, ex)
            torch.cuda.synchronize()
            send_ctr = ex.send.view(world, ex.block)[:, ex.ctr_off:ex.ctr_off + 320].cpu().numpy().reshape(world, 10, 32)[:, :, 0]
            exchange_into(ex.recv, ex.send)
            torch.cuda.synchronize()
            recv_ctr = ex.recv.view(world, ex.block)[:, ex.ctr_off:ex.ctr_off + 320].cpu().numpy().reshape(world, 10, 32)[:, :, 0]
            s = torch.cuda.current_stream(dev).cuda_stream
            import ctypes as C
            ex.home_finish(rank, out_idx, out_cnt, C.c_void_p(s))
            torch.cuda.synchronize()
            ovf = int(ex.overflow.item())
            got = out_idx.cpu().numpy().view(np.uint32)
            bad = np.flatnonzero((got != want[lo:hi]).any(1) | (out_cnt.cpu().numpy() != wcnt[lo:hi]))
            # the simulated send of every shard with the same caps
            sim_ctr = []
            for g in Gs:
                e2 = Exchange(q, count, world, dev, row_cap=ex.row_cap, part_cap=ex.part_cap)
                g.home_block(tg, e2)
                torch.cuda.synchronize()
                sim_ctr.append(e2.send.view(world, e2.block)[:, e2.ctr_off:e2.ctr_off + 320].cpu().numpy()
                               .reshape(world, 10, 32)[:, :, 0].tolist())
            rec[f"k{count}"] = {
                "caps": [ex.row_cap, ex.part_cap], "block": ex.block, "lo_hi": [lo, hi], "overflow": ovf,
                "send_ctr": send_ctr.tolist(), "recv_ctr": recv_ctr.tolist(), "sim_send_ctr": sim_ctr,
                "bad_rows": int(bad.size), "bad_first": bad[:20].tolist(),
                "bad_blocks": np.unique((bad + lo) // 256).tolist(),
                "first_bad": None if bad.size == 0 else {
                    "got": got[bad[0]][:6].tolist(), "cnt": int(out_cnt[bad[0]]),
                    "want": want[lo + bad[0]][:6].tolist(), "wcnt": int(wcnt[lo + bad[0]])}}
        G.close()
        for g in Gs:
            g.close()
    except Exception as e:
        import traceback
        rec["error"] = traceback.format_exc()
    finally:
        out.put(rec)
        dist.destroy_process_group()


def main():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for _ in procs:
        print(json.dumps(q.get(timeout=240)), flush=True)
    for p in procs:
        p.join(timeout=60)


if __name__ == "__main__":
    main()
