"""Diagnostic: the exact query() path of test_global_shard_query_world2_gloo_gpu (two gloo ranks on one GPU),
counts 1, 8, 14, 32, with the exchange wrapped to print the send and receive counters of every step."""
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
    from opendht_amd import global_shard as GS
    from opendht_amd import synth as S
    from opendht_amd.sharded import ShardSpec
    from test_global_shard import _targets

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    orig = GS.exchange_into

    mode = os.environ.get("GLOO_DIAG_MODE", "both")

    def wrapped(recv, send, group=None):
        ex_block = recv.numel() // world
        if mode == "inspect":  # exchange_into's gloo path, logging what the host copy of `send` held
            import ctypes as C
            hip = C.CDLL("libamdhip64.so")
            cur = torch.cuda.current_stream()
            q0 = hip.hipStreamQuery(C.c_void_p(cur.cuda_stream))
            cs = send.cpu()
            ctr_cs = [cs[d * ex_block:(d + 1) * ex_block][-320:].numpy().reshape(10, 32)[:, 0].tolist() for d in range(world)]
            torch.cuda.synchronize()
            cs2 = send.cpu()
            ctr_cs2 = [cs2[d * ex_block:(d + 1) * ex_block][-320:].numpy().reshape(10, 32)[:, 0].tolist() for d in range(world)]
            orig(recv, send, group)
            log.append({"block": ex_block, "stream": cur.cuda_stream, "query_before": q0, "ctr_first_copy": ctr_cs,
                        "ctr_after_sync": ctr_cs2, "same": bool(torch.equal(cs, cs2))})
            return
        if mode in ("before", "both"):
            torch.cuda.synchronize()
        if mode == "stream":  # the current (torch) stream only: the stream the step's kernels were launched on
            torch.cuda.current_stream().synchronize()
        if mode == "null":  # the legacy null stream only
            torch.cuda.Stream(stream_ptr=0).synchronize() if hasattr(torch.cuda, "Stream") else None
        orig(recv, send, group)
        if mode in ("after", "both"):
            torch.cuda.synchronize()
        log.append({"block": ex_block, "stream": torch.cuda.current_stream().cuda_stream})

    GS.exchange_into = wrapped
    rec = {"rank": rank}
    try:
        dev = torch.device("cuda:0")
        spec = ShardSpec(n_shards=world, depth=9, mean_per_bucket=6.0, seed=0x5A, good_pct=40, expired_pct=30)
        ids, st, off, lo_b, hi_b, base, good = GS.build_plain_shard(spec, rank)
        gp = GS.global_good_prefix(good)
        G = GS.GlobalShard(ids, st, off, lo_b, hi_b, spec.depth, base, gp, device=0)
        targets = _targets(spec, 2000, seed=3)
        tg = torch.from_numpy(targets).to(dev)
        gids, gst, goff = spec.bucket_range(0, spec.n_buckets)
        gfirst = S.bucket_firsts(spec.depth, 0, spec.n_buckets)
        for count in (1, 8, 14, 32):
            want, wcnt = O.flat_rt_closest(gids, gst, gfirst, goff, targets, count)
            log.clear()
            lo, idx, cnt = G.query(tg, count, home=True)
            torch.cuda.synchronize()
            m = idx.shape[0]
            bad = int((idx.cpu().numpy().view(np.uint32) != want[lo:lo + m]).any(1).sum())
            rec[f"k{count}"] = {"bad": bad, "steps": G.tries, "log": list(log)}
        G.close()
    except Exception:
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
