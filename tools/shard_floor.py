"""Where the north-star shard kernel's time goes at N = 8: rank 0's shard of config 3's 100M-node
table, kad_rt_shard_batch_home over the replicated 1M-query batch into 8 home blocks, with the shard's reach cut
to 0, 1/64, 1/16 and the whole of its buckets (reach 0 = the floor of reading the batch and locating it). HIP
events around K eager launches; run it under rocprofv3 --kernel-trace for the kernel durations alone."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))


def main():
    import torch

    from bench import device_targets
    from opendht_amd.global_shard import GlobalShard, build_plain_shard, global_good_prefix
    from opendht_amd.sharded import config3_spec

    dev = torch.device("cuda:0")
    spec = config3_spec(1)
    ids, st, off, lo, hi, base, good = build_plain_shard(spec, 0)
    gp = global_good_prefix(good)
    B = off.shape[0] - 1
    h8 = B // 8
    n0 = int(off[h8])
    G0 = GlobalShard(ids[:n0], st[:n0], off[:h8 + 1], 0, h8, spec.depth, 0, gp, device=0)
    del ids, st
    Q, K, NB = 1 << 20, 20, 4
    tgs = device_targets(NB, Q, 0, 0, 0x0D470002, dev)
    full = tuple(G0.reach)
    out = {"shard_buckets": h8, "reach_default": list(full), "by_reach": {}}
    for cnt in (8, 14, 16, 32):
        ex = G0.exchange(Q, cnt, 8)
        for name, r in (("0", (0, 0)), ("1/64", (0, h8 // 64)), ("1/16", (0, h8 // 16)), ("1/8 (default)", full)):
            G0.reach = r
            for j in range(3):
                G0.home_block(tgs[j % NB], ex)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            a.record()
            for j in range(K):
                G0.home_block(tgs[j % NB], ex)
            b.record()
            torch.cuda.synchronize()
            out["by_reach"][f"k{cnt} reach {name}"] = round(a.elapsed_time(b) / K * 1e3, 2)
        G0.reach = full
    G0.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
