"""Config 5 measurement (BASELINE.json configs[4]): a simulated 10M-peer swarm (shape-K tables on the
GPU) and a batch of iterative lookups run to convergence, hop by hop. Prints one JSON object:
table build time, lookups/s over the whole convergence, hops histogram, per-hop time, and the
per-hop findClosestNodes rate. Model: opendht_amd/csrc/kad_swarm.hip (build-defined, parity per hop
in tests/test_swarm.py)."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if os.environ.get("KADGPU_LIB"):  # (an A/B against another engine build, e.g. tools/gpu_swarm_ab.sh)
    from opendht_amd import _lib  # noqa: E402

    _lib.use_library(os.environ["KADGPU_LIB"])
from opendht_amd import synth as S  # noqa: E402
from opendht_amd.swarm import Swarm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--peers", type=int, default=10_000_000)
    ap.add_argument("--lookups", type=int, default=1 << 20)
    ap.add_argument("--offline", type=int, nargs="*", default=[0, 1000],
                    help="peers offline per 10,000 (one run per value)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.perf_counter()
    ids, _ = S.sort_ids(S.random_ids(args.peers, 0x0D470500))
    t_ids = time.perf_counter() - t0
    t0 = time.perf_counter()
    W = Swarm(ids, device=0)
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    rng = np.random.default_rng(9)
    src = torch.from_numpy(rng.integers(0, args.peers, args.lookups).astype(np.int32)).to(dev)
    tg = torch.from_numpy(S.random_targets(args.lookups, seed=0x0D470501)).to(dev)
    # warm-up at the batch size: the timed runs take their search state from the swarm's pool (kad_search_destroy
    # returns it), as a serving loop does after its first batch; the first run, allocations included, is cold_ms
    t0 = time.perf_counter()
    X = W.search(src, tg)
    X.run()
    X.close()
    torch.cuda.synchronize()
    cold_ms = (time.perf_counter() - t0) * 1e3
    for off in args.offline:
        t0 = time.perf_counter()
        X = W.search(src, tg, off)
        hop_ms, active = [], []
        for _ in range(64):
            h0 = time.perf_counter()
            a = X.hop()
            hop_ms.append((time.perf_counter() - h0) * 1e3)
            active.append(a)
            if a == 0:
                break
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        lst, q, bad, n, hops, done, ovf = X.get(full=True)
        queries = int(hops.sum()) * 4 + args.lookups  # findClosestNodes answers (upper bound: <= 4 per hop)
        print(json.dumps({
            "config": f"config5: {args.peers} peers (shape-K tables in HBM), {args.lookups} lookups, alpha 4, "
                      f"list 14, {off / 100:g} % of the peers offline",
            "ids_s": round(t_ids, 2), "table_build_s": round(t_build, 2),
            "table_gb": round(W.device_bytes() / 1e9, 2),
            "lookups_per_s": args.lookups / t_all, "convergence_ms": t_all * 1e3, "cold_ms": cold_ms,
            "rounds": len(hop_ms),
            "hop_ms": [round(x, 3) for x in hop_ms], "active_after_hop": active,
            "hops_hist": np.bincount(hops).tolist(), "mean_hops": float(hops.mean()),
            "done_hist (running, synced, stalled, expired)": np.bincount(done, minlength=4).tolist(),
            "bad_nodes_in_lists_mean": float(bad.sum(axis=1).mean()), "list_overflows": ovf,
            "peer_queries_per_s_upper": queries / t_all,
        }), flush=True)
        X.close()
    W.close()


if __name__ == "__main__":
    main()
