"""Regenerate tests/golden/config1.npz: BASELINE config 1 (10k-node synthetic routing table,
1k targets) in shapes S (reference split policy) and U(10), with the expected outputs of
RoutingTable::findClosestNodes for k = 8/16/32 and NodeCache::getCachedNodes for k = 8/14/32.

Expected outputs come from the CPU oracle (oracle/kad_oracle.cpp, structure-faithful
restatement, cross-checked against the closed-form one). The OpenDHT reference itself cannot
be built in this image (DESIGN.md "Oracle"), so these vectors are "parity unpinned": they pin
the GPU engine to the oracle and guard regressions, not the oracle to the reference.

Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import oracle as O  # noqa: E402
import tables as TB  # noqa: E402
from opendht_amd import synth as S  # noqa: E402


def main():
    out = {}
    targets = S.random_targets(1000)
    for shape, t in (("S", TB.split_config(10_000)), ("U", TB.uniform_config(10_000, 10))):
        out.update({f"{shape}_ids": t["ids"], f"{shape}_status": t["status"], f"{shape}_first": t["first"],
                    f"{shape}_off": t["off"], f"{shape}_targets": targets})
        T = O.FaithfulTable(t["ids"], t["status"], t["first"], t["off"], with_nc=t["sorted"])
        for k in (8, 16, 32):
            idx, cnt = T.rt_closest(targets, k)
            out[f"{shape}_rt_idx_k{k}"], out[f"{shape}_rt_cnt_k{k}"] = idx, cnt
        if t["sorted"]:
            for k in (8, 14, 32):
                idx, cnt = T.nc_closest(targets, k)
                out[f"U_nc_idx_k{k}"], out[f"U_nc_cnt_k{k}"] = idx, cnt
    np.savez_compressed(os.path.join(os.path.dirname(os.path.abspath(__file__)), "config1.npz"), **out)


if __name__ == "__main__":
    main()
