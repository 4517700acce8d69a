"""Kernel-trace medians of tools/shard_ab.py runs (tools/gpu_shard_ab.sh <tag> ...): per library and pass, the
rt_shard_kernel durations of the reach0, k8, k16 and k32 cases (launch order: reach0 1 + 60, then 2 + 60 each).

    python tools/shard_ab_table.py gpurun_out/<tag> [--out profiles/.../ab.json]
"""
import argparse
import csv
import glob
import json
import os

import numpy as np


def cases(trace):
    rows = [r for r in csv.DictReader(open(trace)) if "rt_shard_kernel" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = np.array([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows])
    k8 = [i for i, r in enumerate(rows) if "rt_shard_kernel<8" in r["Kernel_Name"]]
    k16 = [i for i, r in enumerate(rows) if "rt_shard_kernel<16" in r["Kernel_Name"]]
    k32 = [i for i, r in enumerate(rows) if "rt_shard_kernel<32" in r["Kernel_Name"]]
    res = {"reach0": float(np.median(d[k8[1:61]])), "k8": float(np.median(d[k8[63:]])),
           "k32": float(np.median(d[k32[2:]]))}
    if k16:
        res["k16"] = float(np.median(d[k16[2:]]))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {}
    for t in sorted(glob.glob(os.path.join(a.dir, "*", "run_kernel_trace.csv"))):
        res[os.path.basename(os.path.dirname(t))] = {k: round(v, 2) for k, v in cases(t).items()}
    for k, v in res.items():
        print(k, v)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
