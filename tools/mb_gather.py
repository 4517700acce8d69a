"""Random line-gather rate with ROTATING query batches (calibration, not product).

tools/mb_line.hip's k_lane<NX>: per query one random NX*16-byte line of a table, plus the 20-byte
target read and a 32-byte row write. Unlike mb_line.py, every timed launch reads a DIFFERENT batch
of targets (NB distinct 1M-query batches resident in HBM) and writes a different output buffer, so
nothing but the table itself can stay in the 256 MiB Infinity Cache between launches. Table sizes
below and above the Infinity Cache show whether the gather is served from it or from HBM, and the
line sizes show whether HBM-served random gathers are bound by bytes or by requests.

    python tools/mb_gather.py   -> JSON: us per 1M queries, G lines/s, GB/s of line bytes
"""
import ctypes as C
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmbline.so")
src = os.path.join(HERE, "mb_line.hip")
if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(src):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", src, "-o", SO],
                   check=True)
L = C.CDLL(SO)
dev = torch.device("cuda:0")
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
n = 1 << 20
NB = 16
g = torch.Generator(device=dev)
g.manual_seed(7)
tgs = [torch.randint(0, 256, (n * 20,), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
outs = [torch.empty((n * 8,), dtype=torch.int32, device=dev) for _ in range(NB)]
flush = torch.ones((1 << 30) // 4, dtype=torch.int32, device=dev)


def run(tab, nbytes, nx, reps, cold=False, coop=0):
    def one(j):
        L.mb_line(C.c_void_p(tab.data_ptr()), C.c_uint64(nbytes), C.c_void_p(tgs[j % NB].data_ptr()), n, nx, 0, coop,
                  C.c_void_p(outs[j % NB].data_ptr()), s)
    for j in range(4):
        one(j)
    torch.cuda.synchronize()
    if not cold:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for j in range(reps):
            one(j)
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e3
    ts = []
    for j in range(reps):
        _ = flush.sum()  # a 1 GiB READ evicts the Infinity Cache without leaving dirty lines behind
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        one(j)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    res = {}
    for mb in (128, 256, 512, 1024, 2048, 4096):
        tab = torch.randint(0, 1 << 30, ((mb << 20) // 4,), dtype=torch.int32, device=dev)
        for nx, coop in ((1, 0), (2, 0), (4, 0), (8, 0), (8, 1), (16, 0)):
            for cold in (False, True):
                us = run(tab, mb << 20, nx, 32 if not cold else 9, cold, coop)
                key = f"{mb}MB_{16 * nx}B{'_coop' if coop else ''}{'_cold' if cold else ''}"
                res[key] = {
                    "us_per_1M": round(us, 2), "G_lines_s": round(n / us / 1e3, 2),
                    "line_GB_s": round(n * 16 * nx / us / 1e3, 1),
                    "all_GB_s": round(n * (16 * nx + 20 + 32) / us / 1e3, 1)}
                print(json.dumps({key: res[key]}), flush=True)
        del tab
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
