"""Runs tools/microbench.hip patterns on cuda:0 and prints achieved GB/s (calibration, not product)."""
import ctypes as C
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmb.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    os.path.join(HERE, "microbench.hip"), "-o", SO], check=True)
L = C.CDLL(SO)
dev = torch.device("cuda:0")
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
n = 1 << 20


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3  # us


res = {}
inp = torch.randint(0, 255, (n * 20,), dtype=torch.uint8, device=dev)
out = torch.empty((n * 8,), dtype=torch.int32, device=dev)
us = timeit(lambda: L.mb_stream(C.c_void_p(inp.data_ptr()), C.c_void_p(out.data_ptr()), n, s))
res["stream_20r_32w"] = {"us": us, "GBs": n * 52 / us / 1e3}
for mb in ():
    tab = torch.randint(0, 1 << 30, ((mb << 20) // 4,), dtype=torch.int32, device=dev)
    npieces = (mb << 20) // 64
    o = torch.empty((n,), dtype=torch.int32, device=dev)
    for R in (1, 2, 4):
        for D in (1, 2):
            us = timeit(lambda: L.mb_gather(C.c_void_p(tab.data_ptr()), C.c_uint64(npieces), n, R, D,
                                            C.c_void_p(o.data_ptr()), s))
            res[f"gather_{mb}MB_R{R}_D{D}"] = {"us": us, "GBs": n * R * D * 64 / us / 1e3}
            us = timeit(lambda: L.mb_gather_coop(C.c_void_p(tab.data_ptr()), C.c_uint64(npieces), n, R, D,
                                                 C.c_void_p(o.data_ptr()), s))
            res[f"coop_{mb}MB_R{R}_D{D}"] = {"us": us, "GBs": n * R * D * 64 / us / 1e3}
    del tab
tab = torch.randint(0, 1 << 30, ((256 << 20) // 4,), dtype=torch.int32, device=dev)
o = torch.empty((n,), dtype=torch.int32, device=dev)
for R, NX in ((1, 2), (4, 2), (1, 4), (1, 8), (2, 8), (1, 16)):
    for mb in (128, 256):
        us = timeit(lambda: L.mb_gather_sz(C.c_void_p(tab.data_ptr()), C.c_uint64(mb << 20), n, R, NX,
                                           C.c_void_p(o.data_ptr()), s))
        res[f"sz{16*NX}B_R{R}_{mb}MB"] = {"us": us, "GBs": n * R * NX * 16 / us / 1e3}
print(json.dumps(res, indent=1))
