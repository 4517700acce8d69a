"""Dependent-load latency on cuda:0 (pointer chase over random permutation tables of several sizes);
calibration for the exact-path kernel, not product code."""
import ctypes as C
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmbline.so")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                os.path.join(HERE, "mb_line.hip"), "-o", SO], check=True)
L = C.CDLL(SO)
dev = torch.device("cuda:0")
s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
out = torch.empty((1 << 16,), dtype=torch.int32, device=dev)
res = {}
for mb in (2, 32, 128, 512, 2048):
    n = (mb << 20) // 4
    perm = torch.randperm(n, device=dev, dtype=torch.int64).to(torch.int32)
    for hops in (64,):
        for blocks in (1, 256):
            L.mb_chase(C.c_void_p(perm.data_ptr()), n, hops, blocks, C.c_void_p(out.data_ptr()), s)
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            L.mb_chase(C.c_void_p(perm.data_ptr()), n, hops, blocks, C.c_void_p(out.data_ptr()), s)
            b.record()
            torch.cuda.synchronize()
            res[f"{mb}MB_blocks{blocks}"] = round(a.elapsed_time(b) * 1e6 / hops, 1)  # ns per hop
    del perm
print(json.dumps({"ns_per_dependent_load": res}))
