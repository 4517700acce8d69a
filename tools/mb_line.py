"""Runs tools/mb_line.hip on cuda:0: random bucket-record gathers per query (calibration, not product).
Prints us per 1M queries and the implied random-line rate for each pattern."""
import ctypes as C
import json
import os
import subprocess

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmbline.so")
if not os.path.exists(SO):
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                    os.path.join(HERE, "mb_line.hip"), "-o", SO], check=True)
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
tg = torch.randint(0, 255, (n * 20,), dtype=torch.uint8, device=dev)
out = torch.empty((n * 8,), dtype=torch.int32, device=dev)
for mb in (128, 272, 512, 1024):
    tab = torch.randint(0, 1 << 30, ((mb << 20) // 4,), dtype=torch.int32, device=dev)
    for nx, coop in ((8, 0),):
        for p2 in (0, 32, 128):
            us = timeit(lambda: L.mb_line(C.c_void_p(tab.data_ptr()), C.c_uint64(mb << 20), C.c_void_p(tg.data_ptr()),
                                          n, nx, p2, coop, C.c_void_p(out.data_ptr()), s))
            lines = n * (1 + p2 / 256)
            res[f"{mb}MB_{16*nx}B{'_coop' if coop else ''}_p2={p2}"] = {
                "us": round(us, 1), "Gq_s": round(n / us / 1e3, 2), "G_pieces_s": round(lines / us / 1e3, 1)}
    del tab
print(json.dumps(res, indent=1))
