"""FETCH_SIZE / WRITE_SIZE calibration for the short-line access pattern (MI355X_MICROARCH.md: "other access
widths are uncalibrated: calibrate on a known byte count in your own access pattern"). tools/mb_line.hip's
k_lane<NX> reads one random NX*16-byte line of a 128 MB table + a 20-byte target and writes a 32-byte row per
query, 1M queries per launch, a distinct target batch and output per launch: known bytes per launch
  reads  = 1M x (16 NX + 20),  writes = 1M x 32.
Run under tools/pmc.sh (PMC_PROG=tools/mb_calib.py, passes FETCH_SIZE;WRITE_SIZE); tools/calib_json.py turns the
counters into bytes-per-count factors for NX = 4 (64-byte lines) and NX = 8 (128-byte lines)."""
import ctypes as C
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
n, NB = 1 << 20, 8
g = torch.Generator(device=dev)
g.manual_seed(11)
tgs = [torch.randint(0, 256, (n * 20,), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
outs = [torch.empty((n * 8,), dtype=torch.int32, device=dev) for _ in range(NB)]
tab = torch.randint(0, 1 << 30, ((128 << 20) // 4,), dtype=torch.int32, device=dev)
for nx in (4, 8):
    for j in range(NB):
        L.mb_line(C.c_void_p(tab.data_ptr()), C.c_uint64(128 << 20), C.c_void_p(tgs[j].data_ptr()), n, nx, 0, 0,
                  C.c_void_p(outs[j].data_ptr()), s)
    torch.cuda.synchronize()
print("ok", flush=True)
