"""Where the random 64-byte-line request ceiling sits (round 3): tools/mb_req.hip over a 128 MB table (the bench
shard's short-line footprint), 1M queries per launch, 16 rotated target batches, median of 8 launches (HIP events).
  vec       : one vector-loaded line per query with the target read and row write (the ceiling's form)
  vec_lines : the same lines without the streams (line index from a hash of the query number)
  parts     : the streams alone and in other forms (k_parts<F>: per-lane or coalesced targets and rows,
              non-temporal or plain, with or without the line)
  mix_S     : the first S lanes of every wave fetch their lines through scalar loads, the rest by vector loads
  grid_G    : vec_lines with a grid of G workgroups of 256 (grid-stride): rate against the workgroups in flight
Prints one JSON object per line.

    python tools/mb_req.py
"""
import ctypes
import json
import os
import subprocess
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libmbreq.so")
if not os.path.exists(SO):
    subprocess.check_call(["hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                           os.path.join(HERE, "mb_req.hip"), "-o", SO])
L = ctypes.CDLL(SO)
L.mb_req.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
N, NB, REPS = 1 << 20, 16, 8
g = torch.Generator(device=dev)
g.manual_seed(5)
tgs = [torch.randint(0, 256, (N, 20), dtype=torch.uint8, device=dev, generator=g) for _ in range(NB)]
out = torch.empty(N * 32, dtype=torch.int32, device=dev)
big = torch.randint(0, 1 << 30, ((128 << 20) // 4,), dtype=torch.int32, device=dev, generator=g)
small = big[: (64 << 10) // 4]
st = torch.cuda.current_stream().cuda_stream
k = [0]


def run(tab, nbytes, mode, streams, S=0, blocks=0):
    ts = []
    for _ in range(2):  # warm
        L.mb_req(tab.data_ptr(), nbytes, tgs[k[0] % NB].data_ptr(), N, mode, streams, S, blocks, out.data_ptr(), st)
        k[0] += 1
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        rc = L.mb_req(tab.data_ptr(), nbytes, tgs[k[0] % NB].data_ptr(), N, mode, streams, S, blocks, out.data_ptr(),
                      st)
        b.record()
        torch.cuda.synchronize()
        assert rc == 0, rc
        k[0] += 1
        ts.append(a.elapsed_time(b) * 1e3)
    return round(sorted(ts)[len(ts) // 2], 2)


def emit(name, us):
    print(json.dumps({name: {"us_per_1M": us, "G_lines_s": round(N / us / 1e3, 2)}}), flush=True)


B = 128 << 20
if os.environ.get("MB_REQ32"):  # the count-32 shape: 256-byte lines in a 512 MB table, 128-byte rows
    del big
    big = torch.randint(0, 1 << 30, ((512 << 20) // 4,), dtype=torch.int32, device=dev, generator=g)
    for rep in range(2):
        for f, name in {2: "line256", 4: "rows128", 6: "line256+rows128", 3: "tgt+line256", 7: "tgt+line256+rows128", 8: "rows128Q",
                        10: "line256+rows128Q", 11: "tgt+line256+rows128Q"}.items():
            emit(f"{name}#{rep}", run(big, 512 << 20, 2 + 100 + f, 1))
    sys.exit(0)
PARTS = {1: "tgt", 4: "rows", 5: "tgt+rows", 2: "tgtC", 8: "rowsC", 10: "tgtC+rowsC", 33: "tgt_plain",
         36: "rows_plain", 16: "line", 17: "tgt+line", 20: "line+rows", 21: "tgt+line+rows", 24: "line+rowsC",
         18: "tgtC+line", 26: "tgtC+line+rowsC", 53: "tgt+line+rows_plain"}
for rep in range(2):
    emit(f"vec#{rep}", run(big, B, 0, 1))
    emit(f"vec_lines#{rep}", run(big, B, 0, 0))
    for f, name in PARTS.items():
        emit(f"{name}#{rep}", run(big, B, 2 + f, 1))
for S in (0, 8, 16, 32):
    emit(f"mix_{S}", run(big, B, 1, 1, S))
for G in (64, 128, 256, 1024, 4096):
    emit(f"grid_{G}", run(big, B, 0, 0, 0, G))
