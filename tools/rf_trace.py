"""Diagnostic: where a small refresh's device time goes. Loads the tools build compiled with -DKAD_RF_TRACE
(make -C opendht_amd/csrc ablations ABL_DEFS=-DKAD_RF_TRACE), whose rf_nodes_kernel prints the device wall clock
(100 MHz) at its phase boundaries: [1] phase 1 done (node statuses, appends), [2] NodeCache ranges, [3] buckets
sorted, [4] masks and good counts, [5] line lists, [6] fused line builds. On the bench shard with live node
times: single refreshes passing 1..64 deadlines, each after a query batch (as in the live loop)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from opendht_amd import _lib  # noqa: E402

_lib.use_ablation_build()
import bench  # noqa: E402
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    spec = config3_spec()
    sh = build_shard(spec, 0)
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    Q = 1 << 20
    tg = bench.device_targets(1, Q, spec.shard_bits, 0, 0x0D470002, dev)[0]
    out = torch.empty((Q, 8), dtype=torch.int32, device=dev)
    cnt = torch.empty((Q,), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    s = C.c_void_p(stream.cuda_stream)
    L = _lib.lib()
    h = T._h
    now = 10**15
    t, r, ex = bench.node_times(sh.status, now)
    T.set_times(t, r, ex)
    T.refresh_status(now, stream=stream.cuda_stream)
    torch.cuda.synchronize()
    MIN = 60 * 10**9
    D = np.unique(np.minimum(t + 10 * MIN, r + 120 * MIN)[ex == 0])
    for rep in range(3):
        for k in (1, 2, 4, 8, 16, 64, 100, 128):
            i0 = int(np.searchsorted(D, now, "right"))
            target = int(D[i0 + k - 1]) + 1
            L.kad_rt_closest_batch(h, C.c_void_p(tg.data_ptr()), Q, 8, C.c_void_p(out.data_ptr()),
                                   C.c_void_p(cnt.data_ptr()), s)
            assert L.kad_table_refresh_status(h, C.c_int64(target), s) == 0
            torch.cuda.synchronize()
            print(f"TICK rep={rep} k={k}", flush=True)
            now = target
    T.close()


if __name__ == "__main__":
    main()
