"""NodeCache k = 14 on the bench shard, a few launches of the kernel KAD_NC_KERNEL selects (for rocprofv3)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opendht_amd import DeviceTable  # noqa: E402
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

dev = torch.device("cuda:0")
spec = config3_spec()
sh = build_shard(spec, 0)
tg = torch.from_numpy(spec.targets_for(0, 1 << 20, seed=0x0D470002)).to(dev)
T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
for _ in range(5):
    T.nc_closest(tg, 14)
torch.cuda.synchronize()
print("ok")
