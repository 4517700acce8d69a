import os, sys
sys.path.insert(0, "/root/repo")
os.environ["KAD_DEBUG"] = "1"
from opendht_amd import DeviceTable
from opendht_amd import synth as S
n = 12_500_000
ids = S.random_ids(n, 0xB5); st = S.random_status(n, 0xB6)
perm, first, off = S.split_table(ids)
T = DeviceTable(ids[perm], st[perm], first, off, device=0)
print(T.info())
