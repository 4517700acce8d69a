"""How far the NodeCache walk for count 32 (node_cache.cpp:36-66: the greedy merge by XOR distance of the runs left
and right of lower_bound, expired nodes skipped) reaches on each side: 2M uniform 63-bit keys, 10 % expired, 20k
uniform targets. Decides whether a 256-byte line (60 slots, 28 left of the slot) could answer count 32: it cannot,
a third of the walks leave it. CPU only.

    python tools/nc32_walk_extent.py [count]
"""
import sys

import numpy as np

K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
rng=np.random.default_rng(1)
n=2_000_000
keys=np.sort(rng.integers(0,2**63,size=n,dtype=np.int64))
exp=rng.random(n)<0.10
Q=20000
ts=rng.integers(0,2**63,size=Q,dtype=np.int64)
lbs=np.searchsorted(keys,ts)
L=[];R=[]
for t,lb in zip(ts,lbs):
    l=lb-1; r=lb; kept=0; sl=0; sr=0
    while kept<K:
        dl = (int(keys[l])^int(t)) if l>=0 else None
        dr = (int(keys[r])^int(t)) if r<n else None
        if dr is None or (dl is not None and dl<dr):
            kept += not exp[l]; l-=1; sl+=1
        else:
            kept += not exp[r]; r+=1; sr+=1
    L.append(sl); R.append(sr)
L=np.array(L); R=np.array(R)
print('left mean %.1f p99 %d max %d; right mean %.1f p99 %d max %d'%(L.mean(),np.percentile(L,99),L.max(),R.mean(),np.percentile(R,99),R.max()))
for lim in ((10, 12, 14, 16, 20, 24) if K <= 16 else (24, 28, 32, 40)):
    print(lim, 'P(left>%d)=%.4f'%(lim,(L>lim).mean()), 'P(right>%d)=%.4f'%(lim,(R>lim).mean()))
print('P(left>28 or right>28)=%.4f'%((L>28)|(R>28)).mean(), 'P(left>28 or right>30)=%.4f'%((L>28)|(R>30)).mean())
