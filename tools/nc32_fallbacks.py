"""Which NodeCache count-32 queries the 512-byte lines hand to the wave path, and why (a diagnostic).

  python tools/nc32_fallbacks.py gpu  out.npz   (tools build, GPU: the l32_stats kernel marks them; saves their targets)
  python tools/nc32_fallbacks.py host out.npz   (CPU: the oracle's rows for them and the line's window limits)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
mode, path = sys.argv[1], sys.argv[2]
if mode == "gpu":  # (torch first: its HIP runtime is the one the engine library then binds to; the tools build
    import torch  # noqa: F401                  before anything else loads the library)
    import opendht_amd._lib as _kl

    _kl.use_ablation_build()
from opendht_amd.sharded import build_shard, config3_spec  # noqa: E402

Q, K = 1 << 20, 32
spec = config3_spec()
sh = build_shard(spec, 0)
if mode == "gpu":
    import torch

    from opendht_amd import DeviceTable

    dev = torch.device("cuda:0")
    T = DeviceTable(sh.ids, sh.status, sh.first, sh.off, device=0, index_base=sh.index_base, sorted=True)
    tg = torch.from_numpy(spec.targets_for(0, Q, seed=0x0D470100)).to(dev)
    os.environ["KAD_NC_KERNEL"] = "l32_stats"
    idx, cnt = T.nc_closest(tg, K)
    sel = (cnt == 250).nonzero().flatten()
    np.savez(path, targets=tg[sel].cpu().numpy(), qi=sel.cpu().numpy())
    print(json.dumps({"fallbacks": int(sel.numel()), "share": sel.numel() / Q}))
    T.close()
    sys.exit(0)

import oracle as O  # noqa: E402

d = np.load(path)
tg = d["targets"]
ids = sh.ids
n = ids.shape[0]
hi = ids[:, :8].copy().view(">u8").ravel().astype(np.uint64)
thi = tg[:, :8].copy().view(">u8").ravel().astype(np.uint64)
# the engine's NodeCache radix (choose_radix with 2^23 slots at most)
tb = 1
while (1 << tb) < n and tb < 23:
    tb += 1
mn, mx = int(hi[0]), int(hi[-1])
best = 63
for s in range(63, -1, -1):
    base = (mn >> s) << s
    if ((mx - base) >> s) + 1 <= (1 << tb):
        best = s
    else:
        break
base = (mn >> best) << best
slot = ((thi.astype(object) - base) >> best)
lo_keys = np.array([base + (int(s) << best) for s in slot], dtype=np.uint64)
hi_keys = np.array([base + ((int(s) + 1) << best) for s in slot], dtype=np.uint64)
r0 = np.searchsorted(hi, lo_keys, "left")
r1 = np.searchsorted(hi, hi_keys, "left")
lb = np.searchsorted(hi, thi, "left")
idx, cnt = O.flat_nc_closest(ids, sh.status, tg, K, nthreads=8)
cats = {"clamped_or_wide_slot": 0, "left_run_past_window": 0, "right_run_past_window": 0, "other": 0}
ex = []
for j in range(tg.shape[0]):
    ns = int(r1[j] - r0[j])
    if r0[j] < 56 or r0[j] - 56 + 124 > n or ns > 15:
        cats["clamped_or_wide_slot"] += 1
        continue
    w0 = int(r0[j]) - 56
    row = idx[j][:cnt[j]].astype(np.int64)
    left_used = int(lb[j] - row.min()) if row.size else 0
    right_used = int(row.max() - lb[j] + 1) if row.size else 0
    if left_used > lb[j] - w0:
        cats["left_run_past_window"] += 1
    elif right_used > w0 + 124 - lb[j]:
        cats["right_run_past_window"] += 1
    else:
        # the builder's 24-bit keys for the window (ncl32_build_kernel): a duplicate between neighbours defers the
        # line; a target equal in key24 to a slot node takes the exact path
        wk = [int(x) for x in hi[w0:w0 + 124]]
        P = 64 - (wk[0] ^ wk[-1]).bit_length() if wk[0] != wk[-1] else 64
        Pp = min(P, 64 - best, 40)
        shf = 40 - Pp
        k24 = [(x >> shf) & 0xFFFFFF for x in wk]
        dup = any(k24[e] == k24[e - 1] for e in range(1, 124))
        t24 = (int(thi[j]) >> shf) & 0xFFFFFF
        eq = any(k24[56 + e] == t24 for e in range(ns))
        key = "defer_duplicate_key24" if dup else "target_equals_slot_key24" if eq else "other"
        cats[key] = cats.get(key, 0) + 1
        if key == "other" and len(ex) < 5:
            ex.append({"ns": ns, "p": int(lb[j] - w0), "left_used": left_used, "right_used": right_used, "P": P})
        if dup:
            cats.setdefault("defer_P_hist", {})
            cats["defer_P_hist"][str(P)] = cats["defer_P_hist"].get(str(P), 0) + 1
print(json.dumps({"fallbacks": int(tg.shape[0]), "categories": cats, "examples_other": ex}))
