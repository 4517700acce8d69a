"""Diagnostic: where the incrementally maintained count 9..16 slot lines (SL16) of a split-policy table part from a
fresh build. Mirrors tests/test_status_refresh.py::test_incremental_lines_equal_fresh_build[S20000] and prints, per
step, which line sets differ and, for SL16, the differing slots and whether each side's line is a copy of one of
the table's own GL16 lines."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
import tables as TB  # noqa: E402
from opendht_amd import _lib  # noqa: E402
from opendht_amd.table import DeviceTable  # noqa: E402

LINESETS = ("WL", "WS", "WL16", "WL32", "GL", "GL16", "GL32", "SL", "SL16", "NCL", "NCL32", "GCNT", "DIR")


def lines(T, name):
    return T.export_lines(getattr(_lib, f"KAD_LINESET_{name}"))


def main():
    t = TB.split_config(20_000, seed=0x5ED)
    n = t["ids"].shape[0]
    rng = np.random.default_rng(n ^ 0x5EC)
    MIN = 60 * 10**9
    now = 800 * 3600 * 10**9
    time_ns = now - rng.integers(0, 10 * MIN, n)
    reply_ns = now - rng.integers(0, 120 * MIN, n)
    expired = (rng.random(n) < 0.05).astype(np.uint8)

    def status_at(tnow):
        good = (expired == 0) & (reply_ns >= tnow - 120 * MIN) & (time_ns >= tnow - 10 * MIN)
        return (good.astype(np.uint8) | (expired << 1)).astype(np.uint8)

    out = []

    def compare(T, st, what):
        rec = {"step": what, "differ": {}}
        with DeviceTable(t["ids"], st, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True) as F:
            for name in LINESETS:
                a, b = lines(T, name), lines(F, name)
                if a is None or b is None:
                    if (a is None) != (b is None):
                        rec["differ"][name] = "present in one only"
                    continue
                if not np.array_equal(a, b):
                    rec["differ"][name] = int((a != b).sum())
            if "SL16" in rec["differ"]:
                a, b = lines(T, "SL16").reshape(-1, 128), lines(F, "SL16").reshape(-1, 128)
                gT, gF = lines(T, "GL16").reshape(-1, 128), lines(F, "GL16").reshape(-1, 128)
                keyT = {bytes(r): i for i, r in enumerate(gT)}
                keyF = {bytes(r): i for i, r in enumerate(gF)}
                js = np.flatnonzero((a != b).any(1))
                rec["sl16_slots"] = []
                for j in js[:40]:
                    rec["sl16_slots"].append({
                        "slot": int(j),
                        "T_is_gl16_of": keyT.get(bytes(a[j])), "F_is_gl16_of": keyF.get(bytes(b[j])),
                        "T_copy_of_F_gl16": keyF.get(bytes(a[j])),
                        "bytes_differ": np.flatnonzero(a[j] != b[j]).tolist()[:32],
                        "T_words": a[j].view(np.uint32)[:8].tolist(), "F_words": b[j].view(np.uint32)[:8].tolist()})
                rec["sl16_nslots"] = int(js.size)
        out.append(rec)
        print(json.dumps(rec), flush=True)

    st0 = status_at(now)
    with DeviceTable(t["ids"], st0, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True) as T:
        torch.cuda.synchronize()
        compare(T, st0, "built")
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now)
        torch.cuda.synchronize()
        compare(T, status_at(now), "first refresh")
        for k in (1, 2, 5, 9, 30, 3000):
            d = np.unique(np.minimum(time_ns + 10 * MIN, reply_ns + 120 * MIN)[expired == 0])
            d = d[d >= now]
            prev = status_at(now)
            now = int(d[min(d.size - 1, k - 1)]) + 1
            T.refresh_status(now)
            torch.cuda.synchronize()
            print(json.dumps({"k": k, "flipped": int((status_at(now) != prev).sum())}), flush=True)
            compare(T, status_at(now), f"k={k}")


if __name__ == "__main__":
    main()
