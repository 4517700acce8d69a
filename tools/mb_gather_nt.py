"""The random-line ceiling with the engine's stream policy (round 3): tools/mb_line.hip's k_lane<NX> (plain target
reads and row writes) against k_lane_nt<NX> (non-temporal ones, as the engine's kernels now issue them), 64-byte lines
in a 128 MB table and 128-byte lines in a 256 MB table (the bench shard's short and 128-byte line sets), rotated
batches and cold, interleaved twice (the median). Writes profiles/r03_mb_gather_nt.json ("all" = the non-temporal
rows, what bench.py's roofline.random_line_ceiling now reads; "plain" = the round-2 form).

    python tools/mb_gather_nt.py
"""
import json
import os
import sys

sys.argv = sys.argv[:1]
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import mb_gather as G  # noqa: E402  (builds libmbline.so, allocates the batches; its own sweep runs at import)

import torch  # noqa: E402

ROOT = os.path.dirname(HERE)


def main():
    out = {"all": {}, "plain": {}}
    for mb, nx in ((128, 4), (256, 8)):
        tab = torch.randint(0, 1 << 30, ((mb << 20) // 4,), dtype=torch.int32, device=G.dev)
        for cold in (False, True):
            key = f"{mb}MB_{16 * nx}B{'_cold' if cold else ''}"
            t = {"nt": [], "plain": []}
            for _ in range(2):
                for pol, coop in (("plain", 0), ("nt", 2)):
                    t[pol].append(G.run(tab, mb << 20, nx, 32 if not cold else 9, cold, coop))
            for pol, dst in (("nt", "all"), ("plain", "plain")):
                us = sorted(t[pol])[len(t[pol]) // 2]
                out[dst][key] = {"us_per_1M": round(us, 2), "G_lines_s": round(G.n / us / 1e3, 2),
                                 "runs_us": [round(x, 2) for x in t[pol]]}
            print(json.dumps({key: {"nt": out["all"][key], "plain": out["plain"][key]}}), flush=True)
        del tab
    out["what"] = ("one random 16*NX-byte line per query + a 20-byte target read + a 32-byte row write, 1M queries per "
                   "launch, 16 rotated batches (cold: after a 1 GiB read); all = non-temporal target reads and row "
                   "writes (the engine's policy since round 3), plain = plain ones")
    p = os.path.join(ROOT, "profiles", "r03_mb_gather_nt.json")
    json.dump(out, open(p, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
