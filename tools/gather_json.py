"""profiles/r02_mb_gather.json from a tools/mb_gather.py log: the random 128-byte line-gather ceiling
(one random line + a 20-byte target read + a 32-byte row write per query, rotated batches) that
bench.py reports beside its roofline fraction.

    python tools/gather_json.py gpurun_out/r02a/mb_gather.log profiles/r02_mb_gather.json
"""
import json
import sys

src, dst = sys.argv[1], sys.argv[2]
res = {}
for line in open(src):
    line = line.strip()
    if line.startswith('{"') and line.endswith("}}"):
        res.update(json.loads(line))
hot, cold = res["256MB_128B"], res["256MB_128B_cold"]
out = {
    "ceiling": {
        "what": "random 128-byte line gather + 20 B target read + 32 B row write per query, 1M queries per "
                "launch, a distinct target batch and output per launch (tools/mb_gather.py, k_lane<8>)",
        "table_MB": 256, "line_bytes": 128,
        "us_per_1M_rotated": hot["us_per_1M"], "us_per_1M_cold": cold["us_per_1M"],
        "G_lines_s_rotated": hot["G_lines_s"], "G_lines_s_cold": cold["G_lines_s"],
        "cold": "each launch after a 1 GiB read that empties the Infinity Cache",
    },
    "all": res,
    "source": src,
}
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out["ceiling"], indent=1))
