"""profiles/r02_calib.json: bytes per FETCH_SIZE unit for random-line gathers of 64 and 128 bytes, from the
tools/mb_calib.py PMC passes (known bytes per launch: 1M x (16 NX + 20) read, 1M x 32 written).

    python tools/calib_json.py gpurun_out/r02n profiles/r02_calib.json
"""
import json
import os
import sys

d, dst = sys.argv[1], sys.argv[2]
n = 1 << 20
out = {"what": "tools/mb_calib.py: per query one random line of a 128 MB table + 20-byte target read + 32-byte row "
               "write, 1M queries per launch, distinct batches", "source": d}
for nx in (4, 8):
    pm = json.load(open(os.path.join(d, f"calib_k_lane<{nx}>.json")))
    reads, writes = n * (16 * nx + 20), n * 32
    out[f"line{16 * nx}B"] = {"known_read_bytes": reads, "FETCH_SIZE_KiB": pm["FETCH_SIZE"],
                              "read_bytes_per_fetch_byte": reads / (pm["FETCH_SIZE"] * 1024),
                              "known_write_bytes": writes, "WRITE_SIZE_KiB": pm["WRITE_SIZE"],
                              "write_bytes_per_write_byte": writes / (pm["WRITE_SIZE"] * 1024)}
out["reading"] = ("FETCH_SIZE counts one 64-byte unit per random line request whether the line is 64 or 128 bytes, "
                  "and half the bytes of the coalesced target stream: x2 (the guide's correction) is right for "
                  "128-byte lines only; 64-byte lines take this file's factor")
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
