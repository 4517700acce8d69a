"""HBM traffic per launch of the bench's dominant kernel from rocprofv3 PMC passes (tools/pmc.sh),
corrected as /opt/skills/guides/MI355X_MICROARCH.md ("HBM [CDNA4]") prescribes: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half the bytes of 128-byte reads, so it is
doubled (every read of the kernel is a whole 128-byte line or a 16-byte-per-lane streaming load).
Writes: profiles/traffic_<tag>.json, read by bench.py for roofline.traffic.

    python tools/traffic_json.py gpurun_out/pmc rt_wl_kernel r01
"""
import json
import os
import subprocess
import sys
import time

d, ksub, tag = sys.argv[1], sys.argv[2], sys.argv[3]
count = int(sys.argv[4]) if len(sys.argv) > 4 else 8
args = sys.argv[5] if len(sys.argv) > 5 else "--steps 5 --warmup 2 --no-cpu"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pm = json.loads(subprocess.check_output([sys.executable, os.path.join(root, "tools", "parse_pmc.py"), d, ksub]))
# 128-byte line kernels: x2 (the guide's gfx950 correction, checked by profiles/r02_calib.json); the 64-byte
# short-line kernel: the factor calibrated on the same access pattern with 64-byte lines (profiles/r02_calib.json)
factor, basis = 2.0, "FETCH_SIZE x2 (gfx950 128-B requests tallied at 64 B), KiB -> bytes"
if "rt_ws_kernel" in ksub:
    cal = json.load(open(os.path.join(root, "profiles", "r02_calib.json")))["line64B"]
    factor = cal["read_bytes_per_fetch_byte"]
    basis = (f"FETCH_SIZE x {factor:.4f}: bytes per FETCH_SIZE byte measured on tools/mb_calib.py's 64-byte random "
             "lines + 20-byte targets (profiles/r02_calib.json); KiB -> bytes")
fetch = factor * pm["FETCH_SIZE"] * 1024
write = pm["WRITE_SIZE"] * 1024
out = {"kernel": ksub, "count": count, "hbm_bytes_per_launch": fetch + write, "read_bytes": fetch, "write_bytes": write,
       "raw_kib": {"FETCH_SIZE": pm["FETCH_SIZE"], "WRITE_SIZE": pm["WRITE_SIZE"]},
       "l2_hit_rate": pm["TCC_HIT_sum"] / (pm["TCC_HIT_sum"] + pm["TCC_MISS_sum"]) if "TCC_HIT_sum" in pm else None,
       "correction": basis,
       "source": f"rocprofv3 --pmc passes over bench.py {args} ({d})",
       "date": time.strftime("%Y-%m-%d")}
p = os.path.join(root, "profiles", f"traffic_{tag}.json")
json.dump(out, open(p, "w"), indent=1)
print(json.dumps(out, indent=1))
