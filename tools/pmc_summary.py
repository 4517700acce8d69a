"""Per-kernel PMC summary from rocprofv3 --pmc passes (tools/pmc.sh): for every kernel whose name contains
one of the given substrings, the mean per dispatch of each counter, HBM bytes per launch (2 x FETCH_SIZE +
WRITE_SIZE, KiB -> bytes: the gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md), the L2 hit rate,
VALU busy (SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)), the split of wave cycles (parked on
s_waitcnt / issue-stalled / issuing) and VALU instructions per wave; with a timing JSON, HBM GB/s per launch.

    python tools/pmc_summary.py <pmc_dir> <timings.log> <out.json> name=substring[:timing_key] ...
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

pmc_dir, tlog, out = sys.argv[1], sys.argv[2], sys.argv[3]
specs = [a.split("=", 1) for a in sys.argv[4:]]
txt = open(tlog).read() if os.path.exists(tlog) else ""
blocks = re.findall(r"\{[^{}]*\}", txt)
times = json.loads(blocks[-1]) if blocks else {}
rows = []
for f in glob.glob(os.path.join(pmc_dir, "**", "*counter_collection.csv"), recursive=True):
    rows += [dict(r, _f=f) for r in csv.DictReader(open(f))]
res = {"source": f"rocprofv3 --pmc passes ({pmc_dir}); launch times from {tlog}", "kernels": {}}
for name, spec in specs:
    sub, _, tkey = spec.partition(":")
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        if sub in r.get("Kernel_Name", ""):
            per[r["Counter_Name"]][(r["Dispatch_Id"], r["_f"])] += float(r["Counter_Value"])
    pm = {c: sum(v.values()) / len(v) for c, v in per.items() if v}
    if not pm:
        continue
    e = {"kernel_substring": sub, "counters_per_dispatch": pm}
    if "FETCH_SIZE" in pm:
        e["hbm_read_bytes"] = 2 * pm["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in pm:
        e["hbm_write_bytes"] = pm["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in pm:
        e["l2_hit_rate"] = pm["TCC_HIT_sum"] / max(1.0, pm["TCC_HIT_sum"] + pm["TCC_MISS_sum"])
    if "SQ_ACTIVE_INST_VALU" in pm and "GRBM_GUI_ACTIVE" in pm:
        e["valu_busy"] = pm["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * pm["GRBM_GUI_ACTIVE"] / 8)
    if all(k in pm for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
        tot = pm["SQ_WAIT_ANY"] + pm["SQ_WAIT_INST_ANY"] + pm["SQ_ACTIVE_INST_ANY"]
        e["wave_cycles_parked_stalled_issuing"] = [round(pm[k] / tot, 3) for k in
                                                   ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")]
    if "SQ_INSTS_VALU" in pm and "SQ_WAVES" in pm:
        e["valu_instr_per_wave"] = pm["SQ_INSTS_VALU"] / max(1.0, pm["SQ_WAVES"])
    t = times.get(tkey) if tkey else None
    if t and "hbm_read_bytes" in e:
        e["launch_us"] = t
        e["hbm_GB_s"] = (e["hbm_read_bytes"] + e.get("hbm_write_bytes", 0.0)) / (t * 1e-6) / 1e9
    res["kernels"][name] = e
json.dump(res, open(out, "w"), indent=1)
for n, e in res["kernels"].items():
    print(n, {k: (round(v, 3) if isinstance(v, float) else v) for k, v in e.items() if k != "counters_per_dispatch"})
