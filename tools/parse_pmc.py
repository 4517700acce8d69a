"""Summarise rocprofv3 --pmc CSV passes (gpurun_out/pmc/p*/.../*counter_collection.csv) per kernel:
mean counter value per dispatch. Usage: python tools/parse_pmc.py [pmc_dir] [kernel_substring]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
ksub = sys.argv[2] if len(sys.argv) > 2 else "rt_wl_kernel"
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        name = row.get("Kernel_Name", "")
        if ksub not in name:
            continue
        key = (row.get("Dispatch_Id"), f)
        vals[row["Counter_Name"]][key].append(float(row["Counter_Value"]))
out = {}
for cn, per in vals.items():
    sums = [sum(v) for v in per.values()]  # a counter may be reported per XCD/instance
    out[cn] = sum(sums) / len(sums)
print(json.dumps(out, indent=1, sort_keys=True))
