"""Per-kernel roofline evidence for every path kernel from the PMC passes of tools/paths_pmc.py:
HBM bytes per launch (FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE, KiB -> bytes), those bytes
over the kernel's launch time (tools/bench_paths.py timings), VALU busy (SQ_ACTIVE_INST_VALU x 4 over
1024 SIMDs x GRBM_GUI_ACTIVE / 8 cycles, the formula DESIGN.md §5 uses for the headline kernel) and
where the waves' cycles go (WAIT_ANY parked on loads, WAIT_INST_ANY issue stalls, ACTIVE_INST_ANY).

    python tools/paths_roofline.py gpurun_out/pmc_paths gpurun_out/paths.log profiles/history/r01_v11/paths_roofline.json
"""
import json
import re
import subprocess
import sys
import os

pmc_dir, paths_log, out = sys.argv[1], sys.argv[2], sys.argv[3]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
txt = open(paths_log).read()
blocks = re.findall(r"\{[^{}]*\}", txt, re.S)
times = json.loads(blocks[-1]) if blocks else {}
KERNELS = [  # (kernel-name substring, path, paths.log timing key)
    ("rt_wl_kernel<0>", "RoutingTable k=8 (window line)", "rt_k8_us"),
    ("rt_wl16_kernel", "RoutingTable k=16 (one line)", "rt_k16_us"),
    ("rt_wl32_kernel", "RoutingTable k=32 (two lines)", "rt_k32_us"),
    ("rt_closest_kernel<32>", "RoutingTable k=32 (lane kernel, KAD_RT_KERNEL=lane)", "rt_k32_lane_us"),
    ("nc_line_kernel", "NodeCache k=14 (line)", "nc_k14_us"),
    ("nc_multi_kernel<2>", "NodeCache k=14 (wave per query, KAD_NC_KERNEL=multi2)", "nc_k14_multi2_us"),
    ("rt_dual_wl_kernel", "dual family k=8", "dual_k8_us"),
    ("buffer_nodes_kernel", "bufferNodes v4 (k=8 rows)", "buffer_nodes_v4_us"),
]
res = {"source": f"rocprofv3 --pmc passes over tools/paths_pmc.py ({pmc_dir}); times from {paths_log}",
       "hbm_peak_GB_s": 8000.0, "kernels": {}}
for ks, path, tkey in KERNELS:
    pm = json.loads(subprocess.check_output([sys.executable, os.path.join(root, "tools", "parse_pmc.py"), pmc_dir, ks]))
    if "FETCH_SIZE" not in pm:
        continue
    rd, wr = 2 * pm["FETCH_SIZE"] * 1024, pm.get("WRITE_SIZE", 0.0) * 1024
    t_us = times.get(tkey)
    e = {"path": path, "launch_us": t_us, "hbm_read_bytes": rd, "hbm_write_bytes": wr,
         "hbm_GB_s": (rd + wr) / (t_us * 1e-6) / 1e9 if t_us else None}
    if e["hbm_GB_s"]:
        e["hbm_frac_of_peak"] = e["hbm_GB_s"] / 8000.0
    if "SQ_ACTIVE_INST_VALU" in pm and "GRBM_GUI_ACTIVE" in pm:
        e["valu_busy"] = pm["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * pm["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAVE_CYCLES" in pm and "SQ_WAIT_ANY" in pm:
        wc = pm["SQ_WAVE_CYCLES"]
        e["wave_cycles"] = {"parked_on_loads": pm["SQ_WAIT_ANY"] / wc,
                            "issue_stalled": pm.get("SQ_WAIT_INST_ANY", 0) / wc,
                            "issuing": pm.get("SQ_ACTIVE_INST_ANY", 0) / wc}
    if "SQ_INSTS_VALU" in pm and "SQ_WAVES" in pm:
        e["valu_insts_per_wave"] = pm["SQ_INSTS_VALU"] / pm["SQ_WAVES"]
    res["kernels"][ks] = e
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
