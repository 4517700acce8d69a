"""Per-kernel PMC table at HEAD: the counters of tools/gpu_pmc_r05.sh's --pmc passes per kernel
(mean per dispatch), the kernel's duration from the kernel-trace --stats run of the same mode, and what bounds it.

  HBM bytes      2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the gfx950 correction of MI355X_MICROARCH.md; FETCH_SIZE
                 counts Infinity-Cache hits too and one 64-byte unit per random line request)
  VALU busy      SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)
  wave cycles    parked on s_waitcnt (SQ_WAIT_ANY) / stalled issuing (SQ_WAIT_INST_ANY) / issuing (SQ_ACTIVE_INST_ANY)
  bound          "integer" when VALU busy >= 0.75; "memory (request latency)" when VALU busy < 0.5 and most wave
                 cycles wait on memory; "latency (few waves)" for kernels of a few workgroups; else "both"

    python tools/pmc_table_r05.py <pmc dir (gpurun_out/pmc_r05...)> ... --out profiles/r05/paths_pmc.json
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KERNELS = [  # (label, mode, kernel-name substring, what)
    ("rt_ws", "lines", "rt_ws_kernel", "RoutingTable k=8, bench shard (the headline kernel)"),
    ("rt_wl16", "lines", "rt_wl16_kernel", "RoutingTable k=16, bench shard"),
    ("rt_wl32q", "lines", "rt_wl32q_kernel", "RoutingTable k=32, bench shard"),
    ("nc_line", "lines", "nc_line_kernel", "NodeCache k=14, bench shard"),
    ("nc32_line", "lines", "nc32_line_kernel", "NodeCache k=32, bench shard"),
    ("rt_sl", "lines", "rt_sl_kernel", "RoutingTable k=8, split-policy 4M nodes"),
    ("rt_sl16", "lines", "rt_sl16_kernel", "RoutingTable k=14, split-policy 4M nodes"),
    ("rt_gl32q", "lines", "rt_gl32q_kernel", "RoutingTable k=32, split-policy 4M nodes"),
    ("rt_shard<8> reach 0", "shard", "rt_shard_kernel<8,#0", "north-star shard kernel, a batch none of whose targets "
                                                             "rank 0 can reach"),
    ("rt_shard<8> all in reach", "shard", "rt_shard_kernel<8,#1", "north-star shard kernel, every target in reach "
                                                                  "(world 1)"),
    ("rt_shard<8>", "shard", "rt_shard_kernel<8,#2", "north-star shard kernel, rank 0 of 8, replicated batch, k=8"),
    ("rt_shard<32>", "shard", "rt_shard_kernel<32,#0", "north-star shard kernel, rank 0 of 8, k=32"),
    ("gather_scatter_link", "shard", "gather_scatter_link_kernel", "north-star finish over 8 blocks (k=8 and 32)"),
    ("gather_merge", "shard", "gather_merge_kernel", "north-star finish: part merge"),
    ("search_query", "swarm", "search_query_kernel", "config 5 hop: queried peers' windows (2M peers, 256k lookups)"),
    ("search_merge", "swarm", "search_merge_kernel", "config 5 hop: insertNode merge per lookup"),
    ("rf_nodes<true,1>", "refresh", "rf_nodes_kernel<true, 1>", "fused small refresh, 1..100 deadlines"),
    ("route_pack", "route", "route_pack_kernel", "owner routing: pack 1M targets into 8 blocks"),
    ("route_unpack", "route", "route_unpack_kernel<", "owner routing: rows back, k=8"),
    ("rt_ws_packed", "route", "rt_ws_packed_kernel", "owner routing: the owner's k=8 query, rows written packed"),
    ("route_unpack_packed", "route", "route_unpack_packed4_kernel", "owner routing: packed rows back, k=8"),
]


GROUP = 6  # tools/paths_pmc_r05.py runs REPS = 6 launches per case; "name#k" picks the k-th case of that kernel


def _pick(sub):
    name, _, k = sub.partition("#")
    return name, (int(k) if k else None)


def counters(pmc_dirs, mode, sub):
    name, k = _pick(sub)
    per = defaultdict(lambda: defaultdict(float))
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, f"pmc_{mode}", "**", "*counter_collection.csv"), recursive=True):
            rows = [r for r in csv.DictReader(open(f)) if name in r.get("Kernel_Name", "")]
            ids = sorted({int(r["Dispatch_Id"]) for r in rows})
            keep = set(ids[GROUP * k:GROUP * (k + 1)]) if k is not None else set(ids)
            for r in rows:
                if int(r["Dispatch_Id"]) in keep:
                    per[r["Counter_Name"]][(r["Dispatch_Id"], f)] += float(r["Counter_Value"])
    return {c: sum(v.values()) / len(v) for c, v in per.items() if v}


def durations(pmc_dirs, mode, sub):
    name, k = _pick(sub)
    out = []
    for d in pmc_dirs:
        for f in glob.glob(os.path.join(d, f"stats_{mode}", "*kernel_trace.csv")):
            rows = [r for r in csv.DictReader(open(f)) if name in r["Kernel_Name"]]
            rows.sort(key=lambda r: int(r["Start_Timestamp"]))
            if k is not None:
                rows = rows[GROUP * k:GROUP * (k + 1)]
            out += [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out", default="profiles/r05/paths_pmc.json")
    a = ap.parse_args()
    res = {"source": a.dirs, "formulas": __doc__.split("\n\n")[1], "kernels": {}}
    for label, mode, sub, what in KERNELS:
        pm = counters(a.dirs, mode, sub)
        du = durations(a.dirs, mode, sub)
        if not pm:
            continue
        e = {"what": what, "mode": mode, "dispatches_timed": len(du)}
        if du:
            du.sort()
            e["duration_us_median"] = du[len(du) // 2]
            e["duration_us_min_max"] = [du[0], du[-1]]
        if "FETCH_SIZE" in pm and "WRITE_SIZE" in pm:
            e["hbm_read_MB"] = 2 * pm["FETCH_SIZE"] * 1024 / 1e6
            e["hbm_write_MB"] = pm["WRITE_SIZE"] * 1024 / 1e6
            if du:
                e["hbm_GB_s"] = (e["hbm_read_MB"] + e["hbm_write_MB"]) * 1e6 / (e["duration_us_median"] * 1e-6) / 1e9
        if "TCC_HIT_sum" in pm:
            e["l2_hit"] = pm["TCC_HIT_sum"] / max(1.0, pm["TCC_HIT_sum"] + pm["TCC_MISS_sum"])
        if "SQ_ACTIVE_INST_VALU" in pm and "GRBM_GUI_ACTIVE" in pm:
            e["valu_busy"] = pm["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * pm["GRBM_GUI_ACTIVE"] / 8)
        if all(k in pm for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")):
            tot = pm["SQ_WAIT_ANY"] + pm["SQ_WAIT_INST_ANY"] + pm["SQ_ACTIVE_INST_ANY"]
            e["wave_cycles_parked_stalled_issuing"] = [round(pm[k] / tot, 3) for k in
                                                       ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")]
        if "SQ_INSTS_VALU" in pm and "SQ_WAVES" in pm:
            e["waves"] = pm["SQ_WAVES"]
            e["valu_instr_per_wave"] = pm["SQ_INSTS_VALU"] / max(1.0, pm["SQ_WAVES"])
            e["vmem_rd_per_wave"] = pm.get("SQ_INSTS_VMEM_RD", 0.0) / max(1.0, pm["SQ_WAVES"])
        v = e.get("valu_busy")
        w = e.get("wave_cycles_parked_stalled_issuing")
        if e.get("waves", 1e9) < 64 * 16:
            e["bound"] = "latency (a few workgroups: VALU busy is a share of the whole GPU)"
        elif v is not None and v >= 0.75:
            e["bound"] = f"integer ops (VALU busy {v:.2f})"
        elif v is not None and w and v < 0.5 and w[0] + w[1] >= 0.7:
            e["bound"] = f"memory requests (VALU busy {v:.2f}, {w[0] + w[1]:.2f} of wave cycles waiting on memory)"
        elif v is not None:
            e["bound"] = f"both (VALU busy {v:.2f})"
        e["counters_per_dispatch"] = pm
        res["kernels"][label] = e
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(f"| kernel | what | µs | HBM MB rd + wr | GB/s | L2 hit | VALU busy | parked / stalled / issuing | "
          f"VALU instr / wave | bound |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    for k, e in res["kernels"].items():
        w = e.get("wave_cycles_parked_stalled_issuing", [0, 0, 0])
        print(f"| `{k}` | {e['what']} | {e.get('duration_us_median', 0):.1f} | {e.get('hbm_read_MB', 0):.0f} + "
              f"{e.get('hbm_write_MB', 0):.0f} | {e.get('hbm_GB_s', 0):.0f} | {e.get('l2_hit', 0):.2f} | "
              f"{e.get('valu_busy', 0):.2f} | {w[0]:.2f} / {w[1]:.2f} / {w[2]:.2f} | {e.get('valu_instr_per_wave', 0):.0f} "
              f"| {e.get('bound', '')} |")


if __name__ == "__main__":
    main()
