"""Per-kernel PMC table at HEAD, round 6 (tools/pmc_table_r05.py with the round-6 kernel list): the kernels this round
changed or added, from tools/gpu_pmc_r06.sh's runs (modes shard, swarm, route); the unchanged ones (lines, refresh)
keep their round-5 rows (profiles/r05/paths_pmc.json).

    python tools/pmc_table_r06.py gpurun_out/pmc_r06 --out profiles/r06/paths_pmc.json
"""
import sys

import pmc_table_r05 as P

P.KERNELS = [k for k in P.KERNELS if k[1] in ("shard", "swarm")] + [
    ("route_pack (20 B)", "route", "route_pack_kernel<false>", "owner routing: pack 1M 20-byte targets into 8 blocks"),
    ("route_pack (keys)", "route", "route_pack_kernel<true>", "owner routing: pack 1M targets as 8-byte keys into 8 blocks"),
    ("route_unpack", "route", "route_unpack_kernel<", "owner routing: rows back, k=8"),
    ("rt_ws_packed (20 B)", "route", "rt_ws_packed_kernel<false>", "owner routing: the owner's k=8 query from 20-byte "
                                                                   "targets, rows written packed"),
    ("rt_ws_packed (keys)", "route", "rt_ws_packed_kernel<true>", "owner routing: the owner's k=8 query from 8-byte "
                                                                 "keys, rows written packed"),
    ("route_unpack_packed", "route", "route_unpack_packed4_kernel#0", "owner routing: packed rows back, k=8"),
    ("route_unpack_packed_fold", "route", "route_unpack_packed4_kernel#1", "owner routing: packed rows back + the "
                                                                           "counter fold and reset, k=8"),
]

if __name__ == "__main__":
    if "--out" not in sys.argv:
        sys.argv += ["--out", "profiles/r06/paths_pmc.json"]
    P.main()
