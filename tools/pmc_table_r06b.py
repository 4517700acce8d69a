"""Per-kernel PMC table for the kernels round 6's second session changed (tools/pmc_table_r05.py's formulas): the
count <= 14 NodeCache lane kernel (mode lines) and the swarm hop kernels with every peer online (mode swarm0: the
16-register merge) and with 10 % offline (mode swarm: the 32-entry merge), from tools/gpu_pmc_r06.sh's runs.

    python tools/pmc_table_r06b.py gpurun_out/pmc_r06b --out profiles/r06/paths_pmc_b.json
"""
import sys

import pmc_table_r05 as P

P.KERNELS = [
    ("ncl2_lane", "lines", "ncl2_lane_kernel", "NodeCache k=14, bench shard: one lane per query, its 128-byte line"),
    ("search_query (online)", "swarm0", "search_query_kernel", "config 5 hop, 2M peers, 256k lookups, all online: "
                                                                "queried peers' tables as lines"),
    ("search_merge<16> (online)", "swarm0", "search_merge_kernel<false, 16u>", "config 5 hop, all online: insertNode "
                                                                                "merge, 16-register lists"),
    ("search_query (10 % offline)", "swarm", "search_query_kernel", "config 5 hop, 2M peers, 256k lookups, 10 % "
                                                                     "offline"),
    ("search_merge<32> (10 % offline)", "swarm", "search_merge_kernel<false, 32u>", "config 5 hop, 10 % offline: "
                                                                                     "insertNode merge, 32-entry lists"),
]

if __name__ == "__main__":
    if "--out" not in sys.argv:
        sys.argv += ["--out", "profiles/r06/paths_pmc_b.json"]
    P.main()
