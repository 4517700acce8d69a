"""Per-kernel PMC table of the swarm hop kernels at the end of round 6 (tools/pmc_table_r05.py's formulas): the query
kernel (findClosestNodes by the sorting network, level lines with the index rule) and the merge network with every
peer online (mode swarm0), and the query and 32-entry merge with 10 % offline (mode swarm), from tools/gpu_pmc_r06.sh's
runs.

    python tools/pmc_table_r06c.py gpurun_out/pmc_r06c --out profiles/r06/paths_pmc_c.json
"""
import sys

import pmc_table_r05 as P

P.KERNELS = [
    ("search_query (online)", "swarm0", "search_query_kernel", "config 5 hop, 2M peers, 256k lookups, all online: "
                                                                "the window ranked by the sorting network"),
    ("search_merge_net (online)", "swarm0", "search_merge_net_kernel", "config 5 hop, all online: the merge network, "
                                                                        "next answers loaded ahead"),
    ("search_query (10 % offline)", "swarm", "search_query_kernel", "config 5 hop, 2M peers, 256k lookups, 10 % "
                                                                     "offline"),
    ("search_merge<32> (10 % offline)", "swarm", "search_merge_kernel<false, 32u, false>", "config 5 hop, 10 % offline: "
                                                                                     "insertNode merge, 32-entry lists"),
]

if __name__ == "__main__":
    if "--out" not in sys.argv:
        sys.argv += ["--out", "profiles/r06/paths_pmc_c.json"]
    P.main()
