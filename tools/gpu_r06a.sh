# Round 6, first GPU session: the owner-routing / pipeline tests (RCCL world 1, gloo world 2, one-rank pipeline),
# then the default bench line (owner_routed.rccl_world1 and the pipelined objects).
# Usage (on the GPU box): bash tools/gpu_r06a.sh [tag]; output under gpurun_out/<tag>/.
set -o pipefail
T=${1:-r06a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_owner_route.py tests/test_rccl_world1.py tests/test_global_shard.py::test_global_shard_query_world2_gloo_gpu tests/test_bench_multirank.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit $?
echo done > $O/done.txt
