# Round-5 GPU session: the new refresh-limit / delayed-block-0 / one-rank RCCL tests first, then the whole GPU
# suite and the default bench line. Usage (on the GPU box): bash tools/gpu_r05.sh [tag] [full]
# output under gpurun_out/<tag>/.
set -o pipefail
T=${1:-r05a}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_refresh_limits.py tests/test_rccl_world1.py tests/test_owner_route.py tests/test_status_refresh.py -x -v \
  --timeout 250 --timeout-method thread > $O/pytest_new.log 2>&1 || exit $?
if [ "$2" = "full" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
  timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
fi
echo done > $O/done.txt
