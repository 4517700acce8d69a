# Round-4 GPU session: focused tests first (status refresh, service), then the whole GPU suite, then the default
# bench line. Usage (on the GPU box): bash tools/gpu_r04.sh <tag> [quick]; output under gpurun_out/<tag>/.
set -o pipefail
T=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_status_refresh.py tests/test_global_shard.py tests/test_serve.py -x -v --timeout 200 --timeout-method thread > $O/pytest_focus.log 2>&1 || exit $?
if [ "$2" != "quick" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
fi
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
echo done > $O/done.txt
