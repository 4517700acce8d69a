# Round 6: the whole GPU suite, the default bench line and smoke() at HEAD.
# Usage (on the GPU box): bash tools/gpu_r06_full.sh [tag]; output under gpurun_out/<tag>/.
set -o pipefail
T=${1:-r06full}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done > $O/done.txt
