# Round 6: key-only owner routing + native executor: route / RCCL world-1 / multirank tests, then the bench line.
set -o pipefail
T=${1:-r06f}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest tests/test_owner_route.py tests/test_rccl_world1.py tests/test_bench_multirank.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.log 2>&1 || exit $?
echo done > $O/done.txt
