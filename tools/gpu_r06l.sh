# Round 6: fused swarm hop kernel: the swarm tests (fused), then bench_swarm fused and split (KAD_SWARM_SPLIT), the
# fused one under rocprofv3 kernel trace.
set -o pipefail
T=${1:-r06l}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_swarm.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_swarm.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/bench_swarm.py > $O/fused.json 2> $O/fused.err || exit $?
KAD_SWARM_SPLIT=1 timeout -k 10 200 python3 tools/bench_swarm.py > $O/split.json 2> $O/split.err || exit $?
timeout -k 10 200 python3 tools/bench_swarm.py > $O/fused2.json 2> $O/fused2.err || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sw -- python3 $R/tools/bench_swarm.py > $O/fused_prof.json 2> $O/fused_prof.err || exit $?
echo done > $O/done.txt
