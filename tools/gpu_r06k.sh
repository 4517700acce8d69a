# Round 6: swarm merge / query memory rework + north-star finish rework: their tests, then kernel-trace profiles of
# tools/bench_swarm.py and tools/ns_finish_probe.py.
set -o pipefail
T=${1:-r06k}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_swarm.py tests/test_global_shard.py tests/test_rccl_world1.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_swarm -o sw -- python3 $R/tools/bench_swarm.py > $O/swarm.json 2> $O/swarm.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_ns -o ns -- python3 $R/tools/ns_finish_probe.py 30 > $O/ns.json 2> $O/ns.err || exit $?
timeout -k 10 200 python3 $R/tools/bench_swarm.py > $O/swarm_noprof.json 2> $O/swarm_noprof.err || exit $?
echo done > $O/done.txt
