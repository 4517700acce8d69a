# Round 6: key-only routing, native executor, one-wave-per-chain merge: the route / RCCL / global-shard / multirank
# tests, the bench line, and a kernel-trace profile of the native probe.
set -o pipefail
T=${1:-r06g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_owner_route.py tests/test_rccl_world1.py tests/test_global_shard.py tests/test_bench_multirank.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest_sel.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_probe -o probe -- python3 $R/tools/native_pipe_probe.py 20 > $O/probe.json 2> $O/probe.err || exit $?
echo done > $O/done.txt
