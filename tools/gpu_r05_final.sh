# Round-5 confirmation session: GPU parity suite, default bench line, rocprof kernel stats of the
# headline alone, the headline's PMC traffic passes (FETCH_SIZE, WRITE_SIZE), rocprof of the live refresh loop,
# and smoke() at HEAD.
# Usage (on the GPU box): bash tools/gpu_r05_final.sh [tag]; output under gpurun_out/<tag>/.
set -o pipefail
T=${1:-r05final}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu --no-extras > $O/prof.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_$c -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu --no-extras > $O/pmc_$c.log 2>&1 || exit $?
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_live -o live -- python3 $R/tools/live_diag.py 400 > $O/live_diag_prof.json 2> $O/live_diag_prof.err || exit $?
cd $R
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
echo done > $O/done.txt
