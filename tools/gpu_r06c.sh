# Round 6: the bench line alone, eager pipelines (host issue time).
set -o pipefail
T=${1:-r06c}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.log 2>&1 || exit $?
echo done > $O/done.txt
