# Everything of one iteration: the service tests and latency (gpu_serve.sh), the full GPU parity suite, the
# default bench line, rocprof of the headline, its PMC traffic passes (gpu_r03.sh), then the NodeCache and
# RoutingTable per-count timings (nc_time.py, rt_time.py).
set -o pipefail
T=${1:-all}
R=${GRAFT_REPO_ROOT:-$(pwd)}
FULL=1 bash tools/gpu_serve.sh $T || exit $?
cd $R
timeout -k 10 300 python -u tools/nc_time.py > gpurun_out/$T/nc_time.json 2> gpurun_out/$T/nc_time.err || exit $?
timeout -k 10 300 python -u tools/rt_time.py > gpurun_out/$T/rt_time.json 2> gpurun_out/$T/rt_time.err || exit $?
