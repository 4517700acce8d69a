# NodeCache ablations (tools build) + the default bench with the other-count timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2f
mkdir -p $O
timeout -k 10 300 python -u tools/nc_abl.py > $O/nc_abl.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 50 > $O/bench.log 2>&1 || exit $?
