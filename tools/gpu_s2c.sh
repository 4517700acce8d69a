# NodeCache radix experiment + default bench with the host-buffer pass.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2c
mkdir -p $O
timeout -k 10 400 python -u tools/nc_radix.py > $O/nc_radix.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 50 > $O/bench.log 2>&1 || exit $?
