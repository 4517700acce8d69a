# Default bench line (host_buffers with reused result arrays) and the host ABI timing tool.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3f
mkdir -p $O
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/host_abi_time.py > $O/host_abi.log 2>&1 || exit $?
