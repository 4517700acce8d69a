# Pipelined host-pointer batches: the host-entry parity tests, the C++ shim, and the bench's host_buffers rates.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3d
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_cpp_shim.py tests/test_abi.py -m gpu -k "host or shim or abi" > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
