# Host-pointer batch tests and the C++ shim after hardening the pipeline's setup.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_cpp_shim.py tests/test_mirror.py tests/test_status_refresh.py -m gpu > $O/pytest.log 2>&1 || exit $?
