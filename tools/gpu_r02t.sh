set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02t
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_nc_lines32.py tests/test_gpu_parity.py tests/test_status_refresh.py tests/test_nc_mirror.py tests/test_config4.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_time.py > $O/nc_time.log 2>&1 || exit $?
