# NodeCache kernel with 32 KB staging per block: NodeCache parity + timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2t
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nc_lines32.py tests/test_nc_mirror.py tests/test_config4.py tests/test_status_refresh.py -x -q --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_time.py > $O/nc_time.log 2>&1 || exit $?
