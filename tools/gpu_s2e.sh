# NodeCache line kernel: emission by LDS scatter + coalesced rows. Parity (all NodeCache tests) + timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nc_lines32.py tests/test_nc_mirror.py tests/test_config4.py tests/test_status_refresh.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_time.py > $O/nc_time.log 2>&1 || exit $?
