# NodeCache line kernel with wave-cooperative line loads: parity (all NodeCache tests) + ablations + timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_nc_lines32.py tests/test_nc_mirror.py tests/test_config4.py tests/test_status_refresh.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_abl.py > $O/nc_abl.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_time.py > $O/nc_time.log 2>&1 || exit $?
