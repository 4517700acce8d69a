# NodeCache kernel iteration: its parity suites, then tools/nc_time.py (timings + identity against the two-pass path).
set -o pipefail
T=${1:-nc}
mkdir -p gpurun_out/$T
timeout -k 10 400 python -u -m pytest tests/test_nc_lines32.py tests/test_gpu_parity.py tests/test_nc_mirror.py -k "nc" -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/pytest_nc.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/nc_time.py > gpurun_out/$T/nc_time.json 2> gpurun_out/$T/nc_time.err || exit $?
