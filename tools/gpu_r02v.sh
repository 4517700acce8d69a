set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02v
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_status_refresh.py tests/test_short_lines.py tests/test_nc_lines32.py tests/test_general_lines.py tests/test_gpu_parity.py tests/test_mirror.py tests/test_nc_mirror.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-allgather > $O/bench.log 2>&1 || exit $?
