# Cooperative line loads in rt_wl32_kernel: the count 17..32 parity suites and the timings per count.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2y
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/rt_time.py > $O/rt_time.log 2>&1 || exit $?
