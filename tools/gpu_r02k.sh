set -o pipefail
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_short_lines.py tests/test_gpu_parity.py tests/test_status_refresh.py > $O/pytest_ws.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-allgather > $O/bench.log 2>&1 || exit $?
KAD_RT_KERNEL=wl timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --no-allgather --no-extras > $O/bench_wl.log 2>&1 || exit $?
