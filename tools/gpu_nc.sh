set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread -k "nc" > $O/pytest_nc.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py > $O/paths.log 2>&1 || exit $?
