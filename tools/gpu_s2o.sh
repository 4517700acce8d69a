# Dual count-16 kernel with the wl32 wave fallback: config-4 parity, dual tests, per-path timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_config4.py tests/test_gpu_parity.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py > $O/paths.log 2>&1 || exit $?
