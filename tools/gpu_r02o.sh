set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_short_lines.py tests/test_gpu_parity.py tests/test_config4.py tests/test_global_shard.py tests/test_sharded.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench.log 2>&1 || exit $?
