# Count 9..16 uniform lines with the count-14 prefix first and the wave wl32 fallback: parity + per-path timings.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_short_lines.py tests/test_status_refresh.py tests/test_config4.py tests/test_sharded.py tests/test_global_shard.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py > $O/paths.log 2>&1 || exit $?
