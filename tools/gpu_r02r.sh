set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_short_lines.py tests/test_gpu_parity.py tests/test_status_refresh.py tests/test_config4.py tests/test_global_shard.py tests/test_mirror.py > $O/pytest.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/ws_stats.py > $O/ws_paths.json 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_bench.py --variants ws,ws_abl5,ws_abl3,ws_abl1,wl --rounds 9 --reps 16 > $O/ab.log 2>&1 || exit $?
