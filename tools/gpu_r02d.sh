# round 2: full GPU suite, refresh timings, bench line
set -o pipefail
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/prof_refresh.py > $O/refresh.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench_k20.log 2>&1 || exit $?
