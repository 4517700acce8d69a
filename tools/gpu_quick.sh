# Quick GPU session: GPU parity tests, both bench modes (no CPU baseline), full-table A/B.
set -o pipefail
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --mode allgather --steps 20 --warmup 3 > $O/bench_ag.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --no-cpu > $O/bench.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_full.py > $O/abfull.log 2>&1 || exit $?
