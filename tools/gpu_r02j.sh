set -o pipefail
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_swarm.py tests/test_sharded.py > $O/pytest_swarm.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_swarm.py > $O/swarm_10M.log 2>&1 || exit $?
