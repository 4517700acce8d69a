# round 2: incremental status refresh + reference-signature shim on the GPU, then the bench line.
set -o pipefail
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_status_refresh.py tests/test_cpp_shim.py tests/test_mirror.py > $O/pytest_new.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/bench_k20.log 2>&1 || exit $?
