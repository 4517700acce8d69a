# Sparse mirror plan: mirror parity tests + the cost breakdown on the bench shard.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_mirror.py tests/test_general_lines.py tests/test_cpp_shim.py tests/test_nc_mirror.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
KAD_DEBUG=1 timeout -k 10 400 python -u tools/bench_mirror.py > $O/mirror.log 2>&1 || exit $?
