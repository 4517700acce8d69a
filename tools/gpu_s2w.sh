# Mirror suite and mirror costs after moving the host plan into kad_mirror_plan.cpp.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2w
mkdir -p $O
cd $R
timeout -k 10 500 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_mirror.py tests/test_cpp_shim.py -m gpu > $O/pytest_mirror.log 2>&1 || exit $?
KAD_DEBUG=1 timeout -k 10 400 python -u tools/bench_mirror.py > $O/mirror.log 2>&1 || exit $?
