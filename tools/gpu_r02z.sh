set -o pipefail
R=$(pwd)
O=$R/gpurun_out/r02z
mkdir -p $O
KAD_DEBUG=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_general_lines.py tests/test_mirror.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || exit $?
KAD_DEBUG=1 timeout -k 10 600 python -u tools/bench_shapes.py 12500000 > $O/shapes.log 2>&1 || exit $?
