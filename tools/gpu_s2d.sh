# Slot lines for counts 9..16: general-line parity + the shapes timing.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2d
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_general_lines.py tests/test_status_refresh.py tests/test_mirror.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
KAD_DEBUG=1 timeout -k 10 300 python -u tools/bench_shapes.py 12500000 > $O/shapes.log 2>&1 || exit $?
