# Dual-family general lines: parity (general lines, config 4) + shapes timing incl. the dual batch.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_general_lines.py tests/test_config4.py -x -v --timeout 400 --timeout-method thread > $O/pytest.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/bench_shapes.py 12500000 > $O/shapes.log 2>&1 || exit $?
