# General-line (split-policy table) iteration: their parity suites, then tools/bench_shapes.py on a 12.5M-node table.
set -o pipefail
T=r03v
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_general_lines.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_gl.log 2>&1 || exit $?
timeout -k 10 600 python -u tools/bench_shapes.py 12500000 > gpurun_out/$T/shapes.log 2>&1 || exit $?
