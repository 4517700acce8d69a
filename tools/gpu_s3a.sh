# Full-size split-policy parity (12.5M nodes, 1M queries, every query against the oracle).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3a
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_general_lines.py -m gpu -k full_size --durations=5 > $O/pytest.log 2>&1 || exit $?
