# Whole 100M-node table on one GPU: every one of 1M queries against the oracle.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s3b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_global_shard.py -m gpu -k whole_100M --durations=3 > $O/pytest.log 2>&1 || exit $?
