# Global-shard suite (plain single-rank batch and the shard kernel path) and the default bench line.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2v
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_global_shard.py -m gpu > $O/pytest_global.log 2>&1 || exit $?
timeout -k 10 500 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
