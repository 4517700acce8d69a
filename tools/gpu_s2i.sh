# Confirmation at HEAD: whole GPU suite, per-path timings (exact rows at k=14/16), default bench, rocprof stats.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/s2i
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/bench_paths.py > $O/paths.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py > $O/bench_default.log 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --no-cpu > $O/prof.log 2>&1 || exit $?
